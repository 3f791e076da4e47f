"""Generates tests/golden/bench_digests.json: the CPU oracle's outputs for the
exact inputs bench.py decodes, as sha256 digests (bench.output_digest).

bench.py hashes the outputs of its last timed step and reports
``outputs_match_oracle``; tools/abv.sh withholds the timing of any variant
whose outputs differ.  Inputs are drawn exactly as bench.make_inputs draws them
(numpy default_rng(20251015 + rank), float32 [T, B, C] ~ N(0, 1), seq_len = T)
for ranks 0..7 of cfg2, cfg3 and cfg4; cfg5's logits are drawn on the device
by torch (30.7 GB) and have no fixture.  The oracle (shared mode, the
restatement pinned by the reference's golden vector, test.py:20-100) decodes
the batch in item shards over worker processes; the items are independent
(kernels.cc:68-90) and the SparseTensor packing (kernels.cc:163-257) is done
once over the whole batch.

Run in the build container: python tests/golden/make_bench_digests.py [-j N]
"""
import argparse
import json
import multiprocessing as mp
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import bench  # noqa: E402  (CONFIGS, output_digest: no GPU import at module level)
import oracle  # noqa: E402


def _shard(args):
    x, T, W, P, merge, blank = args
    B = x.shape[1]
    dec, ali, lp, _ = oracle.raw_decode(x, np.full(B, T, np.int32), W, P, merge, blank, -1, mode="shared")
    return dec, ali, lp


def digest_for(cfg_name, rank, pool, per_shard):
    B, T, C, W, P, merge, blank = bench.CONFIGS[cfg_name]
    rng = np.random.default_rng(20251015 + rank)   # bench.make_inputs, numpy branch
    x = rng.standard_normal((T, B, C), dtype=np.float32)
    jobs = [(np.ascontiguousarray(x[:, lo:lo + per_shard]), T, W, P, merge, blank)
            for lo in range(0, B, per_shard)]
    dec, ali, lps = [], [], []
    for d, a, lp in pool.map(_shard, jobs):
        dec += d
        ali += a
        lps.append(lp)
    di, dv, ds = oracle.pack_sparse(dec, B, P)
    ai, av, ash = oracle.pack_sparse(ali, B, P)
    out = (di, dv, ds, ai, av, ash, np.concatenate(lps, axis=0).astype(np.float32))
    return bench.output_digest(out, P), {"decoded": int(sum(len(v) for v in dv)),
                                         "alignment": int(sum(len(v) for v in av))}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("-j", type=int, default=os.cpu_count() or 1)
    ap.add_argument("--configs", default="cfg2,cfg3,cfg4")
    ap.add_argument("--ranks", type=int, default=8)
    args = ap.parse_args()
    path = os.path.join(HERE, "bench_digests.json")
    res = json.load(open(path)) if os.path.exists(path) else {}
    with mp.get_context("spawn").Pool(args.j) as pool:
        for name in args.configs.split(","):
            B, T, C, W, P, merge, blank = bench.CONFIGS[name]
            e = {"batch_per_gpu": B, "seq_len": T, "num_classes": C, "beam_width": W, "top_paths": P,
                 "merge_repeated": merge, "blank_index": blank, "blank_label": -1,
                 "inputs": "numpy default_rng(20251015 + rank).standard_normal((T, B, C), float32), seq_len = T",
                 "oracle_mode": "shared", "digests": {}, "sizes": {}}
            for r in range(args.ranks):
                t0 = time.time()
                d, sz = digest_for(name, r, pool, max(1, B // (4 * args.j)))
                e["digests"][str(r)] = d
                e["sizes"][str(r)] = sz
                print(name, r, d[:16], sz, "%.1fs" % (time.time() - t0), flush=True)
            res[name] = e
            json.dump(res, open(path, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
