"""bench.py — decoded frames/s of the MI355X CTC ext beam search decoder.

Workload (BASELINE.json metric, configs[2] = "cfg3"): per GPU a batch of
B=256 items, T=1500 frames, C=29 classes, beam_width=128, top_paths=3,
merge_repeated=True; float32 logits [T,B,C] ~ N(0,1) from
numpy.random.default_rng(20251015) (rank r>0: seed 20251015+r), already in
HBM when the timed region starts.  One step = one full decode call through the
C ABI -- row normaliser, beam decode, traceback, int64 SparseTensor components
packed on the device and materialised on the host ("logits
already resident on device, output SparseTensor components materialised on
host") -- plus, for N>1, the RCCL gather of every rank's outputs to rank 0.
Weak scaling: the global batch is 256*N.  Extras beside `value`: the same call
with the components left in HBM (`device_outputs`) and with host logits in
(`host_io`, PCIe both ways).

Prints ONE JSON line on rank 0 (see the contract in the task statement), with
a roofline object for the dominant kernel (ctcx_beam_decode, timed with HIP
events on the stream it runs on) and a cpu_baseline object (the oracle's
reference-cost mode on a bounded sample, N=1 only).
"""
import argparse
import json
import multiprocessing as mp
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "ctc-beam-search-op_amd"))

CONFIGS = {
    # name: (B per GPU, T, C, beam_width, top_paths, merge_repeated, blank_index)
    "cfg1": (2, 50, 6, 4, 1, False, 0),
    "cfg2": (32, 1000, 29, 64, 1, False, 0),
    "cfg3": (256, 1500, 29, 128, 3, True, 0),
    "cfg4": (128, 2000, 1000, 64, 1, False, 0),      # 1024 over 8 GPUs
    "cfg5": (512, 3000, 5000, 256, 1, False, 0),
}
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
# Calibration of the CPU baseline (BASELINE.md "Calibration of the CPU
# baseline", tools/cpu_calibrate.py): the oracle's reference-cost mode ("port")
# timed in the build container on SURVEY.md 6's cfg3-shape item (C=29, W=128,
# P=3, T=1500, merge), one cold call per fresh process as cpu_baseline runs it:
# median 156.9 frames/s per core against the compiled reference's 189 measured
# by the survey on the same container type.  The reference-equivalent CPU
# figure is the port's divided by this ratio.
PORT_OVER_REFERENCE = 0.83


HOST_GEN_LIMIT = 4 << 30   # logits above 4 GiB (cfg5: 30.7 GB) are drawn on the device


def make_inputs(cfg, rank, dev):
    """float32 [T,B,C] N(0,1) logits (distribution A) and seq_len = T.  numpy's
    default_rng(20251015 + rank) as BASELINE.md says; past HOST_GEN_LIMIT a
    seeded torch generator on the device instead (cfg5's 30.7 GB would take
    minutes of host time)."""
    import torch
    B, T, C = cfg[0], cfg[1], cfg[2]
    sl = np.full(B, T, dtype=np.int32)
    if T * B * C * 4 > HOST_GEN_LIMIT:
        g = torch.Generator(device=dev)
        g.manual_seed(20251015 + rank)
        return None, torch.randn((T, B, C), generator=g, device=dev, dtype=torch.float32), sl, "torch-device"
    rng = np.random.default_rng(20251015 + rank)
    x = rng.standard_normal((T, B, C), dtype=np.float32)
    return x, torch.as_tensor(x, device=dev), sl, "numpy"


def lib_hash():
    """sha256 of the libctcext.so this run loads (stamps the PMC traffic file)."""
    import hashlib
    from ctcext_amd import _lib
    with open(_lib.LIB_PATH, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()[:16]


def _build_info():
    path = os.path.join(ROOT, "ctc-beam-search-op_amd", "ctcext_amd", "lib", "build_info.json")
    try:
        return json.load(open(path))
    except (OSError, ValueError):
        return None


def cpu_share():
    """CPUs this process may use: the affinity mask, bounded by a cgroup v2
    quota when one is set (the GPU box's nproc shows the whole machine)."""
    n = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = max(1, int(int(q) // int(per)))
    except (OSError, ValueError):
        pass
    return (min(n, quota) if quota else n), {"nproc": os.cpu_count(), "affinity": n, "cgroup_quota": quota}


def algorithmic_bytes(sl, C, P, out, tsize=4):
    """logits read + seq_len + int64 SparseTensor components +
    shapes + log_prob, from the actual output sizes."""
    n = sum(int(np.prod(out.decoded_values[p].shape)) + int(np.prod(out.alignment_values[p].shape))
            for p in range(P))
    B = len(sl)
    return int(np.sum(sl, dtype=np.int64)) * C * tsize + 4 * B + 24 * n + 32 * P + B * P * tsize


def output_digest(out, P):
    """sha256 over one decode call's outputs, in the op's order: per path the
    int64 SparseTensor components (decoded indices / values / shape, then the
    alignment's), then log_probability ([B, P], the input dtype), each as
    little-endian C-order bytes.  The oracle's outputs for the bench inputs
    hash to tests/golden/bench_digests.json (make_bench_digests.py)."""
    import hashlib
    h = hashlib.sha256()

    def feed(a, dt):
        if hasattr(a, "detach"):
            a = a.detach().cpu().numpy()
        h.update(np.ascontiguousarray(np.asarray(a), dtype=np.dtype(dt).newbyteorder("<")).tobytes())
    for p in range(P):
        for field in (out[0], out[1], out[2], out[3], out[4], out[5]):
            feed(field[p], np.int64)
    lp = out[6]
    feed(lp, lp.dtype if isinstance(lp, np.ndarray) else str(lp.dtype).replace("torch.", ""))
    return h.hexdigest()


def expected_digest(config, rank, B, T):
    """The oracle's digest for this rank's bench inputs, or None (no fixture:
    cfg5's device-drawn logits, or a diagnostics override of B / T)."""
    path = os.path.join(ROOT, "tests", "golden", "bench_digests.json")
    if not os.path.exists(path):
        return None
    e = json.load(open(path)).get(config)
    if not e or e.get("batch_per_gpu") != B or e.get("seq_len") != T:
        return None
    return e["digests"].get(str(rank))


def _cpu_worker(args):
    x, sl, W, P, merge, blank = args
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    t0 = time.perf_counter()
    oracle.raw_decode(x, sl, W, P, merge, blank, -1, mode="faithful")
    return time.perf_counter() - t0


def cpu_baseline(cfg, n_workers, t_cap):
    """The oracle in reference-cost mode (per-candidate std::vector alignment
    copies, per-child heap nodes, TopN heap) on `n_workers` items of the
    workload, one item per process -- the reference op is single-threaded
    (kernels.cc:68), so one process per core is its all-cores form."""
    B, T, C, W, P, merge, blank = cfg
    T = min(T, t_cap)
    rng = np.random.default_rng(20251015)
    jobs = []
    for _ in range(n_workers):
        x = rng.standard_normal((T, 1, C), dtype=np.float32)
        jobs.append((x, np.array([T], np.int32), W, P, merge, blank))
    ctx = mp.get_context("spawn")
    t0 = time.perf_counter()
    with ctx.Pool(n_workers) as pool:
        per_item = pool.map(_cpu_worker, jobs)
    wall = time.perf_counter() - t0
    frames = n_workers * T
    return {"value": frames / wall, "unit": "frames/s", "cores": n_workers, "kind": "port",
            "sample": "%d items x T=%d of the workload shape (C=%d, beam_width=%d, top_paths=%d, "
                      "merge_repeated=%s), oracle reference-cost mode, one item per process"
                      % (n_workers, T, C, W, P, merge),
            "per_core_value": T / float(np.mean(per_item)), "wall_s": wall,
            "calibration": {"port_over_reference": PORT_OVER_REFERENCE,
                            "reference_equivalent_value": frames / wall / PORT_OVER_REFERENCE,
                            "source": "BASELINE.md Calibration: port vs the survey's compiled reference, "
                                      "same container type, cfg3-shape item"}}


def strong_scaling(args, cfg, world, rank, dev, dec, gather_to_root, x):
    """The metric's literal case, a FIXED global batch (BASELINE.json: B=256 on
    1/2/4/8 GPUs; kernels.cc:68-90 loops over it on one core).
    N>1: measured -- the global batch (seed 20251015) is split into contiguous
    shards of B/N items, each rank decodes its shard, the components are
    gathered to rank 0; barrier + max over ranks as for `value`.
    N=1: projected -- the same decode call on the first B/N items for N=2,4,8
    (the shard one GPU of an N-GPU job holds), with device outputs; the N-GPU
    rate is B*T / that time (the gather's few MB over xGMI are left out)."""
    import torch
    import torch.distributed as dist
    import ctcext_amd
    from ctcext_amd import _lib
    B, T, C, W, P, merge, blank = cfg

    def shard(lo, nb):
        # items [lo, lo + nb) of the global batch (seed 20251015): at N=1 the
        # resident x is that batch; otherwise drawn as make_inputs draws it
        # (past HOST_GEN_LIMIT on the device), never a second host copy of it
        if world == 1:
            return x[:, lo:lo + nb].contiguous()
        _, xg, _, _ = make_inputs(cfg, 0, dev)
        xs = xg[:, lo:lo + nb].contiguous()
        del xg
        return xs

    def run(xs, nb, outputs, gather):
        slt = torch.full((nb,), T, dtype=torch.int32, device=dev)
        out = ctcext_amd.ctc_ext_beam_search_decoder(xs, slt, W, P, merge_repeated=merge, blank_index=blank,
                                                     blank_label=-1, outputs=outputs,
                                                     flags=_lib.CTCEXT_FLAG_PROFILE)
        if gather:
            got = gather_to_root(out, rank * nb, P)
            if got is not None:
                [[t.cpu() for t in f] if isinstance(f, list) else f.cpu() for f in got]
        return out
    steps = max(2, min(args.steps, 5))
    if world > 1:
        nb = B // world
        xs = shard(rank * nb, nb)
        run(xs, nb, "device", True)
        torch.cuda.synchronize()
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            run(xs, nb, "device", True)
        torch.cuda.synchronize()
        dist.barrier()
        torch.cuda.synchronize()
        el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
        el = float(el.item())
        return {"global_batch": B, "batch_per_gpu": nb, "n_gpus": world, "steps": steps,
                "frames_per_s": B * T * steps / el, "ms_per_step": 1e3 * el / steps,
                "what": "measured: fixed global batch split over the ranks, %s gather to rank 0"
                        % ("RCCL" if dist.get_backend() == "nccl" else dist.get_backend())}
    proj = []
    for n in (1, 2, 4, 8):
        nb = B // n
        if nb == 0:
            continue
        xs = shard(0, nb)
        run(xs, nb, "device", False)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        kms = []
        for _ in range(steps):
            run(xs, nb, "device", False)
            kms.append(dec.last_stats["decode_kernel_ms"])
        torch.cuda.synchronize()
        ms = 1e3 * (time.perf_counter() - t0) / steps
        proj.append({"n_gpus": n, "batch_per_gpu": nb, "ms_per_step": ms, "decode_kernel_ms": float(np.mean(kms)),
                     "projected_frames_per_s": B * T / (ms * 1e-3)})
    for p in proj:
        p["efficiency_vs_linear"] = p["projected_frames_per_s"] / (proj[0]["projected_frames_per_s"] * p["n_gpus"])
    return {"global_batch": B, "what": "projected from one GPU: per-GPU time of the B/N-item shard "
                                      "(device outputs, gather excluded)", "curve": proj}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="cfg3", choices=sorted(CONFIGS))
    ap.add_argument("--cpu-workers", type=int, default=int(os.environ.get("CTCX_CPU_WORKERS", "0")),
                    help="0: the CPU share of this process (affinity mask and cgroup quota)")
    ap.add_argument("--cpu-tcap", type=int, default=0,
                    help="frames per CPU-baseline item (0: the config's T, or 100 / 20 frames for cfg4 / "
                         "cfg5, whose full items need ~48 GB / ~1.4 TB on the reference's CPU path)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-gather", action="store_true")
    ap.add_argument("--no-host-io", action="store_true", help="skip the host-I/O (PCIe-inclusive) extra")
    ap.add_argument("--seq-len", type=int, default=0, help="diagnostics: override T (not a bench line)")
    ap.add_argument("--batch-per-gpu", type=int, default=0, help="diagnostics: override B per GPU (not a bench line)")
    ap.add_argument("--scorer", choices=["base", "bigram"], default="base",
                    help="diagnostics: the bigram beam scorer with a random <= 0 table (not a bench line)")
    ap.add_argument("--record-ring", action="store_true",
                    help="diagnostics: ask for the LDS record ring (only reachable beam records written to HBM; "
                         "the default where the score-table two-wave kernel runs)")
    ap.add_argument("--no-ring", action="store_true",
                    help="diagnostics: every beam record to HBM (no record ring)")
    ap.add_argument("--no-strong", action="store_true",
                    help="skip the strong-scaling extra (N=1: the per-GPU latency at the B=256/N shards; "
                         "N>1: the measured global-B=256 split)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist
    import ctcext_amd
    from ctcext_amd import _lib
    from ctcext_amd.sharded import gather_to_root

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal knobs for a one-GPU box (the driver's runs use neither):
    # CTCX_ONE_DEVICE=1 puts every rank on cuda:0, CTCX_DIST_BACKEND=gloo
    # replaces RCCL (which refuses two ranks on one device)
    if os.environ.get("CTCX_ONE_DEVICE") == "1":
        local = 0
    backend = os.environ.get("CTCX_DIST_BACKEND", "nccl")
    if world > 1:
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    cfg = CONFIGS[args.config]
    if args.seq_len:
        cfg = (cfg[0], args.seq_len) + cfg[2:]
    if args.batch_per_gpu:
        cfg = (args.batch_per_gpu,) + cfg[1:]
    B, T, C, W, P, merge, blank = cfg
    x_np, x, sl_np, gen = make_inputs(cfg, rank, dev)
    sl = torch.as_tensor(sl_np, device=dev)
    torch.cuda.synchronize()

    flags = (_lib.CTCEXT_FLAG_PROFILE | (_lib.CTCEXT_FLAG_RECORD_RING if args.record_ring else 0)
             | (_lib.CTCEXT_FLAG_NO_RING if args.no_ring else 0))
    dec = ctcext_amd.get_decoder(local)
    skw = {}
    if args.scorer == "bigram":   # ctc_beam_scorer.h's hook with a bigram table of log-probabilities
        g = torch.Generator(device=dev).manual_seed(7)
        skw["scorer_table"] = -torch.rand((C + 1, C), generator=g, device=dev, dtype=torch.float32) * 2.0

    def step(outputs="host"):
        # 8(d): device-resident logits in, SparseTensor components on the host
        # out (world > 1: device outputs, gathered over RCCL to rank 0)
        out = ctcext_amd.ctc_ext_beam_search_decoder(x, sl, W, P, merge_repeated=merge,
                                                     blank_index=blank, blank_label=-1, flags=flags,
                                                     outputs=outputs if world == 1 else "device", **skw)
        if world > 1 and not args.no_gather:
            got = gather_to_root(out, rank * B, P)
            if got is not None:   # rank 0: the whole batch's components to the host
                [[t.cpu() for t in f] if isinstance(f, list) else f.cpu() for f in got]
        return out   # this rank's own decode (its algorithmic bytes)

    for _ in range(args.warmup):
        out = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    kms, lit, red, pms, tms = [], 0, 0, [], []
    for _ in range(args.steps):
        out = step()
        st = dec.last_stats
        kms.append(st["decode_kernel_ms"])
        pms.append(st["norm_kernel_ms"])
        tms.append(st["traceback_ms"])
        lit += st["literal_frames"]
        red += int(st.get("helper_redecodes", 0))
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # the parity gate on the timed workload: the last timed step's outputs
    # against the oracle's for these exact inputs (outside the timed region)
    digest = output_digest(out, P)
    # (the ring flags change no output; the bigram scorer does: no fixture)
    want = expected_digest(args.config, rank, B, T) if args.scorer == "base" else None
    match = None if want is None else digest == want
    redecodes = red
    if world > 1:   # every rank's verdict: -1 no fixture, 0 mismatch, 1 match
        m = torch.tensor([-1 if match is None else int(match), redecodes], dtype=torch.int64, device=dev)
        ms_ = [torch.zeros_like(m) for _ in range(world)]
        dist.all_gather(ms_, m)
        verdicts = [int(v[0]) for v in ms_]
        redecodes = sum(int(v[1]) for v in ms_)
        match = None if any(v < 0 for v in verdicts) else all(v == 1 for v in verdicts)
    frames_per_step = int(sl_np.sum()) * world
    value = frames_per_step * args.steps / elapsed
    ms = 1e3 * elapsed / args.steps
    kavg = float(np.mean(kms))
    abytes = algorithmic_bytes(sl_np, C, P, out)
    achieved = abytes / (kavg * 1e-3) / 1e9
    # HBM bytes per launch from this build's PMC passes (tools/pmc_summary.py);
    # a file stamped with another library build is stale and not used
    traffic, traffic_src = None, "no PMC file for this config"
    pmc = os.path.join(ROOT, "profiles", "pmc_%s.json" % args.config)
    if os.path.exists(pmc):
        pj = json.load(open(pmc))
        if pj.get("lib_sha16") == lib_hash() and pj.get("seq_len", T) == T:
            traffic, traffic_src = pj.get("hbm_bytes_per_launch"), os.path.relpath(pmc, ROOT)
        else:
            traffic_src = "stale: %s is of build %s, this is %s" % (os.path.relpath(pmc, ROOT),
                                                                   pj.get("lib_sha16"), lib_hash())
    metric = "decoded frames/sec at B=256, T=1500, C=29, beam_width=128; 1/2/4/8 GPUs"   # BASELINE.json
    if args.config != "cfg3" or args.seq_len or args.batch_per_gpu or args.scorer != "base":   # diagnostics
        metric = "decoded frames/sec at B=%d, T=%d, C=%d, beam_width=%d (%s%s, not the BASELINE metric)" % (
            B * world, T, C, W, args.config, ", bigram scorer" if args.scorer != "base" else "")
    res = {
        "metric": metric,
        "value": value, "unit": "frames/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": ms, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f32",
        "data": "synthetic N(0,1) logits (%s generator)" % gen,
        "config": {"workload": args.config, "global_batch": B * world, "batch_per_gpu": B,
                   "seq_len": T, "num_classes": C, "beam_width": W, "top_paths": P,
                   "merge_repeated": merge, "parallelism": "batch-shard x%d" % world,
                   "gather": world > 1 and not args.no_gather,
                   "backend": ("rccl" if backend == "nccl" else backend) if world > 1 else None},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": traffic_src,
                     "kernel": "ctcx_beam_decode", "kernel_ms": kavg,
                     "algorithmic_bytes_per_launch": abytes,
                     # beam records the decode kernel wrote to HBM (record_bytes each:
                     # 4 in the two-wave kernel; with the LDS record ring only those
                     # the traceback can reach)
                     "record_ring_frames": st["ring_frames"], "records_written": st["records_written"],
                     "record_bytes": st["record_bytes"], "helper_kernel": st["helper"],
                     # the other kernels of the call (HIP events): the row pre-pass
                     # (normaliser; large C also the row facts) and traceback + pack
                     "prepass_ms": float(np.mean(pms)), "traceback_ms": float(np.mean(tms))},
        "literal_frames_per_step": lit / max(args.steps, 1),
        # tests/golden/bench_digests.json: the oracle's outputs for these
        # inputs (null: no fixture for this config, e.g. cfg5's device-drawn logits)
        "outputs_match_oracle": match, "outputs_sha256": digest,
        # a helper-wave timeout re-decodes with the one-wave kernels: never silent
        "helper_redecodes": redecodes,
        "lib_sha16": lib_hash(),
        # __graft_entry__.build()'s record: recompiled or reused, and the sha
        "build_info": _build_info(),
        "what": ("one decode call: device logits in, int64 SparseTensor components materialised on the host"
                 if world == 1 else "one decode call per rank (device outputs) + %s gather to rank 0"
                 % ("RCCL" if backend == "nccl" else backend)),
    }
    if world == 1 and not args.no_host_io:
        # the same call with the components left in HBM (no device->host copy)
        n_dev = max(1, min(args.steps, 3))
        step("device")
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(n_dev):
            step("device")
        torch.cuda.synchronize()
        dv_s = (time.perf_counter() - t1) / n_dev
        res["device_outputs"] = {"frames_per_s": int(sl_np.sum()) / dv_s, "ms_per_step": 1e3 * dv_s,
                                 "steps": n_dev, "what": "device logits in, components left in HBM"}
    if world == 1 and not args.no_host_io and x_np is not None:
        # SURVEY 8(d)'s end-to-end form, never `value`: host logits in (one PCIe
        # upload), SparseTensor components and log-probabilities back as host
        # numpy arrays; timed outside the region above
        ctcext_amd.ctc_ext_beam_search_decoder(x_np, sl_np, W, P, merge_repeated=merge,
                                               blank_index=blank, blank_label=-1)
        n_io = 2
        t1 = time.perf_counter()
        for _ in range(n_io):
            ctcext_amd.ctc_ext_beam_search_decoder(x_np, sl_np, W, P, merge_repeated=merge,
                                                   blank_index=blank, blank_label=-1)
        io_s = (time.perf_counter() - t1) / n_io
        res["host_io"] = {"frames_per_s": int(sl_np.sum()) / io_s, "ms_per_step": 1e3 * io_s,
                          "steps": n_io, "what": "host numpy logits in, host numpy outputs out (PCIe both ways)"}
    if not args.no_strong and not args.seq_len and not args.batch_per_gpu and B % 2 == 0:
        res["strong"] = strong_scaling(args, cfg, world, rank, dev, dec, gather_to_root, x)
    if rank == 0 and world == 1 and not args.no_cpu:
        share, info = cpu_share()
        nw = args.cpu_workers or share
        tcap = args.cpu_tcap or {"cfg4": 100, "cfg5": 20}.get(args.config, T)
        res["cpu_baseline"] = cpu_baseline(cfg, nw, tcap)
        if tcap < T:
            res["cpu_baseline"]["truncated"] = "T=%d of %d (BASELINE.md: full items do not fit host memory)" % (tcap, T)
        res["cpu_baseline"]["gpu_over_cpu"] = value / res["cpu_baseline"]["value"]
        res["cpu_baseline"]["calibration"]["gpu_over_reference_equivalent"] = (
            value / res["cpu_baseline"]["calibration"]["reference_equivalent_value"])
        res["cpu_baseline"]["host_cpus"] = info
    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
