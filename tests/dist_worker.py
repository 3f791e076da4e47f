"""One rank of tests/test_gpu_sharded.py::test_two_ranks_hip_decoder_gather,
started by torch.distributed.run (RANK / WORLD_SIZE / MASTER_* from the env).

Each rank decodes its contiguous batch shard with the HIP decoder (through the
C ABI) and the shards are gathered to rank 0 by ctcext_amd.sharded
.gather_to_root; rank 0 saves the gathered SparseTensor components to argv[1].
CTCX_ONE_DEVICE=1 puts every rank on cuda:0 and the collectives on gloo (RCCL
refuses two ranks on one device); without it each rank takes cuda:LOCAL_RANK
and RCCL.
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ctc-beam-search-op_amd"))


def workload():
    rng = np.random.default_rng(2024)
    T, B, C, W, P = 80, 7, 29, 16, 2
    x = rng.standard_normal((T, B, C)).astype(np.float32)
    sl = rng.integers(1, T + 1, size=B).astype(np.int32)
    return x, sl, W, P, dict(merge_repeated=True, blank_index=0, blank_label=-1)


def main():
    import torch
    import torch.distributed as dist

    import ctcext_amd
    from ctcext_amd.sharded import gather_to_root, shard_bounds

    rank = int(os.environ["RANK"])
    world = int(os.environ["WORLD_SIZE"])
    one = os.environ.get("CTCX_ONE_DEVICE") == "1"
    local = 0 if one else int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if one:
        dist.init_process_group("gloo")
    else:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    x, sl, W, P, kw = workload()
    lo, hi = shard_bounds(x.shape[1], rank, world)
    dev = torch.device("cuda", local)
    out = ctcext_amd.ctc_ext_beam_search_decoder(torch.as_tensor(x[:, lo:hi], device=dev),
                                                 torch.as_tensor(sl[lo:hi], device=dev), W, P, **kw)
    got = gather_to_root(out, lo, P)
    if rank == 0:
        arrs = {"log_probability": got.log_probability.cpu().numpy()}
        for k in got._fields[:-1]:
            arrs.update({"%s_%d" % (k, p): v.cpu().numpy() for p, v in enumerate(getattr(got, k))})
        np.savez(sys.argv[1], **arrs)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
