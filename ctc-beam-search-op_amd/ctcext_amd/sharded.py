"""Batch-sharded decoding across GPUs (one process per GPU, torch.distributed).

The reference decodes batch items independently (kernels.cc:68-90, one
decoder Reset() per item), so the batch axis shards with no exchange during
decoding.  The only collective is the final gather of each rank's SparseTensor
components to the root, over RCCL (backend "nccl") on MI355X / xGMI:

  1. all_gather of a fixed-size int64 header per rank (entry counts and
     dense widths per path and kind);
  2. one gather of each rank's packed int64 payload (indices and values of
     every path, zero-padded to the largest rank), plus the log-probabilities.

The root shifts each rank's batch indices by the rank's first item and
concatenates in rank order, which is exactly the single-device output order
for contiguous shards.

The collective is chosen per backend, up front (no exception-driven retry: a
collective that fails on some ranks only would leave the others inside a
different one): RCCL ("nccl") gathers the device tensors directly; gloo runs
its collectives on host copies (its gather takes CPU tensors), which is how
the CPU tests and a one-GPU multi-rank rehearsal run.

For one process driving several GPUs, use the op's ``devices=`` argument
instead (ctcext_create_sharded: peer-copy gather inside the library).
"""
import torch
import torch.distributed as dist

from .ops import CTCExtBeamSearchDecoder

_FIELDS = ("decoded_indices", "decoded_values", "alignment_indices", "alignment_values")


def shard_bounds(batch, rank, world):
    """Contiguous shard [lo, hi) of a batch of ``batch`` items for ``rank``."""
    per, rem = divmod(batch, world)
    lo = rank * per + min(rank, rem)
    return lo, lo + per + (1 if rank < rem else 0)


def _host_collectives(group):
    """gloo: collectives on CPU tensors; nccl (RCCL): on the device tensors."""
    return dist.get_backend(group) == "gloo"


def _gather(t, dst, group, world):
    """dist.gather of equal-sized tensors to ``dst`` (a list there, None elsewhere),
    returned on ``t``'s device."""
    rank = dist.get_rank(group)
    dev = t.device
    if _host_collectives(group):
        t = t.cpu()
    lst = [torch.empty_like(t) for _ in range(world)] if rank == dst else None
    dist.gather(t, lst, dst=dst, group=group)
    if lst is None:
        return None
    return [x.to(dev) for x in lst]


def gather_to_root(out, first_item, top_paths, dst=0, group=None):
    """Gather per-rank decoder outputs (torch tensors, same device per rank) to
    ``dst``.  Returns the global CTCExtBeamSearchDecoder on ``dst``, None elsewhere."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    dev = out.log_probability.device
    P = int(top_paths)
    counts = []
    for p in range(P):
        counts += [out.decoded_values[p].numel(), int(out.decoded_shape[p][1]),
                   out.alignment_values[p].numel(), int(out.alignment_shape[p][1])]
    hdr = torch.tensor(counts + [first_item, out.log_probability.shape[0]], dtype=torch.int64,
                       device="cpu" if _host_collectives(group) else dev)
    hdrs = [torch.empty_like(hdr) for _ in range(world)]
    dist.all_gather(hdrs, hdr, group=group)
    hdrs = [h.cpu().tolist() for h in hdrs]
    sizes = [sum(3 * h[4 * p] + 3 * h[4 * p + 2] for p in range(P)) for h in hdrs]
    cap = max(max(sizes), 1)
    parts = []
    for p in range(P):
        parts += [out.decoded_indices[p].reshape(-1), out.decoded_values[p].reshape(-1),
                  out.alignment_indices[p].reshape(-1), out.alignment_values[p].reshape(-1)]
    payload = torch.zeros(cap, dtype=torch.int64, device=dev)
    if parts:
        flat = torch.cat([x.to(torch.int64) for x in parts])
        payload[:flat.numel()] = flat
    got = _gather(payload, dst, group, world)
    lps = _gather_lp(out.log_probability, hdrs, dst, group, world)
    if rank != dst:
        return None
    res = {f: [[] for _ in range(P)] for f in _FIELDS}
    width = {("d", p): 0 for p in range(P)}
    width.update({("a", p): 0 for p in range(P)})
    total_b = 0
    for r in range(world):
        h = hdrs[r]
        buf = got[r]
        o = 0
        first = h[4 * P]
        total_b = max(total_b, first + h[4 * P + 1])
        for p in range(P):
            nd, wd, na, wa = h[4 * p:4 * p + 4]
            di = buf[o:o + 2 * nd].reshape(nd, 2).clone(); o += 2 * nd
            dv = buf[o:o + nd]; o += nd
            ai = buf[o:o + 2 * na].reshape(na, 2).clone(); o += 2 * na
            av = buf[o:o + na]; o += na
            di[:, 0] += first
            ai[:, 0] += first
            res["decoded_indices"][p].append(di); res["decoded_values"][p].append(dv)
            res["alignment_indices"][p].append(ai); res["alignment_values"][p].append(av)
            width[("d", p)] = max(width[("d", p)], wd)
            width[("a", p)] = max(width[("a", p)], wa)
    cat = {f: [torch.cat(res[f][p]) for p in range(P)] for f in _FIELDS}
    ds = [torch.tensor([total_b, width[("d", p)]], dtype=torch.int64, device=dev) for p in range(P)]
    ash = [torch.tensor([total_b, width[("a", p)]], dtype=torch.int64, device=dev) for p in range(P)]
    return CTCExtBeamSearchDecoder(cat["decoded_indices"], cat["decoded_values"], ds,
                                   cat["alignment_indices"], cat["alignment_values"], ash, lps)


def _gather_lp(lp, hdrs, dst, group, world):
    P = lp.shape[1] if lp.dim() == 2 else 1
    bmax = max(h[-1] for h in hdrs)
    pad = torch.zeros((max(bmax, 1), P), dtype=lp.dtype, device=lp.device)
    pad[:lp.shape[0]] = lp
    got = _gather(pad, dst, group, world)
    if got is None:
        return None
    return torch.cat([got[r][:hdrs[r][-1]] for r in range(world)])
