"""Full-size checks (BASELINE.json configs at their real B and T) through
size-independent properties, where the CPU oracle would take hours:

* structure: every alignment spans its item's frames, values are labels or
  blank_label, indices are row-major and dense, shapes are the maxima
  (StoreAllDecodedSequences, kernels.cc:163-257);
* consistency: the CTC collapse of a path's best alignment is its label
  prefix (the alignment candidates extend the prefix, ctc_beam_entry.h:190-228),
  and with merge_repeated the decoded sequence is that prefix with equal
  neighbours merged (LabelSeq, ctc_beam_entry.h:123-136);
* ordering: log_probability is non-increasing over the top paths (TopPaths
  extracts in descending order, decoder.h:245-252);
* batch independence (the property the batch sharding relies on,
  kernels.cc:68-90): decoding any contiguous shard gives exactly the rows the
  full batch gives, and repeated calls are bit-identical.

Oracle parity at these shapes is pinned on full-length items: the committed
oracle fixtures tests/golden/full_length.json (cfg3 T=1500, cfg4 T=2000, cfg5
T=3000 and the peaky distribution; test_gpu_parity.py::test_full_length_golden,
and cfg4's items inside the whole B=1024 workload,
test_gpu_sharded.py::test_cfg4_whole_workload_eight_shards), plus the live
oracle at cfg2/cfg3 (test_cfg2_full_length_parity, test_cfg3_full_length_parity).
"""
import numpy as np
import pytest
import torch

import ctcext_amd
from parity_util import to_numpy

pytestmark = pytest.mark.gpu

BLANK_LABEL = -1


def _logits(T, B, C, seed, peaky=False):
    rng = np.random.default_rng(seed)
    x = rng.standard_normal((T, B, C), dtype=np.float32)
    if peaky:   # distribution B of BASELINE.md
        hot = np.where(rng.random((T, B)) < 0.6, 0, rng.integers(1, C, size=(T, B)))
        np.put_along_axis(x, hot[..., None], np.take_along_axis(x, hot[..., None], 2) + 6, 2)
    return x


def _rows(ind, val, B):
    ind, val = to_numpy(ind), to_numpy(val)
    rows = [[] for _ in range(B)]
    for (b, i), v in zip(ind.tolist(), val.tolist()):
        assert i == len(rows[b]), "indices not dense/row-major"
        rows[b].append(v)
    if len(ind):
        assert np.all(np.diff(ind[:, 0]) >= 0), "batch index not sorted"
    return rows


def _collapse(ali):
    out, prev = [], None
    for a in ali:
        if a != BLANK_LABEL and a != prev:
            out.append(a)
        prev = a
    return out


def _merge(seq):
    return [s for k, s in enumerate(seq) if k == 0 or s != seq[k - 1]]


def _decode(x, sl, W, P, merge, blank=0):
    out = ctcext_amd.ctc_ext_beam_search_decoder(x, sl, W, P, merge_repeated=merge, blank_index=blank,
                                                 blank_label=BLANK_LABEL)
    torch.cuda.synchronize()
    return out


def _check_structure(out, sl, C, P, merge, blank=0):
    B = len(sl)
    lp = to_numpy(out.log_probability)
    assert lp.shape == (B, P)
    assert np.all(np.isfinite(lp))
    assert np.all(np.diff(lp, axis=1) <= 0), "top paths not in descending order"
    for p in range(P):
        dec = _rows(out.decoded_indices[p], out.decoded_values[p], B)
        ali = _rows(out.alignment_indices[p], out.alignment_values[p], B)
        assert to_numpy(out.alignment_shape[p]).tolist() == [B, max(len(a) for a in ali)]
        assert to_numpy(out.decoded_shape[p]).tolist() == [B, max(len(d) for d in dec)]
        for b in range(B):
            assert len(ali[b]) == sl[b], (p, b)
            assert all(a == BLANK_LABEL or (0 <= a < C and a != blank) for a in ali[b])
            prefix = _collapse(ali[b])
            assert dec[b] == (_merge(prefix) if merge else prefix), (p, b)


def _assert_same_rows(full, part, lo, B_part, P):
    for p in range(P):
        for k in ("decoded", "alignment"):
            fr = _rows(getattr(full, k + "_indices")[p], getattr(full, k + "_values")[p],
                       to_numpy(full.log_probability).shape[0])
            pr = _rows(getattr(part, k + "_indices")[p], getattr(part, k + "_values")[p], B_part)
            assert fr[lo:lo + B_part] == pr, (k, p)
    np.testing.assert_array_equal(to_numpy(full.log_probability)[lo:lo + B_part], to_numpy(part.log_probability))


@pytest.mark.parametrize("peaky", [False, True])
def test_cfg3_full_size_properties(peaky):
    # cfg3: B=256, T=1500, C=29, W=128, P=3, merge; ragged lengths U[T/2, T]
    B, T, C, W, P = 256, 1500, 29, 128, 3
    x = torch.as_tensor(_logits(T, B, C, 20251016, peaky), device="cuda")
    sl_np = np.random.default_rng(20251016).integers(T // 2, T + 1, size=B).astype(np.int32)
    sl_np[0] = T
    sl = torch.as_tensor(sl_np, device="cuda")
    full = _decode(x, sl, W, P, True)
    _check_structure(full, sl_np, C, P, True)
    # batch independence: two shards of 128 (the 2-GPU split) and a ragged middle shard
    for lo, hi in ((0, 128), (128, 256), (37, 101)):
        part = _decode(x[:, lo:hi].contiguous(), sl[lo:hi].contiguous(), W, P, True)
        _assert_same_rows(full, part, lo, hi - lo, P)
    again = _decode(x, sl, W, P, True)
    _assert_same_rows(full, again, 0, B, P)


def test_cfg2_full_size_properties():
    # cfg2: B=32, T=1000, C=29, W=64, P=1, no merge
    B, T, C, W, P = 32, 1000, 29, 64, 1
    x = torch.as_tensor(_logits(T, B, C, 20251015), device="cuda")
    sl_np = np.full(B, T, np.int32)
    sl = torch.as_tensor(sl_np, device="cuda")
    full = _decode(x, sl, W, P, False)
    _check_structure(full, sl_np, C, P, False)
    part = _decode(x[:, 8:24].contiguous(), sl[8:24].contiguous(), W, P, False)
    _assert_same_rows(full, part, 8, 16, P)


@pytest.mark.parametrize("cfg", ["cfg4", "cfg5"])
def test_large_vocab_full_size_properties(cfg):
    # cfg4 per-GPU shard (B=128 of 1024 over 8 GPUs, T=2000, C=1000, W=64) and
    # cfg5 whole (B=512, T=3000, C=5000, W=256, blank_index=0: 30.7 GB of
    # logits, drawn on the device) at full length; ragged lengths U[T/2, T]
    if cfg == "cfg4":
        B, T, C, W, P = 128, 2000, 1000, 64, 1
    else:
        B, T, C, W, P = 512, 3000, 5000, 256, 1
    g = torch.Generator(device="cuda")
    g.manual_seed(4000 if cfg == "cfg4" else 5000)
    x = torch.randn((T, B, C), generator=g, device="cuda", dtype=torch.float32)
    sl_np = np.random.default_rng(9).integers(T // 2, T + 1, size=B).astype(np.int32)
    sl_np[:2] = T
    sl = torch.as_tensor(sl_np, device="cuda")
    full = _decode(x, sl, W, P, False)
    _check_structure(full, sl_np, C, P, False)
    lo, n = B // 2 - 3, 8
    part = _decode(x[:, lo:lo + n].contiguous(), sl[lo:lo + n].contiguous(), W, P, False)
    _assert_same_rows(full, part, lo, n, P)
    del x
    torch.cuda.empty_cache()


@pytest.mark.parametrize("cfg", ["cfg4", "cfg5"])
def test_large_vocab_shape_properties(cfg):
    # cfg4 (C=1000, W=64) and cfg5 (C=5000, W=256, blank_index=0) per-GPU
    # shapes on a shortened T (the full T runs in bench.py --config)
    if cfg == "cfg4":
        B, T, C, W, P = 128, 200, 1000, 64, 1
    else:
        B, T, C, W, P = 64, 40, 5000, 256, 1
    x = torch.as_tensor(_logits(T, B, C, 7), device="cuda")
    sl_np = np.random.default_rng(8).integers(T // 2, T + 1, size=B).astype(np.int32)
    sl = torch.as_tensor(sl_np, device="cuda")
    full = _decode(x, sl, W, P, False)
    _check_structure(full, sl_np, C, P, False)
    part = _decode(x[:, 5:21].contiguous(), sl[5:21].contiguous(), W, P, False)
    _assert_same_rows(full, part, 5, 16, P)
