"""The large-vocabulary pre-pass alone (ctcext_row_facts, C ABI diagnostics
entry): each row's record -- maximum, NaN/+inf flag, 64-class block maxima,
the top set S and the largest non-blank value outside it -- checked against a
numpy restatement of its definition (S bit-exact, in order; the maxima and
the outside value by value, as +0.0 and -0.0 tie), on rows built to
stress the selection: ties at the boundary, -inf, signed zeros, fewer finite
labels than the set holds, the blank anywhere, C just above 64 up to 8196,
and both the register path (float, C % 4 == 0: ctcx_row_facts) and the LDS
path (ctcx_row_prep).  The decode parity tests cover the same records only
through their effect on results; S is the gather's exactness bound
(DESIGN.md "Kernels"), so it is pinned here directly.  The normaliser the
same launch writes (fused into ctcx_row_facts on the register path) is
checked bit-exact against the oracle's (oracle.row_norm, decoder.h:72-80),
NaN / +inf rows included, and rows past an item's length are left alone."""
import ctypes
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ctc-beam-search-op_amd"))

import oracle  # noqa: E402  (tests/conftest.py puts oracle/ on the path)

pytestmark = pytest.mark.gpu

K = 64   # kTopK


def _fkey(bits):
    u = bits.astype(np.uint64)
    return np.where(u >> 31, u ^ 0xFFFFFFFF, u ^ 0x80000000)


def _ref(row, blank):
    """(xmax, bad, block maxima, S bits, S label indices, xout) by definition:
    S = the non-blank labels whose order-preserving key lies above the (K+1)-th
    largest key (every label when there are at most K), in label order; xout =
    the largest non-blank value outside S (-inf: none)."""
    C = row.size
    bad = bool(np.isnan(row).any() or np.isposinf(row).any())
    xmax = np.float32(row.max())
    bmax = np.array([row[k:k + 64].max() for k in range(0, C, 64)], dtype=np.float32)
    cls = np.array([c for c in range(C) if c != blank])
    vals = row[cls]
    keys = _fkey(vals.view(np.uint32))
    lab = cls - (cls > blank)
    if C - 1 <= K:
        inS = np.ones(cls.size, bool)
        xout = np.float32(-np.inf)
    else:
        v = np.sort(keys)[::-1][K]
        inS = keys > v
        xout = vals[keys == v][0]
    return xmax, bad, bmax, vals[inS].view(np.uint32), lab[inS], np.float32(xout)


def _rows(rng, C, kind, n):
    x = rng.standard_normal((n, C)).astype(np.float32)
    if kind == "ties":
        x = (np.round(x * 2) / 2).astype(np.float32)
    elif kind == "neg_inf":
        x[rng.random((n, C)) < 0.4] = -np.inf
    elif kind == "few_finite":   # fewer finite labels than S holds
        x[:] = -np.inf
        for r in range(n):
            x[r, rng.choice(C, size=min(C, 10), replace=False)] = rng.standard_normal(min(C, 10))
    elif kind == "zeros":        # +0.0 / -0.0 (distinct keys, equal values)
        x = np.where(rng.random((n, C)) < 0.5, np.float32(0.0), np.float32(-0.0)).astype(np.float32)
        x[:, : C // 7] = rng.standard_normal((n, C // 7)).astype(np.float32)
    elif kind == "flat":
        x[:] = np.float32(1.25)
    elif kind == "all_neg_inf":  # a row of -inf only: maximum -inf, every term NaN
        x[0, :] = -np.inf
        if n > 2:
            x[2, : C // 2] = -np.inf
    elif kind == "bad":
        x[0, C // 3] = np.nan
        if n > 1:
            x[1, C // 2] = np.inf
    return x


def _run(x_tb, C, blank, dtype=np.float32, seq_len=None):
    import torch
    import ctcext_amd
    from ctcext_amd import _lib
    T, B = x_tb.shape[:2]
    d = ctcext_amd.get_decoder(0)
    lib = d.lib
    rb = ctypes.c_int64()
    dt = _lib.CTCEXT_F64 if dtype == np.float64 else _lib.CTCEXT_F32
    xs = torch.as_tensor(np.ascontiguousarray(x_tb.astype(dtype)), device="cuda")
    if seq_len is None:
        seq_len = np.full(B, T, np.int32)
    sl = torch.as_tensor(np.asarray(seq_len, np.int32), device="cuda")
    assert lib.ctcext_row_facts(d.handle, None, dt, T, B, C, blank, None, None, None, ctypes.byref(rb)) == 0
    prep = torch.zeros(T * B * rb.value, dtype=torch.uint8, device="cuda")
    norm = torch.full((T * B,), 7.5, dtype=torch.float64 if dtype == np.float64 else torch.float32, device="cuda")
    rc = lib.ctcext_row_facts(d.handle, ctypes.c_void_p(xs.data_ptr()), dt, T, B, C, blank,
                              ctypes.c_void_p(sl.data_ptr()), ctypes.c_void_p(prep.data_ptr()),
                              ctypes.c_void_p(norm.data_ptr()), ctypes.byref(rb))
    assert rc == 0, lib.ctcext_last_error()
    return prep.cpu().numpy().reshape(T * B, rb.value), norm.cpu().numpy()


def _check_norm(x_tb, norm, seq_len=None):
    T, B, C = x_tb.shape
    want = oracle.row_norm(x_tb.reshape(-1, C))
    live = np.ones((T, B), bool) if seq_len is None else np.arange(T)[:, None] < np.asarray(seq_len)[None, :]
    live = live.reshape(-1)
    got = norm
    same = (got.view(np.uint32 if got.dtype == np.float32 else np.uint64)
            == want.view(np.uint32 if want.dtype == np.float32 else np.uint64)) | (np.isnan(got) & np.isnan(want))
    assert same[live].all(), (C, np.flatnonzero(live & ~same)[:8], got[live & ~same][:4], want[live & ~same][:4])
    assert (got[~live] == 7.5).all(), "rows past an item's length are not written"


def _check_f32(x_tb, C, blank, seq_len=None):
    rec, norm = _run(x_tb, C, blank, seq_len=seq_len)
    _check_norm(x_tb, norm, seq_len)
    rows = x_tb.reshape(-1, C)
    nblk = (C + 63) // 64
    top_off = 16 + ((nblk * 4 + 15) & ~15)
    live = None if seq_len is None else (np.arange(x_tb.shape[0])[:, None] < np.asarray(seq_len)[None, :]).reshape(-1)
    for r in range(rows.shape[0]):
        if live is not None and not live[r]:
            continue
        xmax, bad, bmax, sb, sl_, xout = _ref(rows[r], blank)
        h = rec[r]
        gmax = h[0:4].view(np.float32)[0]
        gbad = h[8:12].view(np.int32)[0]
        assert bool(gbad) == bad, (C, blank, r)
        if bad:
            continue
        # maxima by value: of equal values (+0.0 / -0.0) either may be kept
        assert gmax == xmax, (C, blank, r, gmax, xmax)
        assert np.array_equal(h[16:16 + 4 * nblk].view(np.float32), bmax), (C, blank, r)
        ns = h[12:16].view(np.int32)[0]
        gxout = h[4:8].view(np.float32)[0]
        assert ns == sb.size, (C, blank, r, ns, sb.size)
        top = h[top_off:top_off + 8 * ns].view(np.uint32).reshape(ns, 2)
        assert np.array_equal(top[:, 0], sb), (C, blank, r)
        assert np.array_equal(top[:, 1], sl_.astype(np.uint32)), (C, blank, r)
        assert gxout == xout, (C, blank, r, gxout, xout)


@pytest.mark.parametrize("C", [68, 256, 260, 1000, 2048, 5000, 8196, 65, 1001, 5001])
def test_row_facts_match_definition(C):
    rng = np.random.default_rng(7000 + C)
    for kind in ("normal", "ties", "neg_inf", "few_finite", "zeros", "flat", "all_neg_inf", "bad"):
        for blank in (0, C - 1, C // 2):
            x = _rows(rng, C, kind, 6).reshape(2, 3, C)
            _check_f32(x, C, blank)


@pytest.mark.parametrize("C", [124, 128, 512, 516, 772, 1020, 1024, 1028, 2048, 3072])
def test_row_facts_nv_boundaries(C):
    # the row widths at the edges of each compiled NV (and of the fused
    # normaliser's C <= 1024), 5 x 7 rows: the last block of eight (two rows
    # per wave, fused) or four rows only partly filled
    rng = np.random.default_rng(7200 + C)
    x = (rng.standard_normal((5, 7, C)) * 2).astype(np.float32)
    x[1, 2, :] = -np.inf
    x[3, 4, C // 3] = np.nan
    _check_f32(x, C, C // 5, seq_len=[5, 4, 5, 2, 5, 3, 1])


@pytest.mark.parametrize("C", [68, 1000, 5000, 5001])
def test_row_facts_ragged_lengths(C):
    # items of different lengths: some of a block's four rows are past their
    # item's end (the fused kernel's waves still meet its barriers)
    rng = np.random.default_rng(7100 + C)
    T, B = 5, 7
    x = rng.standard_normal((T, B, C)).astype(np.float32) * 3
    x[2, 3, C // 5] = np.nan
    x[4, 0, 1] = np.inf
    _check_f32(x, C, 0, seq_len=[5, 1, 0, 3, 4, 2, 5])


def test_row_facts_f64_header_and_block_maxima():
    # double rows carry no top set (|S| = 0: the decode takes the plain path)
    C = 300
    rng = np.random.default_rng(7300)
    x = rng.standard_normal((2, 3, C))
    rec, norm = _run(x, C, 5, np.float64)
    _check_norm(x, norm)
    rows = x.reshape(-1, C)
    nblk = (C + 63) // 64
    for r in range(rows.shape[0]):
        h = rec[r]
        assert h[0:8].view(np.float64)[0] == rows[r].max()
        assert h[16:20].view(np.int32)[0] == 0
        bm = np.array([rows[r][k:k + 64].max() for k in range(0, C, 64)])
        assert np.array_equal(h[32:32 + 8 * nblk].view(np.float64), bm)
