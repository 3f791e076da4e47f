"""The extract by rank (help_rank_extract, ctcx_decode.hip): at C <= 64 and
beams of 16..128 the helper wave ranks the final heap and places every
position above the highest group of equal totals, and wave 0's sort_heap
stops there.  Against the oracle's literal sort_heap (oracle/ctc_oracle.cpp,
TopN Extract, decoder.h:84) on the three regimes the placement can take:
totals all distinct (the helper places every position), ties at the top (it
places none) and ties part-way down, at beam widths on both sides of the
threshold and of each extract segment (96, 64, 32).  (A build whose helper
wrote position r ^ 1 instead of r failed 6 of these 13 on the GPU.)"""
import numpy as np
import pytest

import ctcext_amd
from parity_util import compare, oracle_or_error
from test_gpu_parity import _gpu_or_error

pytestmark = pytest.mark.gpu


def _run(x, sl, W, P, kw):
    ref, rerr = oracle_or_error(x, sl, W, P, kw)
    out, gerr = _gpu_or_error(x, sl, W, P, kw)
    assert rerr == gerr, (rerr, gerr)
    if ref is not None:
        compare(out, ref, P)
    st = ctcext_amd.get_decoder(0).last_stats
    assert st["helper"] == 3, st   # the scored queue: the kernel that ranks


@pytest.mark.parametrize("W", [15, 16, 33, 64, 65, 97, 128])
def test_rank_extract_distinct_totals(W):
    # short sequences of spread logits: the totals of a frame rarely tie, so
    # the helper's stop sits at or near the beam's end
    rng = np.random.default_rng(100 + W)
    for T in (2, 3, 4, 6):
        x = (rng.standard_normal((T, 3, 29)) * 4).astype(np.float32)
        sl = np.full(3, T, np.int32)
        _run(x, sl, W, min(3, W), dict(merge_repeated=True))


@pytest.mark.parametrize("W", [16, 64, 128])
def test_rank_extract_tied_totals(W):
    # logits on a coarse grid: most totals tie, many at the top
    rng = np.random.default_rng(200 + W)
    for T in (3, 8, 40):
        x = (np.round(rng.standard_normal((T, 3, 29)) * 2) / 2).astype(np.float32)
        sl = np.array([T, max(T - 1, 1), T], np.int32)
        _run(x, sl, W, min(3, W), dict(merge_repeated=bool(T % 2)))


@pytest.mark.parametrize("W", [48, 100, 128])
def test_rank_extract_long_sequences(W):
    # cfg3-like rows: ties appear as |total| grows, so the highest tie climbs
    # toward the top over the sequence
    rng = np.random.default_rng(300 + W)
    T = 300
    x = rng.standard_normal((T, 2, 29)).astype(np.float32)
    sl = np.array([T, T - 37], np.int32)
    _run(x, sl, W, 3, dict(merge_repeated=True))
