"""oracle.row_norm (the softmax normaliser restated from
ctc_ext_beam_search_decoder.h:72-80, ctc_oracle.cpp row_normaliser), the
checker test_gpu_prepass.py holds the device normalisers to: against float64
log-sum-exp (close), on rows with -inf, NaN and +inf, and bit-exact against
a class-order loop over Python's libm for double rows."""
import math

import numpy as np

import oracle


def test_row_norm_matches_logsumexp():
    rng = np.random.default_rng(11)
    x = rng.standard_normal((20, 300)).astype(np.float32) * 3
    got = oracle.row_norm(x)
    want = np.log(np.exp(x.astype(np.float64)).sum(1))
    assert np.allclose(got, want, rtol=0, atol=1e-5)


def test_row_norm_special_rows():
    C = 70
    rng = np.random.default_rng(12)
    x = rng.standard_normal((5, C)).astype(np.float32)
    x[1, :] = -np.inf                   # max -inf: every term NaN
    x[2, 5] = np.nan
    x[3, 7] = np.inf
    x[4, 10:] = -np.inf
    got = oracle.row_norm(x)
    assert np.isnan(got[1]) and np.isnan(got[2]) and np.isnan(got[3])
    assert np.isfinite(got[0]) and np.isfinite(got[4])
    want4 = np.log(np.exp(x[4, :10].astype(np.float64)).sum())
    assert abs(float(got[4]) - want4) < 1e-5


def test_row_norm_class_order_f64():
    rng = np.random.default_rng(13)
    x = rng.standard_normal((4, 129))
    got = oracle.row_norm(x)
    assert got.dtype == np.float64
    for r in range(4):
        m = x[r].max()
        s = 0.0
        for v in x[r]:
            s += math.exp(v - m)
        assert got[r] == m + math.log(s)
