"""Helpers shared by the parity tests: run the product (GPU through the C ABI)
and the oracle (CPU restatement) on the same inputs and compare every output.

Tolerance: the north star requires decoded/alignment indices, values and
shapes bit-exact and log_probability within 1e-5.  The device path reproduces
the reference's float arithmetic operation for operation, so the tests demand
log_probability bit-exact too (assert_array_equal); 1e-5 is sub-ULP once
|lp| >= 128 anyway.
"""
import numpy as np

import oracle


def to_numpy(a):
    if hasattr(a, "detach"):
        return a.detach().cpu().numpy()
    return np.asarray(a)


def compare(out, ref, top_paths, lp_exact=True):
    for p in range(top_paths):
        for name in ("decoded_indices", "decoded_values", "decoded_shape",
                     "alignment_indices", "alignment_values", "alignment_shape"):
            got = to_numpy(getattr(out, name)[p])
            exp = np.asarray(getattr(ref, name)[p])
            assert got.dtype == np.int64, (name, got.dtype)
            np.testing.assert_array_equal(got.reshape(exp.shape), exp, err_msg="%s[%d]" % (name, p))
    lp = to_numpy(out.log_probability)
    if lp_exact:
        np.testing.assert_array_equal(lp, ref.log_probability)
    else:
        np.testing.assert_allclose(lp, ref.log_probability, rtol=0, atol=1e-5)


def random_case(rng, T_max=40, B_max=3, C_max=11, W_max=15, ties=False, neg_inf=False, dtype=np.float32,
                C_min=2, scale=1.0, W_min=1):
    T = int(rng.integers(1, T_max + 1))
    B = int(rng.integers(1, B_max + 1))
    C = int(rng.integers(C_min, C_max + 1))
    W = int(rng.integers(W_min, W_max + 1))
    P = int(rng.integers(1, W + 1))
    x = (rng.standard_normal((T, B, C)) * scale).astype(dtype)
    if ties:
        x = (np.round(x * 2) / 2).astype(dtype)
    if neg_inf:
        x[rng.random(x.shape) < 0.15] = -np.inf
    sl = rng.integers(max(T // 2, 0), T + 1, size=B).astype(np.int32)
    kw = dict(merge_repeated=bool(rng.integers(2)), blank_index=int(rng.integers(C)),
              blank_label=int(rng.integers(-1, C)))
    return x, sl, W, P, kw


def oracle_or_error(x, sl, W, P, kw, mode="shared"):
    try:
        return oracle.decode(x, sl, W, P, mode=mode, **kw), None
    except oracle.OracleError as e:
        return None, str(e)
