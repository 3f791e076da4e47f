"""Parity of the HIP path (through libctcext.so's C ABI) against the oracle and
the reference's golden vector.  Needs an MI355X."""
import json
import os

import numpy as np
import pytest

import ctcext_amd
from ctcext_amd import _lib
from parity_util import compare, oracle_or_error, random_case, to_numpy
import oracle

pytestmark = pytest.mark.gpu

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "paper_example.json")))


def _gpu_or_error(x, sl, W, P, kw, device=False, flags=0):
    try:
        if device:
            import torch
            xt = torch.as_tensor(x, device="cuda")
            slt = torch.as_tensor(sl, device="cuda")
            return ctcext_amd.ctc_ext_beam_search_decoder(xt, slt, W, P, flags=flags, **kw), None
        return ctcext_amd.ctc_ext_beam_search_decoder(x, sl, W, P, flags=flags, **kw), None
    except ctcext_amd.OpError as e:
        return None, e.message


@pytest.mark.parametrize("device", [False, True])
def test_paper_golden_f32(device):
    a = GOLD["attrs"]
    logits = np.log(np.asarray(GOLD["probs"])).astype(np.float32)
    out, err = _gpu_or_error(logits, np.asarray(GOLD["sequence_length"], np.int32), a["beam_width"],
                             a["top_paths"], dict(merge_repeated=a["merge_repeated"],
                                                  blank_index=a["blank_index"],
                                                  blank_label=a["blank_label"]), device=device)
    assert err is None, err
    for p in range(a["top_paths"]):
        np.testing.assert_array_equal(to_numpy(out.decoded_indices[p]), GOLD["decoded_indices"][p])
        np.testing.assert_array_equal(to_numpy(out.decoded_values[p]), GOLD["decoded_values"][p])
        np.testing.assert_array_equal(to_numpy(out.decoded_shape[p]), GOLD["decoded_shape"][p])
        np.testing.assert_array_equal(to_numpy(out.alignment_indices[p]), GOLD["alignment_indices"][p])
        np.testing.assert_array_equal(to_numpy(out.alignment_values[p]), GOLD["alignment_values"][p])
        np.testing.assert_array_equal(to_numpy(out.alignment_shape[p]), GOLD["alignment_shape"][p])
    np.testing.assert_allclose(to_numpy(out.log_probability), GOLD["log_probability"], rtol=1e-6, atol=1e-6)
    ref = oracle.decode(logits, GOLD["sequence_length"], a["beam_width"], a["top_paths"],
                        a["merge_repeated"], a["blank_index"], a["blank_label"])
    compare(out, ref, a["top_paths"])


def _run_random(seed, n, flags=0, device=False, **kw_case):
    rng = np.random.default_rng(seed)
    for it in range(n):
        x, sl, W, P, kw = random_case(rng, **kw_case)
        ref, rerr = oracle_or_error(x, sl, W, P, kw)
        out, gerr = _gpu_or_error(x, sl, W, P, kw, flags=flags, device=device and it % 2 == 1)
        assert rerr == gerr, (it, rerr, gerr)
        if ref is not None:
            compare(out, ref, P)


def test_random_small():
    _run_random(1234, 150)


def test_random_tie_heavy():
    _run_random(4321, 100, ties=True)


def test_random_mid():
    _run_random(99, 12, T_max=120, B_max=4, C_max=30, W_max=64)


def test_force_literal_matches_oracle():
    rng = np.random.default_rng(5)
    for it in range(40):
        x, sl, W, P, kw = random_case(rng, ties=bool(it % 2))
        ref, rerr = oracle_or_error(x, sl, W, P, kw)
        out, gerr = _gpu_or_error(x, sl, W, P, kw, flags=_lib.CTCEXT_FLAG_FORCE_LITERAL)
        assert rerr == gerr, (it, rerr, gerr)
        if ref is not None:
            compare(out, ref, P)


def _dup_frames():
    return ctcext_amd.get_decoder(0).last_stats["duplicate_frames"]


def test_neg_inf_logits():
    rng = np.random.default_rng(77)
    dup_cases = 0
    for it in range(60):
        x, sl, W, P, kw = random_case(rng, neg_inf=True)
        st = {}
        try:
            ref, rerr = oracle.decode(x, sl, W, P, stats=st, **kw), None
        except oracle.OracleError as e:
            ref, rerr = None, str(e)
        out, gerr = _gpu_or_error(x, sl, W, P, kw)
        assert rerr == gerr, (it, rerr, gerr)
        if ref is not None:
            compare(out, ref, P)
            assert _dup_frames() == st["duplicate_frames"], it
            dup_cases += st["duplicate_frames"] > 0
    print("neg-inf cases whose beam held an entry twice: %d of 60" % dup_cases)


def _dup_family(seed, n_want, dtype=np.float32, max_tries=4000):
    """Seeded single-item -inf-heavy cases that the oracle reports reaching the
    duplicate-entry state (decoder.h:142 pushes every branch, :189-199 re-pushes
    a non-Active branch as a child, so one BeamEntry sits in the beam twice)."""
    rng = np.random.default_rng(seed)
    got = []
    for _ in range(max_tries):
        T = int(rng.integers(2, 30)); C = int(rng.integers(2, 8)); W = int(rng.integers(1, 10))
        x = rng.standard_normal((T, 1, C)).astype(dtype)
        x[rng.random(x.shape) < (0.3 if rng.random() < 0.5 else 0.5)] = -np.inf
        P = int(rng.integers(1, W + 1))
        kw = dict(merge_repeated=bool(rng.integers(2)), blank_index=int(rng.integers(C)),
                  blank_label=int(rng.integers(-1, C)))
        st = {}
        try:
            ref = oracle.decode(x, [T], W, P, stats=st, **kw)
        except oracle.OracleError:
            continue
        if st["duplicate_frames"]:
            got.append((x, np.array([T], np.int32), W, P, kw, ref, st["duplicate_frames"]))
            if len(got) == n_want:
                break
    assert len(got) == n_want
    return got


@pytest.mark.parametrize("dtype,flags", [(np.float32, 0), (np.float64, 0),
                                         (np.float32, _lib.CTCEXT_FLAG_FORCE_LITERAL),
                                         (np.float32, _lib.CTCEXT_FLAG_RING_MIN)])
def test_duplicate_entry_state(dtype, flags):
    # the reference's beam holding one BeamEntry twice, reproduced bit-exactly:
    # second roll empties old_cands, second recursion accumulates, shared
    # children (ctcx_decode.hip literal_step); the device counts the same
    # number of duplicate frames as the oracle
    for k, (x, sl, W, P, kw, ref, nd) in enumerate(_dup_family(31337, 30, dtype)):
        out, err = _gpu_or_error(x, sl, W, P, kw, flags=flags)
        assert err is None, (k, err)
        compare(out, ref, P)
        assert _dup_frames() == nd, (k, _dup_frames(), nd)


def test_duplicate_entry_batch_with_finite_items():
    # duplicate items next to ordinary items in one batch (per-item state)
    rng = np.random.default_rng(1)
    for (x, sl, W, P, kw, _, nd) in _dup_family(4242, 6):
        Tb = x.shape[0]
        big = rng.standard_normal((Tb, 3, x.shape[2])).astype(np.float32)
        big[:, 1] = x[:, 0]
        slb = np.array([Tb, Tb, max(Tb - 3, 0)], np.int32)
        st = {}
        ref = oracle.decode(big, slb, W, P, stats=st, **kw)
        out, err = _gpu_or_error(big, slb, W, P, kw, device=True)
        assert err is None, err
        compare(out, ref, P)
        assert _dup_frames() == st["duplicate_frames"]


def test_cfg1_exact_workload():
    # BASELINE configs[0]: B=2, T=50, C=6, beam_width=4, top_paths=1, the reference's
    # CPU plumbing case, on both input distributions of BASELINE.md
    rng = np.random.default_rng(20251015)
    x = rng.standard_normal((50, 2, 6), dtype=np.float32)
    sl = np.full(2, 50, np.int32)
    kw = dict(merge_repeated=False, blank_index=0, blank_label=-1)
    ref = oracle.decode(x, sl, 4, 1, **kw)
    for device in (False, True):
        out, err = _gpu_or_error(x, sl, 4, 1, kw, device=device)
        assert err is None, err
        compare(out, ref, 1)
    hot = np.where(rng.random((50, 2)) < 0.6, 0, rng.integers(1, 6, size=(50, 2)))
    xb = x.copy()
    np.put_along_axis(xb, hot[..., None], np.take_along_axis(xb, hot[..., None], 2) + 6, 2)
    out, err = _gpu_or_error(xb, sl, 4, 1, kw)
    assert err is None, err
    compare(out, oracle.decode(xb, sl, 4, 1, **kw), 1)


def test_cfg2_shape_parity():
    # cfg2 shape (C=29, W=64, P=1) at a length the oracle finishes quickly
    rng = np.random.default_rng(20251015)
    x = rng.standard_normal((300, 4, 29)).astype(np.float32)
    sl = np.array([300, 250, 300, 17], np.int32)
    kw = dict(merge_repeated=False, blank_index=0, blank_label=-1)
    ref = oracle.decode(x, sl, 64, 1, **kw)
    out, err = _gpu_or_error(x, sl, 64, 1, kw, device=True)
    assert err is None, err
    compare(out, ref, 1)


def test_cfg3_shape_parity():
    # cfg3 attrs (C=29, W=128, P=3, merge) on a shortened T
    rng = np.random.default_rng(20251016)
    x = rng.standard_normal((200, 3, 29)).astype(np.float32)
    sl = np.array([200, 200, 150], np.int32)
    kw = dict(merge_repeated=True, blank_index=0, blank_label=-1)
    ref = oracle.decode(x, sl, 128, 3, **kw)
    out, err = _gpu_or_error(x, sl, 128, 3, kw, device=True)
    assert err is None, err
    compare(out, ref, 3)


def test_peaky_distribution_parity():
    # distribution B of BASELINE.md: +6 on blank w.p. 0.6 else on a random label
    rng = np.random.default_rng(3)
    T, B, C = 150, 3, 29
    x = rng.standard_normal((T, B, C)).astype(np.float32)
    hot = np.where(rng.random((T, B)) < 0.6, 0, rng.integers(1, C, size=(T, B)))
    np.put_along_axis(x, hot[..., None], np.take_along_axis(x, hot[..., None], 2) + 6, 2)
    sl = np.full(B, T, np.int32)
    kw = dict(merge_repeated=True, blank_index=0, blank_label=-1)
    ref = oracle.decode(x, sl, 32, 2, **kw)
    out, err = _gpu_or_error(x, sl, 32, 2, kw)
    assert err is None, err
    compare(out, ref, 2)


def test_edge_cases():
    kw = dict(merge_repeated=False, blank_index=0, blank_label=-1)
    # zero-length item: empty paths, lp 0 (only top_paths=1 is possible)
    x = np.random.default_rng(0).standard_normal((5, 3, 4)).astype(np.float32)
    sl = np.array([5, 0, 3], np.int32)
    ref = oracle.decode(x, sl, 4, 1, **kw)
    out, err = _gpu_or_error(x, sl, 4, 1, kw)
    assert err is None
    compare(out, ref, 1)
    # errors, verbatim
    _, err = _gpu_or_error(x, sl, 2, 3, kw)
    assert err == "requested more paths than the beam width."
    _, err = _gpu_or_error(x[:1], np.array([1, 1, 1], np.int32), 10, 5, kw)
    assert err == "Less leaves in the beam search than requested."
    _, err = _gpu_or_error(x, np.array([6, 1, 1], np.int32), 4, 1, kw)
    assert err == "sequence_length(0) <= 5"
    # C = 2, W = 1, blank last
    x2 = np.random.default_rng(1).standard_normal((30, 2, 2)).astype(np.float32)
    for W, P, blank in ((1, 1, 1), (3, 2, 0)):
        kw2 = dict(merge_repeated=True, blank_index=blank, blank_label=7)
        ref = oracle.decode(x2, [30, 29], W, P, **kw2)
        out, err = _gpu_or_error(x2, np.array([30, 29], np.int32), W, P, kw2)
        assert err is None
        compare(out, ref, P)


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_single_class(dtype):
    # num_classes == 1: the blank alone, no label is ever offered (decoder.h:
    # 146-209 loops over no label); the root is the only leaf, so only
    # top_paths == 1 decodes.  Routed to the literal path (the fast
    # paths' offer arithmetic divides by C - 1)
    rng = np.random.default_rng(5)
    x = rng.standard_normal((40, 3, 1)).astype(dtype)
    sl = np.array([40, 0, 17], np.int32)
    for W, blank_label in ((1, -1), (4, 0), (128, 3), (200, -1)):
        kw = dict(merge_repeated=True, blank_index=0, blank_label=blank_label)
        ref = oracle.decode(x, sl, W, 1, **kw)
        out, err = _gpu_or_error(x, sl, W, 1, kw)
        assert err is None, err
        compare(out, ref, 1)
    _, err = _gpu_or_error(x, sl, 4, 2, dict(merge_repeated=False, blank_index=0, blank_label=-1))
    assert err == "Less leaves in the beam search than requested."


def test_wide_beams():
    # R = 4 and R = 8 register tiers (beam_width > 128)
    rng = np.random.default_rng(11)
    for W in (200, 400):
        x = rng.standard_normal((25, 2, 40)).astype(np.float32)
        sl = np.array([25, 20], np.int32)
        kw = dict(merge_repeated=False, blank_index=3, blank_label=-1)
        ref = oracle.decode(x, sl, W, 4, **kw)
        out, err = _gpu_or_error(x, sl, W, 4, kw)
        assert err is None, err
        compare(out, ref, 4)


def test_repeat_calls_stable():
    # the reference's memory-leak test (test.py:102-123) calls the op 1000x;
    # here: repeated calls reuse the workspace and give identical outputs
    a = GOLD["attrs"]
    logits = np.log(np.asarray(GOLD["probs"])).astype(np.float32)
    first = None
    for _ in range(200):
        out = ctcext_amd.ctc_ext_beam_search_decoder(logits, [8], 10, 5, blank_index=0, blank_label=0)
        if first is None:
            first = out
        else:
            for p in range(5):
                np.testing.assert_array_equal(out.alignment_values[p], first.alignment_values[p])
            np.testing.assert_array_equal(out.log_probability, first.log_probability)


def test_cfg3_full_length_parity():
    # full cfg3 item length: from frame ~7 on most frames hold exactly tied beam
    # totals (float grid at |lp| ~ 10^3), so this pins the TopN tie order
    rng = np.random.default_rng(20251015)
    x = rng.standard_normal((1500, 2, 29)).astype(np.float32)
    sl = np.array([1500, 1400], np.int32)
    kw = dict(merge_repeated=True, blank_index=0, blank_label=-1)
    ref = oracle.decode(x, sl, 128, 3, **kw)
    out, err = _gpu_or_error(x, sl, 128, 3, kw, device=True)
    assert err is None, err
    compare(out, ref, 3)


def test_cfg2_full_length_parity():
    rng = np.random.default_rng(77)
    x = rng.standard_normal((1000, 2, 29)).astype(np.float32)
    sl = np.array([1000, 1000], np.int32)
    kw = dict(merge_repeated=False, blank_index=0, blank_label=-1)
    ref = oracle.decode(x, sl, 64, 1, **kw)
    out, err = _gpu_or_error(x, sl, 64, 1, kw, device=True)
    assert err is None, err
    compare(out, ref, 1)


# ---- T=double (the reference's own test runs float64, test.py:25) ----------

@pytest.mark.parametrize("device", [False, True])
def test_paper_golden_f64(device):
    a = GOLD["attrs"]
    logits = np.log(np.asarray(GOLD["probs"], np.float64))
    out, err = _gpu_or_error(logits, np.asarray(GOLD["sequence_length"], np.int32), a["beam_width"],
                             a["top_paths"], dict(merge_repeated=a["merge_repeated"],
                                                  blank_index=a["blank_index"],
                                                  blank_label=a["blank_label"]), device=device)
    assert err is None, err
    assert to_numpy(out.log_probability).dtype == np.float64
    for p in range(a["top_paths"]):
        np.testing.assert_array_equal(to_numpy(out.decoded_values[p]), GOLD["decoded_values"][p])
        np.testing.assert_array_equal(to_numpy(out.alignment_values[p]), GOLD["alignment_values"][p])
        np.testing.assert_array_equal(to_numpy(out.alignment_indices[p]), GOLD["alignment_indices"][p])
    np.testing.assert_allclose(to_numpy(out.log_probability), GOLD["log_probability"], rtol=1e-6, atol=1e-6)
    ref = oracle.decode(logits, GOLD["sequence_length"], a["beam_width"], a["top_paths"],
                        a["merge_repeated"], a["blank_index"], a["blank_label"])
    compare(out, ref, a["top_paths"])


def test_random_small_f64():
    _run_random(2468, 100, dtype=np.float64)


def test_random_tie_heavy_f64():
    _run_random(8642, 60, ties=True, dtype=np.float64)


def test_force_literal_f64():
    rng = np.random.default_rng(55)
    for it in range(20):
        x, sl, W, P, kw = random_case(rng, ties=bool(it % 2), dtype=np.float64)
        ref, rerr = oracle_or_error(x, sl, W, P, kw)
        out, gerr = _gpu_or_error(x, sl, W, P, kw, flags=_lib.CTCEXT_FLAG_FORCE_LITERAL)
        assert rerr == gerr, (it, rerr, gerr)
        if ref is not None:
            compare(out, ref, P)


def test_cfg3_shape_parity_f64():
    rng = np.random.default_rng(20251017)
    x = rng.standard_normal((300, 2, 29))
    sl = np.array([300, 260], np.int32)
    kw = dict(merge_repeated=True, blank_index=0, blank_label=-1)
    ref = oracle.decode(x, sl, 128, 3, **kw)
    out, err = _gpu_or_error(x, sl, 128, 3, kw, device=True)
    assert err is None, err
    compare(out, ref, 3)


def test_random_reoffer_heavy():
    # small C and W over longer T: frequent evictions of branches, re-offers,
    # deactivations and branch turns that close mid-chunk
    _run_random(777, 300, T_max=60, B_max=3, C_max=6, W_max=10, ties=True)
    _run_random(778, 150, T_max=60, B_max=2, C_max=40, W_max=6)


def test_random_large_c_skips():
    # C > 64 runs the large-C kernel (branch scan 64 branches per step, block-max
    # window scan, per-label refinement); W > 64 makes the branch scan take more
    # than one step; peaked rows (scale 4) make most branches and windows
    # skippable, ties and small W make evictions and re-offers (bloom) frequent
    _run_random(881, 25, T_max=40, B_max=2, C_min=65, C_max=400, W_max=150, scale=4.0)
    _run_random(882, 25, T_max=40, B_max=2, C_min=65, C_max=300, W_max=8, ties=True)
    _run_random(883, 15, T_max=30, B_max=2, C_min=65, C_max=200, W_max=100)
    # the float64 large-C instantiation
    _run_random(884, 10, T_max=30, B_max=2, C_min=65, C_max=300, W_max=80, scale=4.0, dtype=np.float64)


def test_random_large_c_compacted():
    # the large-C gather (compacted chunks): wide beams (nb > 64: several
    # branch groups; W > 128: the RN=2 heap) make most branches parents, so
    # children are merged into the row's top set or found by the window path;
    # C near 65 puts nearly every label in the top set; tie-heavy rows put ties
    # at the top set's threshold; long beams fill chunks mid-branch
    _run_random(891, 12, T_max=30, B_max=2, C_min=65, C_max=130, W_min=100, W_max=256, scale=1.5)
    _run_random(892, 12, T_max=30, B_max=2, C_min=65, C_max=70, W_min=30, W_max=128)
    _run_random(893, 12, T_max=30, B_max=2, C_min=100, C_max=400, W_min=20, W_max=200, ties=True)
    _run_random(894, 8, T_max=40, B_max=2, C_min=300, C_max=1200, W_min=64, W_max=256, scale=2.5)


def test_random_large_c_top_set():
    # the row's top set S (ctcx_row_prep, 64 labels): C just above it makes S a
    # strict subset; flat rows (small scale) and wide beams give top branches
    # more hot offers than S holds (the window path takes over) and many
    # branch children to merge; ties put equal values at the threshold and in
    # S; C above 2048 (a wider S was tried there)
    _run_random(911, 10, T_max=30, B_max=2, C_min=66, C_max=200, W_min=100, W_max=256, scale=0.3)
    _run_random(912, 6, T_max=16, B_max=2, C_min=2049, C_max=2400, W_min=100, W_max=256, scale=0.3)
    _run_random(913, 6, T_max=16, B_max=2, C_min=2049, C_max=2200, W_min=20, W_max=200, ties=True)
    _run_random(914, 4, T_max=24, B_max=2, C_min=2049, C_max=4000, W_min=64, W_max=256, scale=0.5)


def test_random_wide_beam_events():
    # beams of 129..256 (float): the two-group asm event loop (heap_events_m2_f32)
    # with the stop in either group, small C (64-offer chunks) and large C
    # (compacted chunks); tie-heavy rows exercise the right-on-ties picks of
    # both groups and the stop at node 63's right child
    _run_random(901, 10, T_max=40, B_max=2, C_min=3, C_max=40, W_min=129, W_max=256)
    _run_random(902, 10, T_max=40, B_max=2, C_min=3, C_max=30, W_min=129, W_max=256, ties=True)
    _run_random(903, 8, T_max=30, B_max=2, C_min=65, C_max=500, W_min=129, W_max=256, ties=True)


# ---- large vocabularies (cfg4-like C=1000/W=64, cfg5-like
# C=5000/W=256), against committed oracle outputs (tests/golden/make_fixtures.py)

LARGE = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "large_vocab.json")))


@pytest.mark.parametrize("name", sorted(LARGE))
def test_large_vocab_golden(name):
    import hashlib
    import torch
    fx = LARGE[name]
    seed, T, B, C, W, P, merge, blank, blabel, sl = fx["case"]
    x = np.random.default_rng(seed).standard_normal((T, B, C), dtype=np.float32)
    assert hashlib.sha256(x.tobytes()).hexdigest() == fx["sha256"], "input stream changed"
    out = ctcext_amd.ctc_ext_beam_search_decoder(
        torch.as_tensor(x, device="cuda"), torch.as_tensor(np.asarray(sl, np.int32), device="cuda"),
        W, P, merge_repeated=merge, blank_index=blank, blank_label=blabel)
    for p in range(P):
        for k in ("decoded_indices", "decoded_values", "decoded_shape",
                  "alignment_indices", "alignment_values", "alignment_shape"):
            got = to_numpy(getattr(out, k)[p])
            exp = np.asarray(fx[k][p], np.int64)
            np.testing.assert_array_equal(got.reshape(exp.shape), exp, err_msg="%s[%d]" % (k, p))
    lp = np.asarray([[float.fromhex(h) for h in row] for row in fx["log_probability_hex"]], np.float32)
    np.testing.assert_array_equal(to_numpy(out.log_probability), lp)


# ---- full item lengths (BASELINE.json cfg4 T=2000, cfg5 T=3000, cfg3 under the
# peaky distribution B), against committed oracle outputs
# (tests/golden/make_fixtures_full.py): the large-C gather, the row's top set,
# the branch runs and the beam-256 loops over the whole length, where exact
# float ties between beams are the norm

FULL_PATH = os.path.join(os.path.dirname(__file__), "golden", "full_length.json")
FULL = json.load(open(FULL_PATH)) if os.path.exists(FULL_PATH) else {}


@pytest.mark.parametrize("name", sorted(FULL))
def test_full_length_golden(name):
    import hashlib
    import sys
    import torch
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    import make_fixtures_full
    fx = FULL[name]
    case = fx["case"]
    x, sl = make_fixtures_full.inputs(case)
    assert hashlib.sha256(x.tobytes()).hexdigest() == fx["sha256"], "input stream changed"
    _, _, T, B, C, W, P, merge, blank, blabel, _ = case
    out = ctcext_amd.ctc_ext_beam_search_decoder(
        torch.as_tensor(x, device="cuda"), torch.as_tensor(sl, device="cuda"),
        W, P, merge_repeated=merge, blank_index=blank, blank_label=blabel)
    di, dv, ds = oracle.pack_sparse(fx["decoded"], B, P)
    ai, av, ash = oracle.pack_sparse(fx["alignment"], B, P)
    lp = np.asarray([[float.fromhex(h) for h in row] for row in fx["log_probability_hex"]], np.float32)
    compare(out, oracle.OracleOutput(di, dv, ds, ai, av, ash, lp), P)


# ---- the global-state tier: beam state in HBM, 16-byte records, the literal
# path every frame (ctcx_decode.hip CTCX_GSTATE) -- the shapes the LDS tier
# cannot hold (num_classes > 65535 or past the LDS row, beams past the
# LDS-resident state), forced onto every random family by a testing flag

GS = _lib.CTCEXT_FLAG_GLOBAL_STATE


def _tier():
    return ctcext_amd.get_decoder(0).last_stats["tier"]


def test_global_state_tier_random_families():
    _run_random(7001, 60, flags=GS, device=True)
    assert _tier() == 1
    _run_random(7002, 40, flags=GS, ties=True)
    _run_random(7003, 15, flags=GS, T_max=30, B_max=2, C_min=65, C_max=300, W_max=100)
    _run_random(7004, 30, flags=GS, dtype=np.float64)
    _run_random(7005, 40, flags=GS, neg_inf=True)


def test_global_state_tier_duplicate_entries():
    for k, (x, sl, W, P, kw, ref, nd) in enumerate(_dup_family(31337, 15)):
        out, err = _gpu_or_error(x, sl, W, P, kw, flags=GS)
        assert err is None, (k, err)
        compare(out, ref, P)
        assert _dup_frames() == nd, (k, _dup_frames(), nd)


@pytest.mark.parametrize("T,B,C,W,P,merge,blank", [
    (12, 2, 70000, 8, 2, True, 0),        # num_classes past the 8-byte record (65535)
    (6, 1, 131072, 4, 1, False, 131071),  # ... and past any LDS row; blank last
    (40, 2, 8, 600, 3, True, 0),          # beams past the LDS-resident state
    (25, 2, 5, 1000, 2, False, 2),        # ... and past 512 (the 8-byte record's link)
])
def test_global_state_tier_shapes(T, B, C, W, P, merge, blank):
    rng = np.random.default_rng(T * 7 + C)
    x = rng.standard_normal((T, B, C)).astype(np.float32)
    sl = np.array([T, max(T - 3, 1)][:B], np.int32)
    kw = dict(merge_repeated=merge, blank_index=blank, blank_label=-1)
    ref = oracle.decode(x, sl, W, P, **kw)
    out, err = _gpu_or_error(x, sl, W, P, kw, device=True)
    assert err is None, err
    assert _tier() == 1
    compare(out, ref, P)


def test_lds_tier_is_used_within_its_limits():
    x = np.random.default_rng(1).standard_normal((10, 2, 29)).astype(np.float32)
    out, err = _gpu_or_error(x, np.array([10, 8], np.int32), 128, 2, dict(merge_repeated=True))
    assert err is None and _tier() == 0


# ---- beam-scorer hook (util/ctc_beam_scorer.h:31-65).  Parity unpinned: the
# reference op always runs BaseBeamScorer (kernels.cc:260), so the bigram
# scorer's only checker is the oracle's restatement of the hook call sites
# (decoder.h:103, 114, 171-182, 226).

def _bigram(rng, C, dtype, scale=2.0, sparse=False):
    tab = -np.abs(rng.standard_normal((C + 1, C))) * scale
    if sparse:   # mostly free transitions, a few penalised ones
        tab[rng.random(tab.shape) < 0.8] = 0.0
    return tab.astype(dtype)


def _run_scored(seed, n, dtype=np.float32, flags=0, device=False, **kw_case):
    rng = np.random.default_rng(seed)
    for it in range(n):
        x, sl, W, P, kw = random_case(rng, dtype=dtype, **kw_case)
        tab = _bigram(rng, x.shape[2], dtype, sparse=bool(it % 2))
        try:
            ref, rerr = oracle.decode(x, sl, W, P, scorer_table=tab, **kw), None
        except oracle.OracleError as e:
            ref, rerr = None, str(e)
        try:
            if device:
                import torch
                out = ctcext_amd.ctc_ext_beam_search_decoder(
                    torch.as_tensor(x, device="cuda"), torch.as_tensor(sl, device="cuda"), W, P,
                    flags=flags, scorer_table=torch.as_tensor(tab, device="cuda"), **kw)
            else:
                out = ctcext_amd.ctc_ext_beam_search_decoder(x, sl, W, P, flags=flags, scorer_table=tab, **kw)
            gerr = None
        except ctcext_amd.OpError as e:
            out, gerr = None, e.message
        assert rerr == gerr, (it, rerr, gerr)
        if ref is not None:
            compare(out, ref, P)


def test_scorer_random_small():
    _run_scored(6001, 120)
    _run_scored(6002, 60, ties=True)


def test_scorer_f64_literal_device():
    _run_scored(6003, 40, dtype=np.float64)
    _run_scored(6004, 30, flags=_lib.CTCEXT_FLAG_FORCE_LITERAL)
    _run_scored(6005, 20, device=True, T_max=80, C_max=30, W_max=40)


def test_scorer_large_c_and_neg_inf():
    # large C runs the skip scans, whose bounds need scores <= 0
    _run_scored(6006, 12, T_max=30, B_max=2, C_min=65, C_max=300, W_max=100, scale=4.0)
    _run_scored(6007, 30, neg_inf=True)


def test_scorer_global_state_tier():
    _run_scored(6009, 30, flags=GS)
    _run_scored(6010, 10, dtype=np.float64, flags=GS)


def test_scorer_zero_table_is_identity():
    rng = np.random.default_rng(6008)
    x = rng.standard_normal((200, 3, 29)).astype(np.float32)
    sl = np.array([200, 150, 199], np.int32)
    kw = dict(merge_repeated=True, blank_index=0, blank_label=-1)
    base = ctcext_amd.ctc_ext_beam_search_decoder(x, sl, 64, 3, **kw)
    zero = ctcext_amd.ctc_ext_beam_search_decoder(x, sl, 64, 3, scorer_table=np.zeros((30, 29), np.float32), **kw)
    compare(zero, oracle.decode(x, sl, 64, 3, **kw), 3)
    compare(base, oracle.decode(x, sl, 64, 3, **kw), 3)


def test_scorer_rejects_positive_scores():
    x = np.zeros((3, 1, 4), np.float32)
    tab = np.zeros((5, 4), np.float32)
    tab[2, 1] = 0.5
    with pytest.raises(ctcext_amd.InvalidArgumentError) as e:
        ctcext_amd.ctc_ext_beam_search_decoder(x, [3], 2, 1, scorer_table=tab)
    assert "log-probabilities" in e.value.message
    with pytest.raises(ValueError):
        ctcext_amd.ctc_ext_beam_search_decoder(x, [3], 2, 1, scorer_table=np.zeros((4, 4), np.float32))


# ---- the LDS record ring (CTCEXT_FLAG_RECORD_RING, ctcx_decode.hip
# ring_flush): only the records the traceback can reach are written to HBM,
# compacted and renumbered.  At its smallest size (8 frames) the random
# families flush several times per item.

RMIN = _lib.CTCEXT_FLAG_RING_MIN


def _stats():
    return ctcext_amd.get_decoder(0).last_stats


def test_record_ring_random_families():
    _run_random(8101, 80, flags=RMIN, device=True)
    assert _stats()["ring_frames"] == 8
    _run_random(8102, 60, flags=RMIN, ties=True)
    _run_random(8103, 40, flags=RMIN, neg_inf=True)
    _run_random(8104, 30, flags=RMIN, dtype=np.float64)
    _run_random(8105, 15, flags=RMIN, T_max=40, B_max=2, C_min=65, C_max=300, W_max=100)
    _run_random(8106, 20, flags=RMIN, T_max=60, W_min=100, W_max=256, C_max=8)


def test_record_ring_matches_direct_records():
    # cfg3's shape at full item length (ragged): the ring (128 frames at W=128:
    # six items, one per CU) and every record written to HBM give the same
    # outputs, and the ring writes fewer records
    rng = np.random.default_rng(77)
    T, B, C, W, P = 1500, 6, 29, 128, 3
    x = rng.standard_normal((T, B, C)).astype(np.float32)
    sl = np.array([1500, 1499, 33, 8, 1, 1200], np.int32)
    kw = dict(merge_repeated=True)
    a, err = _gpu_or_error(x, sl, W, P, kw, device=True, flags=_lib.CTCEXT_FLAG_RECORD_RING)
    assert err is None, err
    st = dict(_stats())
    b, err = _gpu_or_error(x, sl, W, P, kw, device=True, flags=_lib.CTCEXT_FLAG_NO_RING)
    assert err is None, err
    assert st["ring_frames"] == 128 and _stats()["ring_frames"] == 0
    full = _stats()["records_written"]
    # the score-table kernel's default is the ring
    _gpu_or_error(x, sl, W, P, kw, device=True)
    assert _stats()["ring_frames"] == 128 and _stats()["helper"] == 3
    assert 0 < st["records_written"] < full, (st["records_written"], full)
    for p in range(P):
        for name in ("decoded_indices", "decoded_values", "decoded_shape",
                     "alignment_indices", "alignment_values", "alignment_shape"):
            np.testing.assert_array_equal(to_numpy(getattr(a, name)[p]), to_numpy(getattr(b, name)[p]))
    np.testing.assert_array_equal(to_numpy(a.log_probability), to_numpy(b.log_probability))


# ---- the two-wave kernels (ctcx_decode.hip help_score_chunks, the score
# table: float, beams <= 128, C <= 64; help_gather_chunks, the gather queue:
# float, beams <= 256, C > 64) are the default for the base scorer, and every
# family above runs through them; the one-wave kernels stay the path for the
# other shapes and are forced here (CTCEXT_HELPER=0) on the same families


def test_helper_kernel_selection():
    rng = np.random.default_rng(3)
    x = rng.standard_normal((20, 2, 29)).astype(np.float32)
    ctcext_amd.ctc_ext_beam_search_decoder(x, [20, 20], 16, 1)
    assert _stats()["helper"] == 3 and _stats()["record_bytes"] == 4   # scored queue, small C
    x2 = rng.standard_normal((20, 2, 300)).astype(np.float32)
    ctcext_amd.ctc_ext_beam_search_decoder(x2, [20, 20], 100, 1)
    assert _stats()["helper"] == 3 and _stats()["record_bytes"] == 8   # scored queue, large C
    ctcext_amd.ctc_ext_beam_search_decoder(x2, [20, 20], 200, 1)
    assert _stats()["helper"] == 2 and _stats()["record_bytes"] == 8   # gather queue, beams > 128
    ctcext_amd.ctc_ext_beam_search_decoder(x[:, :, :20].copy(), [20, 20], 200, 1)
    assert _stats()["helper"] == 0   # small C, beams > 128: the one-wave kernel
    ctcext_amd.ctc_ext_beam_search_decoder(x.astype(np.float64), [20, 20], 16, 1)
    assert _stats()["helper"] == 0
    ctcext_amd.ctc_ext_beam_search_decoder(x, [20, 20], 300, 1)
    assert _stats()["helper"] == 0


@pytest.fixture
def one_wave(monkeypatch):
    monkeypatch.setenv("CTCEXT_HELPER", "0")


def test_one_wave_kernels_random_families(one_wave):
    _run_random(9101, 60)
    assert _stats()["helper"] == 0 and _stats()["record_bytes"] == 8
    _run_random(9102, 40, ties=True)
    _run_random(9103, 15, T_max=30, B_max=2, C_min=65, C_max=300, W_max=100)
    _run_random(9104, 30, flags=RMIN)
    _run_random(9105, 10, T_max=40, B_max=2, C_min=3, C_max=40, W_min=129, W_max=256)
    _run_random(9106, 8, T_max=30, B_max=2, C_min=65, C_max=500, W_min=129, W_max=256, ties=True)


# ---- the two-wave kernels' failure path (ctcx_decode.hip wait_expired,
# kCtlDead): a hand-over wait that runs out of time (~1 s of the 100 MHz
# clock) ends every later grow without reading the table or queue, and the
# host decodes the call again with the one-wave kernels -- or, with
# CTCEXT_FLAG_HELPER_STRICT, fails it.  CTCEXT_FLAG_TEST_HELPER_DEAD starts the
# helper out timed out, so both paths run without a real deadlock or a hang.

DEAD = _lib.CTCEXT_FLAG_TEST_HELPER_DEAD


# (shape, CTCEXT_HELPER): the C=29 shape under both of its two-wave kernels --
# the default scored queue (kind 3) and the score table (kind 1), whose dead
# path is its own (ctcx_decode.hip: `if (cx.tabdead) stop = true` before the
# window loop, the break after its wait)
TIMEOUT_CASES = [((300, 3, 29, 128, 3), ""), ((300, 3, 29, 128, 3), "1"),
                 ((120, 2, 1000, 64, 2), ""), ((60, 2, 700, 200, 1), "")]
TIMEOUT_IDS = ["c29-scored", "c29-table", "c1000", "c700-w200"]


@pytest.mark.parametrize("shape,hmode", TIMEOUT_CASES, ids=TIMEOUT_IDS)
def test_helper_timeout_strict_fails_cleanly(shape, hmode, monkeypatch):
    if hmode:
        monkeypatch.setenv("CTCEXT_HELPER", hmode)
    T, B, C, W, P = shape
    rng = np.random.default_rng(C + W)
    x = rng.standard_normal((T, B, C)).astype(np.float32)
    sl = np.full(B, T, np.int32)
    with pytest.raises(ctcext_amd.InternalError) as ei:
        ctcext_amd.ctc_ext_beam_search_decoder(x, sl, W, P, merge_repeated=True,
                                               flags=DEAD | _lib.CTCEXT_FLAG_HELPER_STRICT)
    assert ei.value.error_code == _lib.CTCEXT_INTERNAL
    assert "hand-over wait timed out" in str(ei.value)
    # the handle stays usable: the next call decodes normally
    out = ctcext_amd.ctc_ext_beam_search_decoder(x, sl, W, P, merge_repeated=True)
    compare(out, oracle.decode(x, sl, W, P, True), P)
    assert _stats()["helper"] == (1 if hmode == "1" else 2 if W > 128 else 3), _stats()
    assert _stats()["helper_redecodes"] == 0


@pytest.mark.parametrize("shape,hmode", TIMEOUT_CASES, ids=TIMEOUT_IDS)
def test_helper_timeout_redecodes_one_wave(shape, hmode, monkeypatch):
    if hmode:
        monkeypatch.setenv("CTCEXT_HELPER", hmode)
    T, B, C, W, P = shape
    rng = np.random.default_rng(C * W)
    x = rng.standard_normal((T, B, C)).astype(np.float32)
    sl = np.full(B, T, np.int32)
    # the re-decode is never silent: the op warns
    with pytest.warns(RuntimeWarning, match="hand-over wait timed out"):
        out = ctcext_amd.ctc_ext_beam_search_decoder(x, sl, W, P, merge_repeated=True, flags=DEAD)
    st = _stats()
    assert st["helper_redecodes"] == 1 and st["helper"] == 0, st
    compare(out, oracle.decode(x, sl, W, P, True), P)
