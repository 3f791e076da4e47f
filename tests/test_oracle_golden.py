"""Pins the CPU oracle (test infrastructure) to the reference's only golden
vector: python/ops/ctc_ext_beam_search_decoder_ops_test.py:20-100."""
import json
import os

import numpy as np
import pytest

import oracle

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "paper_example.json")))


def _check(out):
    a = GOLD["attrs"]
    for p in range(a["top_paths"]):
        np.testing.assert_array_equal(out.decoded_indices[p], np.asarray(GOLD["decoded_indices"][p]))
        np.testing.assert_array_equal(out.decoded_values[p], np.asarray(GOLD["decoded_values"][p]))
        np.testing.assert_array_equal(out.decoded_shape[p], np.asarray(GOLD["decoded_shape"][p]))
        np.testing.assert_array_equal(out.alignment_indices[p], np.asarray(GOLD["alignment_indices"][p]))
        np.testing.assert_array_equal(out.alignment_values[p], np.asarray(GOLD["alignment_values"][p]))
        np.testing.assert_array_equal(out.alignment_shape[p], np.asarray(GOLD["alignment_shape"][p]))
    # the reference test's assertAllClose defaults
    np.testing.assert_allclose(out.log_probability, np.asarray(GOLD["log_probability"]), rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("mode", ["faithful", "shared"])
def test_oracle_reproduces_paper_golden(dtype, mode):
    a = GOLD["attrs"]
    logits = np.log(np.asarray(GOLD["probs"])).astype(dtype)
    out = oracle.decode(logits, GOLD["sequence_length"], a["beam_width"], a["top_paths"],
                        a["merge_repeated"], a["blank_index"], a["blank_label"], mode=mode)
    _check(out)


def test_oracle_modes_agree_random():
    rng = np.random.default_rng(7)
    for _ in range(40):
        T, B, C = rng.integers(1, 30), rng.integers(1, 4), rng.integers(2, 9)
        W = int(rng.integers(1, 12))
        P = int(rng.integers(1, W + 1))
        x = rng.standard_normal((T, B, C)).astype(np.float32)
        if rng.random() < 0.3:
            x = np.round(x * 2) / 2   # tie-heavy
        sl = rng.integers(T // 2, T + 1, size=B).astype(np.int32)
        kw = dict(merge_repeated=bool(rng.integers(2)), blank_index=int(rng.integers(C)),
                  blank_label=int(rng.integers(-1, C)))
        try:
            a = oracle.raw_decode(x, sl, W, P, mode="faithful", **kw)
        except oracle.OracleError as e:
            with pytest.raises(oracle.OracleError, match=str(e).split('.')[0]):
                oracle.raw_decode(x, sl, W, P, mode="shared", **kw)
            continue
        b = oracle.raw_decode(x, sl, W, P, mode="shared", **kw)
        assert a[0] == b[0] and a[1] == b[1]
        np.testing.assert_array_equal(a[2], b[2])


@pytest.mark.parametrize("family", ["plain", "ties", "neg_inf", "scorer", "large_c"])
def test_oracle_shared_reclaim_matches_faithful(family):
    """The shared mode's node economy (lazy child materialisation + reclamation
    of pristine unreachable nodes, ctc_oracle.cpp Decoder::reclaim) is cost
    only: with reclamation forced every frame it must equal the faithful
    (reference-shaped) mode exactly, including the -inf duplicate-entry state
    and the scorer hook."""
    from parity_util import random_case
    rng = np.random.default_rng({"plain": 11, "ties": 12, "neg_inf": 13, "scorer": 14, "large_c": 15}[family])
    n = 12 if family == "large_c" else 40
    for _ in range(n):
        if family == "large_c":
            x, sl, W, P, kw = random_case(rng, T_max=25, B_max=2, C_min=65, C_max=300, W_max=40)
        else:
            x, sl, W, P, kw = random_case(rng, T_max=40, ties=family == "ties", neg_inf=family == "neg_inf")
        tab = None
        if family == "scorer":
            tab = (-np.abs(rng.standard_normal((x.shape[2] + 1, x.shape[2]))) * 2).astype(x.dtype)
        res = []
        for mode, gc in (("faithful", 0), ("shared", 1), ("shared", 0)):
            st = {}
            try:
                r = oracle.raw_decode(x, sl, W, P, mode=mode, stats=st, scorer_table=tab, gc_threshold=gc, **kw)
                res.append((r[0], r[1], r[2].tobytes(), r[3], st["duplicate_frames"]))
            except oracle.OracleError as e:
                res.append(str(e))
        assert res[0] == res[1] == res[2]


def test_oracle_shared_reclaim_duplicate_state():
    """-inf-heavy single items that reach the duplicate-entry state (one
    BeamEntry twice in the beam, decoder.h:142 + :189-199): the reclaiming
    shared mode must agree with the faithful mode on those too."""
    rng = np.random.default_rng(31337)
    hits = 0
    for _ in range(3000):
        T = int(rng.integers(2, 30)); C = int(rng.integers(2, 8)); W = int(rng.integers(1, 10))
        x = rng.standard_normal((T, 1, C)).astype(np.float32)
        x[rng.random(x.shape) < (0.3 if rng.random() < 0.5 else 0.5)] = -np.inf
        P = int(rng.integers(1, W + 1))
        kw = dict(merge_repeated=bool(rng.integers(2)), blank_index=int(rng.integers(C)),
                  blank_label=int(rng.integers(-1, C)))
        st = {}
        try:
            a = oracle.raw_decode(x, [T], W, P, mode="faithful", stats=st, **kw)
        except oracle.OracleError:
            continue
        if not st["duplicate_frames"]:
            continue
        st2 = {}
        b = oracle.raw_decode(x, [T], W, P, mode="shared", stats=st2, gc_threshold=1, **kw)
        assert a[0] == b[0] and a[1] == b[1] and a[2].tobytes() == b[2].tobytes()
        assert st2["duplicate_frames"] == st["duplicate_frames"]
        hits += 1
        if hits == 30:
            break
    assert hits == 30


def test_oracle_errors():
    x = np.zeros((4, 1, 3), np.float32)
    with pytest.raises(oracle.OracleError, match="requested more paths than the beam width."):
        oracle.decode(x, [4], 2, 3)
    with pytest.raises(oracle.OracleError, match="Less leaves in the beam search than requested."):
        oracle.decode(x[:1], [1], 10, 5)
    with pytest.raises(oracle.OracleError, match="max_time is 0"):
        oracle.decode(np.zeros((0, 1, 3), np.float32), [0], 2, 1)
    with pytest.raises(oracle.OracleError, match=r"sequence_length\(0\) <= 4"):
        oracle.decode(x, [5], 2, 1)


def test_oracle_scorer_hook():
    """The bigram beam-scorer hook of the oracle (ctc_beam_scorer.h:31-65): an
    all-zero table is the identity (prev + 0 == prev), so it must reproduce the
    BaseBeamScorer decode exactly; a non-trivial table must change the search.
    (Parity unpinned: the reference op never exposes a scorer, kernels.cc:260.)"""
    rng = np.random.default_rng(9)
    x = rng.standard_normal((30, 2, 6)).astype(np.float32)
    sl = [30, 22]
    kw = dict(merge_repeated=True, blank_index=0, blank_label=-1)
    base = oracle.decode(x, sl, 8, 2, **kw)
    zero = oracle.decode(x, sl, 8, 2, scorer_table=np.zeros((7, 6), np.float32), **kw)
    for f in base._fields:
        for a, b in zip(getattr(base, f), getattr(zero, f)):
            np.testing.assert_array_equal(a, b)
    tab = -np.abs(rng.standard_normal((7, 6))).astype(np.float32) * 3
    lm = oracle.decode(x, sl, 8, 2, scorer_table=tab, **kw)
    assert not np.array_equal(lm.log_probability, base.log_probability)
    # the faithful (reference-cost) store agrees with the shared one under a scorer too
    lmf = oracle.decode(x, sl, 8, 2, scorer_table=tab, mode="faithful", **kw)
    for f in lm._fields:
        for a, b in zip(getattr(lm, f), getattr(lmf, f)):
            np.testing.assert_array_equal(a, b)


def test_bench_digest_fixture_reproduces():
    # tests/golden/bench_digests.json pins bench.py's outputs_match_oracle: the
    # oracle's outputs for the exact bench inputs, hashed by bench.output_digest.
    # Rank 0 of cfg2 (B=32, T=1000) recomputed here, in item shards as the
    # generator runs them (the items are independent, kernels.cc:68-90)
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import bench
    B, T, C, W, P, merge, blank = bench.CONFIGS["cfg2"]
    fx = json.load(open(os.path.join(root, "tests", "golden", "bench_digests.json")))["cfg2"]
    assert (fx["batch_per_gpu"], fx["seq_len"], fx["num_classes"], fx["beam_width"]) == (B, T, C, W)
    x = np.random.default_rng(20251015).standard_normal((T, B, C), dtype=np.float32)
    out = oracle.decode(x, np.full(B, T, np.int32), W, P, merge, blank, -1)
    assert bench.output_digest(out, P) == fx["digests"]["0"]
