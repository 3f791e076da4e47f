"""The two-wave kernels' hand-over forms, each against the oracle on the same
families (ctcx_decode.hip): CTCEXT_HELPER=1 runs the score table (C <= 64,
beams <= 128) and the unscored gather queue (C > 64); CTCEXT_HELPER=3 the
scored gather queue (help_gather_scored: beams <= 128 at any C, beams of
129..256 at C > 64), where the
helper gathers and scores the offers that can matter against a stale bottom
and wave 0 pushes them.  Whichever form is the default, the other stays
covered here; the one-wave kernels are test_gpu_parity.py's CTCEXT_HELPER=0.
"""
import hashlib
import os
import sys

import numpy as np
import pytest

import ctcext_amd
import oracle
from parity_util import compare
from test_gpu_parity import FULL, RMIN, _run_random

pytestmark = pytest.mark.gpu

# mode -> CTCEXT_HELPER; the kind a float base-scorer shape then runs
MODES = {"legacy": "1", "scored": "3", "scored_wide": "4"}


def _kind(mode, W, C):
    if mode != "legacy" and W <= 128:
        return 3
    if mode == "scored_wide" and W <= 256 and C > 64:
        return 3
    if C <= 64:
        return 1 if W <= 128 else 0
    return 2 if W <= 256 else 0


@pytest.fixture(params=sorted(MODES))
def mode(request, monkeypatch):
    monkeypatch.setenv("CTCEXT_HELPER", MODES[request.param])
    return request.param


def _check_kind(mode, W, C):
    assert _stats()["helper"] == _kind(mode, W, C), (mode, W, C, _stats()["helper"])


def _probe(mode, W, C):
    # one decode of a shape the family covers, to check which kernel the mode ran
    x = np.random.default_rng(W + C).standard_normal((20, 2, C)).astype(np.float32)
    ctcext_amd.ctc_ext_beam_search_decoder(x, [20, 20], W, 1)
    _check_kind(mode, W, C)


def _stats():
    return ctcext_amd.get_decoder(0).last_stats


def test_helper_mode_random_small_c(mode):
    _probe(mode, 100, 29)
    _run_random(9301, 60, W_max=120)
    _run_random(9302, 50, ties=True, W_max=120)
    _run_random(9303, 30, neg_inf=True)
    _run_random(9304, 20, flags=RMIN)
    _run_random(9305, 20, T_max=50, W_min=60, W_max=128, C_max=40)
    # frequent evictions of branches, re-offers, deactivations and turns that
    # close mid-chunk
    _run_random(9306, 120, T_max=60, B_max=3, C_max=6, W_max=10, ties=True)


def test_helper_mode_random_large_c(mode):
    _probe(mode, 100, 300)
    _run_random(9311, 20, T_max=40, B_max=2, C_min=65, C_max=400, W_max=128, scale=4.0)
    _run_random(9312, 20, T_max=40, B_max=2, C_min=65, C_max=300, W_max=8, ties=True)
    _run_random(9313, 12, T_max=30, B_max=2, C_min=65, C_max=130, W_min=60, W_max=128, scale=1.5)
    _run_random(9314, 10, T_max=30, B_max=2, C_min=100, C_max=400, W_min=20, W_max=128, ties=True)
    _run_random(9315, 8, T_max=30, B_max=2, C_min=66, C_max=200, W_min=60, W_max=128, scale=0.3)
    _run_random(9316, 4, T_max=16, B_max=2, C_min=2049, C_max=2400, W_min=20, W_max=128, ties=True)


def test_helper_mode_random_large_c_wide(mode):
    # beams of 129..256 at large C: the scored queue's one-slot form (the RN=2
    # heap), or the unscored queue four ahead
    _probe(mode, 200, 300)
    _run_random(9321, 12, T_max=30, B_max=2, C_min=65, C_max=600, W_min=129, W_max=256)
    _run_random(9322, 10, T_max=30, B_max=2, C_min=65, C_max=400, W_min=129, W_max=256, ties=True)
    _run_random(9323, 8, T_max=30, B_max=2, C_min=66, C_max=200, W_min=129, W_max=256, scale=0.3)
    _run_random(9324, 6, T_max=40, B_max=2, C_min=300, C_max=1200, W_min=129, W_max=256, scale=2.5)
    _run_random(9325, 4, T_max=16, B_max=2, C_min=2049, C_max=3000, W_min=129, W_max=256, ties=True)


@pytest.mark.parametrize("name", sorted(FULL))
def test_helper_mode_full_length_golden(name, mode):
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
    _check_kind(mode, W, C)
    di, dv, ds = oracle.pack_sparse(fx["decoded"], B, P)
    ai, av, ash = oracle.pack_sparse(fx["alignment"], B, P)
    lp = np.asarray([[float.fromhex(h) for h in row] for row in fx["log_probability_hex"]], np.float32)
    compare(out, oracle.OracleOutput(di, dv, ds, ai, av, ash, lp), P)


def test_helper_mode_cfg3_shape(mode):
    # cfg3's attributes at a length the live oracle finishes quickly
    rng = np.random.default_rng(4242)
    T, B, C, W, P = 400, 4, 29, 128, 3
    x = rng.standard_normal((T, B, C)).astype(np.float32)
    sl = np.array([400, 399, 250, 17], np.int32)
    out = ctcext_amd.ctc_ext_beam_search_decoder(x, sl, W, P, merge_repeated=True)
    _check_kind(mode, W, C)
    compare(out, oracle.decode(x, sl, W, P, True), P)
