"""Diagnostic: the record-ring random families (tests/test_gpu_parity.py
test_record_ring_random_families) case by case, with the two-wave kernels on
and off (CTCEXT_HELPER), printing the first mismatching case of each family."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "ctc-beam-search-op_amd"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
import numpy as np

import ctcext_amd
from ctcext_amd import _lib
from parity_util import compare, oracle_or_error, random_case

FAM = [(8101, 80, {}), (8102, 60, dict(ties=True)), (8103, 40, dict(neg_inf=True)),
       (8104, 30, dict(dtype=np.float64)), (8105, 15, dict(T_max=40, B_max=2, C_min=65, C_max=300, W_max=100)),
       (8106, 20, dict(T_max=60, W_min=100, W_max=256, C_max=8))]
for helper in ("1", "0"):
    os.environ["CTCEXT_HELPER"] = helper
    for seed, n, kw_case in FAM:
        rng = np.random.default_rng(seed)
        bad = 0
        for it in range(n):
            x, sl, W, P, kw = random_case(rng, **kw_case)
            ref, rerr = oracle_or_error(x, sl, W, P, kw)
            try:
                out = ctcext_amd.ctc_ext_beam_search_decoder(x, sl, W, P, flags=_lib.CTCEXT_FLAG_RING_MIN, **kw)
                gerr = None
            except ctcext_amd.OpError as e:
                out, gerr = None, e.message
            st = ctcext_amd.get_decoder(0).last_stats
            ok = rerr == gerr
            if ok and ref is not None:
                try:
                    compare(out, ref, P)
                except AssertionError:
                    ok = False
                except ValueError:
                    ok = False
            if not ok:
                bad += 1
                if bad <= 2:
                    print("helper=%s seed %d case %d: T=%d B=%d C=%d W=%d P=%d sl=%s kw=%s helper_kind=%d ring=%d"
                          % (helper, seed, it, x.shape[0], x.shape[1], x.shape[2], W, P, list(sl), kw,
                             st["helper"], st["ring_frames"]), flush=True)
        print("helper=%s seed %d: %d/%d bad" % (helper, seed, bad, n), flush=True)
