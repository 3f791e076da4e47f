"""Extended GPU parity sweep (diagnostic, beyond the pytest suite): many seeded
random cases per family, HIP decoder through the C ABI vs the oracle (shared
mode), bit-exact decoded/alignment/shapes and log-probabilities.  Prints one
line per family and a total; exits non-zero on the first mismatch.
usage: python tools/parity_sweep.py [cases_per_family]"""
import os
import sys
import time

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
for p in ("ctc-beam-search-op_amd", "oracle", "tests"):
    sys.path.insert(0, os.path.join(ROOT, p))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import ctcext_amd  # noqa: E402
from parity_util import compare, oracle_or_error, random_case  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 40
FAMILIES = {
    # name: (seed, random_case kwargs)
    "small_mixed": (5001, dict()),
    "small_ties": (5002, dict(ties=True)),
    "cfg3_like_w128": (5003, dict(T_max=80, B_max=2, C_min=20, C_max=40, W_min=100, W_max=128)),
    "wide_w129_256": (5004, dict(T_max=40, B_max=2, C_min=3, C_max=40, W_min=129, W_max=256)),
    "wide_ties": (5005, dict(T_max=40, B_max=2, C_min=3, C_max=30, W_min=129, W_max=256, ties=True)),
    "large_c": (5006, dict(T_max=30, B_max=2, C_min=65, C_max=800, W_min=16, W_max=128)),
    "large_c_wide": (5007, dict(T_max=25, B_max=2, C_min=65, C_max=600, W_min=129, W_max=256)),
    "large_c_peaked": (5008, dict(T_max=30, B_max=2, C_min=65, C_max=1500, W_min=8, W_max=200, scale=3.0)),
    "large_c_ties": (5009, dict(T_max=30, B_max=2, C_min=65, C_max=400, W_min=8, W_max=256, ties=True)),
    "neg_inf": (5010, dict(T_max=30, B_max=3, C_max=20, W_max=40, neg_inf=True)),
    "f64_mixed": (5011, dict(T_max=30, B_max=2, C_max=200, W_max=150, dtype=np.float64)),
    # round 3: C above 2048 (pre-pass rows, compacted gather), and the
    # global-state tier forced onto small mixed cases
    "large_c_2k": (5012, dict(T_max=14, B_max=2, C_min=2049, C_max=3000, W_min=32, W_max=256)),
    "gstate_mixed": (5013, dict(T_max=30, B_max=2, C_max=80, W_max=60, flags="gstate")),
    # round 4: the global-state tier's early rejection of new children (beam
    # full, larger C, ties deciding the bottom)
    "gstate_large_c": (5014, dict(T_max=15, B_max=2, C_min=65, C_max=600, W_min=4, W_max=64, flags="gstate")),
    "gstate_ties": (5015, dict(T_max=20, B_max=2, C_max=40, W_max=48, ties=True, flags="gstate")),
    # round 5: the scored gather queue (beams <= 128, any C): re-offers,
    # deactivations and turns closing inside compacted chunks, ties deciding
    # the bottom the helper gathers against
    "sq_reoffer": (5016, dict(T_max=60, B_max=3, C_max=6, W_max=12, ties=True)),
    "sq_cfg3_ties": (5017, dict(T_max=80, B_max=2, C_min=20, C_max=40, W_min=60, W_max=128, ties=True)),
    "sq_large_c_ties": (5018, dict(T_max=30, B_max=2, C_min=65, C_max=600, W_min=8, W_max=128, ties=True)),
}
total = 0
t0 = time.time()
for name, (seed, kw) in FAMILIES.items():
    kw = dict(kw)
    flags = ctcext_amd._lib.CTCEXT_FLAG_GLOBAL_STATE if kw.pop("flags", None) == "gstate" else 0
    rng = np.random.default_rng(seed)
    n_err = 0
    for it in range(N):
        x, sl, W, P, akw = random_case(rng, **kw)
        ref, rerr = oracle_or_error(x, sl, W, P, akw)
        dev = it % 2 == 1   # alternate device and host inputs
        try:
            xin = torch.as_tensor(x, device="cuda:0") if dev else x
            slin = torch.as_tensor(sl, device="cuda:0") if dev else sl
            out = ctcext_amd.ctc_ext_beam_search_decoder(xin, slin, W, P, flags=flags, **akw)
            torch.cuda.synchronize()
            gerr = None
        except ctcext_amd.OpError as e:   # the op's InvalidArgument / FailedPrecondition
            out, gerr = None, e.message
        assert rerr == gerr, (name, it, rerr, gerr)
        if ref is not None:
            compare(out, ref, P)
        else:
            n_err += 1
    total += N
    print("%-16s %4d cases bit-exact (%d error cases matched)  %.0f s" % (name, N, n_err, time.time() - t0), flush=True)
print("total %d cases, all bit-exact" % total, flush=True)
