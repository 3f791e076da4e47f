"""Diagnostic: the first frame where the GPU decode and the oracle differ on
one random parity case (tests/parity_util.random_case), by decoding growing
prefixes with top_paths = beam_width (the whole beam's totals compared).
usage: python tools/diag_first_divergence.py SEED IT [random_case kwargs as k=v ...]"""
import os
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(R, "tests"), os.path.join(R, "oracle"), os.path.join(R, "ctc-beam-search-op_amd")]
import numpy as np  # noqa: E402

import ctcext_amd  # noqa: E402
import oracle  # noqa: E402
from parity_util import random_case  # noqa: E402

seed, it = int(sys.argv[1]), int(sys.argv[2])
kw_case = {k: (float(v) if "." in v else int(v)) for k, v in (a.split("=") for a in sys.argv[3:])}
rng = np.random.default_rng(seed)
for _ in range(it + 1):
    x, sl, W, P, kw = random_case(rng, **kw_case)
print("case", x.shape, list(sl), "W", W, "P", P, kw, flush=True)
T = x.shape[0]
for t in range(1, T + 1):
    s2 = np.minimum(sl, t).astype(np.int32)
    try:
        ref = oracle.decode(x[:t], s2, W, W, kw["merge_repeated"], kw["blank_index"], kw["blank_label"])
    except oracle.OracleError as e:
        continue
    out = ctcext_amd.ctc_ext_beam_search_decoder(x[:t], s2, W, W, **kw)
    st = ctcext_amd.get_decoder(0).last_stats
    a, b = np.asarray(out.log_probability), np.asarray(ref.log_probability)
    if not np.array_equal(a, b):
        for bi in range(a.shape[0]):
            if not np.array_equal(a[bi], b[bi]):
                d = np.nonzero(a[bi] != b[bi])[0]
                print("frame %d item %d (seq_len %d): first differing position %d of %d; helper %d literal_frames %d"
                      % (t, bi, s2[bi], d[0], W, st["helper"], st["literal_frames"]))
                print("  gpu   ", a[bi][max(d[0] - 2, 0):d[0] + 6].tolist())
                print("  oracle", b[bi][max(d[0] - 2, 0):d[0] + 6].tolist())
        break
else:
    print("no divergence")
print("stats of the last call:", {k: v for k, v in ctcext_amd.get_decoder(0).last_stats.items()
                                  if k in ("helper", "duplicate_frames", "literal_frames")})
