"""Diagnostic for the scored-queue check build (-DCTCX_SQ_CHECK): one item of
a random parity case, the first lane whose scored fields differ from wave 0's
recomputation (fields mask: 1 score, 2 branch total, 4 branch child, 8/16
candidate value/back-pointer).  usage: CTCEXT_LIB_PATH=ab/libsqchk.so
CTCEXT_HELPER=3 python tools/diag_sq_check.py SEED IT ITEM T [kwargs]"""
import os
import struct
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(R, "tests"), os.path.join(R, "oracle"), os.path.join(R, "ctc-beam-search-op_amd")]
import numpy as np  # noqa: E402

import ctcext_amd  # noqa: E402
from parity_util import random_case  # noqa: E402

seed, it, item, T = (int(a) for a in sys.argv[1:5])
kw_case = {k: (float(v) if "." in v else int(v)) for k, v in (a.split("=") for a in sys.argv[5:])}
rng = np.random.default_rng(seed)
for _ in range(it + 1):
    x, sl, W, P, kw = random_case(rng, **kw_case)
x = np.ascontiguousarray(x[:T, item:item + 1])
sl = np.minimum(sl[item:item + 1], T).astype(np.int32)
out = ctcext_amd.ctc_ext_beam_search_decoder(x, sl, W, 1, **kw)
st = ctcext_amd.get_decoder(0).last_stats
f = lambda u: struct.unpack("f", struct.pack("I", u & 0xffffffff))[0]
fm, wf, rec, s2 = st["literal_nonfinite"], st["literal_fill"], st["records_written"], st["literal_frames"]
print("x", x.shape, "W", W, kw)
print("fields %d  c(slot) %d c(recomputed) %d  lane %d chunk %d cqn %d  branch %d label %d  bt(slot) %r bt(recomputed) %r bt(slot re-read) %r"
      % (fm & 255, ((fm >> 8) & 255) - 1, ((fm >> 16) & 255) - 1, wf & 255, (wf >> 8) & 255, wf >> 16,
         (rec >> 32) & 0xffff, (rec >> 48) & 0xffff, f(rec), f(s2), f(st["duplicate_frames"])))
print("the other buffer's total of that branch:", float(np.asarray(out.log_probability)[0, 0]))
