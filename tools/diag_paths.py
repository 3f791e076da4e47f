"""Diagnostic: exact path vs forced-literal vs oracle on a few cases."""
import json, os, sys
ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [os.path.join(ROOT, "ctc-beam-search-op_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import numpy as np
import ctcext_amd, oracle
from ctcext_amd import _lib
gold = json.load(open(os.path.join(ROOT, "tests", "golden", "paper_example.json")))
x = np.log(np.asarray(gold["probs"])).astype(np.float32)
cases = [(x, np.array([8], np.int32), 10, 5, dict(blank_index=0, blank_label=0, merge_repeated=False))]
rng = np.random.default_rng(3)
cases.append((rng.standard_normal((60, 2, 7)).astype(np.float32), np.array([60, 50], np.int32), 6, 2, dict(merge_repeated=True)))
cases.append((rng.standard_normal((60, 2, 29)).astype(np.float32), np.array([60, 60], np.int32), 16, 2, dict(merge_repeated=True)))
for ci, (xx, sl, W, P, kw) in enumerate(cases):
    ref = oracle.raw_decode(xx, sl, W, P, **kw)
    for flags in (0, _lib.CTCEXT_FLAG_FORCE_LITERAL):
        out = ctcext_amd.ctc_ext_beam_search_decoder(xx, sl, W, P, flags=flags, **kw)
        st = ctcext_amd.get_decoder(0).last_stats
        ok_lp = np.array_equal(out.log_probability, ref[2])
        ali = [[out.alignment_values[p][out.alignment_indices[p][:, 0] == b].tolist() for p in range(P)] for b in range(len(sl))]
        print(ci, "flags", flags, "lp_ok", ok_lp, "ali_ok", ali == ref[1], "literal", st["literal_frames"],
              "\n   got lp", out.log_probability.ravel()[:6], "\n   ref lp", ref[2].ravel()[:6])
