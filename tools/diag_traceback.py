"""Diagnostic: the same decode with the segmented traceback (default) and the
one-thread-per-walk kernel (CTCEXT_TRACEBACK=0), outputs side by side, with
the call's stats (record format, ring)."""
import json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ctc-beam-search-op_amd"))
import numpy as np
import ctcext_amd

gold = json.load(open(os.path.join(ROOT, "tests", "golden", "paper_example.json")))
a = gold["attrs"]
x = np.log(np.asarray(gold["probs"])).astype(np.float32)
cases = [("paper", x, [8], a["beam_width"], a["top_paths"], dict(merge_repeated=a["merge_repeated"],
          blank_index=a["blank_index"], blank_label=a["blank_label"]))]
rng = np.random.default_rng(3)
cases.append(("cfg3-ish", rng.standard_normal((300, 3, 29)).astype(np.float32), [300, 300, 200], 128, 3,
              dict(merge_repeated=True)))
cases.append(("cfg4-ish", rng.standard_normal((100, 2, 1000)).astype(np.float32), [100, 90], 64, 1, {}))
for name, xx, sl, W, P, kw in cases:
    res = {}
    for mode in ("1", "0"):
        os.environ["CTCEXT_TRACEBACK"] = mode
        out = ctcext_amd.ctc_ext_beam_search_decoder(xx, sl, W, P, **kw)
        st = ctcext_amd.get_decoder(0).last_stats
        res[mode] = out
        print(name, "mode", mode, "stats", {k: st[k] for k in ("helper", "record_bytes", "ring_frames", "records_written", "tier")})
        for p in range(P):
            print("  p%d dec %s ali %s" % (p, out.decoded_values[p][:12].tolist(), out.alignment_values[p][:12].tolist()),
                  "lens", out.decoded_values[p].shape, out.alignment_values[p].shape)
    same = all(np.array_equal(res["1"][f][p], res["0"][f][p]) for f in range(6) for p in range(P))
    print(name, "identical:", same)
