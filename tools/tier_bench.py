"""Diagnostic: decode-kernel time of the global-state tier next to the LDS
tier, same shape otherwise (DESIGN.md "Two tiers").  Three lines:
  1. the LDS tier at beam_width W (default C=5000, W=256, B=64, T=100);
  2. the global-state tier forced on the same shape (CTCEXT_FLAG_GLOBAL_STATE),
     over the first T_gs frames (the literal path is slow; frames/s is the
     comparable figure);
  3. the shape just past the LDS tier's limit, beam_width =
     ctcext_max_beam_width(C, float) + 1, which the dispatcher itself sends to
     the global-state tier, over T_gs frames.
One JSON line per run.

    python tools/tier_bench.py [C T B W T_gs]
"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ctc-beam-search-op_amd"))
import numpy as np
import torch

import ctcext_amd
from ctcext_amd import _lib

C, T, B, W, T_GS = (int(a) for a in (sys.argv[1:6] if len(sys.argv) > 5 else (5000, 100, 64, 256, 10)))
g = torch.Generator(device="cuda")
g.manual_seed(20251015)
x = torch.randn((T, B, C), generator=g, device="cuda", dtype=torch.float32)
d = ctcext_amd.get_decoder(0)
w_max = int(_lib.load().ctcext_max_beam_width(C, _lib.CTCEXT_F32))
runs = (("lds", W, T, 0), ("global-state forced", W, T_GS, _lib.CTCEXT_FLAG_GLOBAL_STATE),
        ("past the LDS limit", w_max + 1, T_GS, 0))
for what, w, t, flags in runs:
    sl = torch.full((B,), t, dtype=torch.int32, device="cuda")
    xs = x[:t].contiguous()
    kms = []
    for rep in range(2):
        ctcext_amd.ctc_ext_beam_search_decoder(xs, sl, w, 1, flags=_lib.CTCEXT_FLAG_PROFILE | flags, outputs="device")
        torch.cuda.synchronize()
        st = d.last_stats
        if rep:
            kms.append(st["decode_kernel_ms"])
    print(json.dumps({"run": what, "C": C, "T": t, "B": B, "beam_width": w, "lds_tier_max_beam_width": w_max,
                      "tier": ["lds", "global-state"][st["tier"]], "helper": st["helper"],
                      "decode_kernel_ms": float(np.mean(kms)), "frames_per_s": B * t / (np.mean(kms) * 1e-3),
                      "literal_frames": st["literal_frames"]}), flush=True)
