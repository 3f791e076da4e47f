"""Diagnostic: decode-kernel time of the global-state tier just past the LDS
tier's limit, next to the LDS tier at the largest beam it holds, same shape
otherwise (DESIGN.md "Two tiers").  Default shape: C=5000, T=100, B=64,
W=256 (LDS tier) vs W=300 (global-state tier); one JSON line per run.

    python tools/tier_bench.py [C T B W_lds W_gs]
"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ctc-beam-search-op_amd"))
import numpy as np
import torch

import ctcext_amd
from ctcext_amd import _lib

C, T, B, W_LDS, W_GS = (int(a) for a in (sys.argv[1:6] if len(sys.argv) > 5 else (5000, 100, 64, 256, 300)))
g = torch.Generator(device="cuda")
g.manual_seed(20251015)
x = torch.randn((T, B, C), generator=g, device="cuda", dtype=torch.float32)
sl = torch.full((B,), T, dtype=torch.int32, device="cuda")
d = ctcext_amd.get_decoder(0)
for W in (W_LDS, W_GS):
    kms = []
    for rep in range(3):
        ctcext_amd.ctc_ext_beam_search_decoder(x, sl, W, 1, flags=_lib.CTCEXT_FLAG_PROFILE, outputs="device")
        torch.cuda.synchronize()
        st = d.last_stats
        if rep:
            kms.append(st["decode_kernel_ms"])
    print(json.dumps({"C": C, "T": T, "B": B, "beam_width": W, "tier": ["lds", "global-state"][st["tier"]],
                      "decode_kernel_ms": float(np.mean(kms)), "frames_per_s": B * T / (np.mean(kms) * 1e-3),
                      "literal_frames": st["literal_frames"]}), flush=True)
