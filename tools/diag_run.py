"""Diagnostic: one decode at a given shape (for rocprofv3 --pmc passes)."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ctc-beam-search-op_amd"))
import numpy as np
import torch
import ctcext_amd
B, T, W, P, C = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5]) if len(sys.argv) > 5 else 29
x = torch.as_tensor(np.random.default_rng(20251015).standard_normal((T, B, C), dtype=np.float32), device="cuda")
sl = torch.full((B,), T, dtype=torch.int32, device="cuda")
for _ in range(2):
    ctcext_amd.ctc_ext_beam_search_decoder(x, sl, W, P, merge_repeated=True)
torch.cuda.synchronize()
print("done")
