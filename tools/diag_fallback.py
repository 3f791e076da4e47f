"""Diagnostic: how often (and why) the fast path falls back to the literal model."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ctc-beam-search-op_amd"))
import numpy as np
import torch
import ctcext_amd
B, T, C, W, P = int(sys.argv[1]), int(sys.argv[2]), 29, int(sys.argv[3]), 3
x = torch.as_tensor(np.random.default_rng(20251015).standard_normal((T, B, C), dtype=np.float32), device="cuda")
sl = torch.full((B,), T, dtype=torch.int32, device="cuda")
out = ctcext_amd.ctc_ext_beam_search_decoder(x, sl, W, P, merge_repeated=True)
print(B, T, W, ctcext_amd.get_decoder(0).last_stats)
