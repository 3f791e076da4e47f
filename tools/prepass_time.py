"""Times the large-vocabulary pre-pass alone (ctcext_row_facts: the row facts
and the normaliser) at the GPU configs' shapes, N calls each, for rocprofv3
--kernel-trace --stats runs (kernel times) with CTCEXT_PREP_SPLIT=0 (fused,
one read of the logits) or 1 (facts + ctcx_row_norm, two reads).
usage: python tools/prepass_time.py [cfg4|cfg5|all] [calls]"""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ctc-beam-search-op_amd"))

import torch  # noqa: E402

import ctcext_amd  # noqa: E402
from ctcext_amd import _lib  # noqa: E402

# (T, B per GPU, C); cfg4 is one of 8 shards; c2k / c3k between them
SHAPES = {"cfg4": (2000, 128, 1000), "c2k": (2000, 128, 2048), "c3k": (2000, 128, 3000), "cfg5": (3000, 512, 5000)}


def main():
    which = sys.argv[1] if len(sys.argv) > 1 else "all"
    calls = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    d = ctcext_amd.get_decoder(0)
    lib = d.lib
    for name in (SHAPES if which == "all" else which.split(",")):
        T, B, C = SHAPES[name]
        g = torch.Generator(device="cuda").manual_seed(5)
        x = torch.randn((T, B, C), device="cuda", dtype=torch.float32, generator=g)
        sl = torch.full((B,), T, dtype=torch.int32, device="cuda")
        rb = ctypes.c_int64()
        assert lib.ctcext_row_facts(d.handle, None, _lib.CTCEXT_F32, T, B, C, 0, None, None, None,
                                    ctypes.byref(rb)) == 0
        prep = torch.empty(T * B * rb.value, dtype=torch.uint8, device="cuda")
        norm = torch.empty(T * B, dtype=torch.float32, device="cuda")
        ms = []
        for i in range(calls + 1):
            t0 = time.perf_counter()
            rc = lib.ctcext_row_facts(d.handle, ctypes.c_void_p(x.data_ptr()), _lib.CTCEXT_F32, T, B, C, 0,
                                      ctypes.c_void_p(sl.data_ptr()), ctypes.c_void_p(prep.data_ptr()),
                                      ctypes.c_void_p(norm.data_ptr()), ctypes.byref(rb))
            assert rc == 0, lib.ctcext_last_error()
            if i:
                ms.append((time.perf_counter() - t0) * 1e3)
        gb = x.numel() * 4 / 1e9
        print(f"{name} T={T} B={B} C={C} split={os.environ.get('CTCEXT_PREP_SPLIT', '0')} "
              f"logits {gb:.2f} GB wall ms/call min {min(ms):.3f} median {sorted(ms)[len(ms) // 2]:.3f} "
              f"norm[0..2] {norm[:3].tolist()}", flush=True)
        del x, prep, norm
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
