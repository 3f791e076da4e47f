"""Diagnostic: per-phase cycle split of ctcx_beam_decode (s_memtime stamps).

Needs the counters build (the product library compiles them out):
  make -C ctc-beam-search-op_amd/csrc phases
  CTCEXT_LIB_PATH=$PWD/tools/libctcext_phases.so python tools/diag_phases.py B T W P [C]
(add -DCTCX_FASTLOOP_PROF to the phases build for the per-event split)."""
import ctypes, os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ctc-beam-search-op_amd"))
import numpy as np
import torch
import ctcext_amd
from ctcext_amd import _lib
B, T, W, P, C = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5]) if len(sys.argv) > 5 else 29
x = torch.as_tensor(np.random.default_rng(20251015).standard_normal((T, B, C), dtype=np.float32), device="cuda")
sl = torch.full((B,), T, dtype=torch.int32, device="cuda")
f = _lib.CTCEXT_FLAG_PHASES | _lib.CTCEXT_FLAG_PROFILE
ctcext_amd.ctc_ext_beam_search_decoder(x, sl, W, P, merge_repeated=True, flags=f)
out = ctcext_amd.ctc_ext_beam_search_decoder(x, sl, W, P, merge_repeated=True, flags=f)
d = ctcext_amd.get_decoder(0)
NPH = 32   # ctcx_kernels.h kPhaseN: [0, 24) wave 0, [24, 32) the helper wave
buf = np.zeros((B, NPH), np.uint64)
rc = d.lib.ctcext_phase_counters(d.handle, ctypes.c_void_p(buf.ctypes.data), B * NPH)
if rc != 0:
    sys.exit("ctcext_phase_counters failed (%d): %s" % (rc, d.lib.ctcext_last_error().decode()))
m = buf.astype(np.float64).mean(0)
fr = m[7]
names = ["rowload", "recursion", "grow", "extract", "commit", "literal", "heap events", "frames",
         "scoring", "eventloop", "score:pre-skip", "chunks", "asm calls", "asm loop", "makeheap", "flush",
         "gather (C>64)", "gather: window steps | C<=64: child-walk steps", "gather: windows | C<=64: child walk",
         "gather: top set",
         "gather: branch select", "gather: branches", "gather: S branches", "gather: select+S test+S hot"]
CYC = {0, 1, 2, 3, 4, 5, 8, 9, 10, 13, 14, 15, 16, 18, 19, 20, 23}
print("B=%d T=%d W=%d P=%d C=%d decode_ms=%.1f" % (B, T, W, P, C, d.last_stats["decode_kernel_ms"]))
for k in range(24):
    if k == 7:
        continue
    print("  %-10s %12.0f %s/frame" % (names[k], m[k] / fr, "cycles" if k in CYC else "count"))
if m[6] > 0:
    print("  asm loop cycles per push (incl. entry/exit): %.0f" % (m[13] / m[6]))
# per item: the kernel ends with its slowest item (one wave per item)
tot = buf[:, [0, 1, 2, 3, 4, 5]].astype(np.float64).sum(1)
o = np.argsort(tot)
print("  per-item cycles/frame: min %.0f mean %.0f max %.0f (items %s slowest)" % (
    tot.min() / fr, tot.mean() / fr, tot.max() / fr, list(o[-4:][::-1])))
for b in o[-3:][::-1]:
    print("    item %d: heap events %.0f/frame, extract %.0f, grow %.0f, eventloop %.0f, scoring %.0f" % (
        b, buf[b, 6] / fr, buf[b, 3] / fr, buf[b, 2] / fr, buf[b, 9] / fr, buf[b, 8] / fr))
print("  mean heap events/frame %.1f, max %.1f" % (buf[:, 6].mean() / fr, buf[:, 6].max() / fr))
# two-wave kernels (cfg2/cfg3 class): the score-table wait and where the waves ran
if True:
    print("  HW table / queue wait %.0f cycles/frame, %.2f s_sleep rounds/frame (first chunk: %.0f cycles)"
          % (m[19] / fr, m[20] / fr, m[14] / fr))
    w0, w1 = buf[:, 21].astype(np.int64), buf[:, 22].astype(np.int64)
    simd0, simd1 = (w0 >> 4) & 3, (w1 >> 4) & 3
    cu0, cu1 = (w0 >> 8) & 15, (w1 >> 8) & 15
    same_cu = (cu0 == cu1) & (((w0 >> 13) & 3) == ((w1 >> 13) & 3)) & (((w0 >> 12) & 1) == ((w1 >> 12) & 1))
    print("  HW waves: same CU %d/%d items, same SIMD %d/%d items (wave0 SIMD histogram %s, helper %s)" % (
        int(same_cu.sum()), B, int((same_cu & (simd0 == simd1)).sum()), B,
        np.bincount(simd0, minlength=4).tolist(), np.bincount(simd1, minlength=4).tolist()))
# the helper wave (two-wave scored-queue kernels; 0 where it does not run)
hn = {24: "helper gather (whole)", 25: "helper to first chunk", 26: "helper waits for wave 0",
      28: "helper rank extract", 29: "helper ring flush"}
for k, name in hn.items():
    print("  %-26s %10.0f cycles/frame" % (name, m[k] / fr))
print("  helper chunks %.2f/frame, scan steps %.2f/frame, child-walk steps %.2f/frame"
      % (m[30] / fr, m[31] / fr, m[27] / fr))
if os.environ.get("CTCX_DIAG_EXTP"):   # (a build with -DCTCX_PHASE_EXTP: the extract's stop)
    h = buf[:, 27].astype(np.uint64)
    cnt = [int(((h >> np.uint64(16 * k)) & np.uint64(0xFFFF)).sum()) for k in range(4)]
    nf = max(1, sum(cnt))
    print("  (raw helper words, items 0-3: %s)" % [hex(int(v)) for v in h[:4]])
    print("  extract stop (helper): p<=2 %.3f, 3..63 %.3f, 64..95 %.3f, 96..128 %.3f of %d frames" % (
        cnt[0] / nf, cnt[1] / nf, cnt[2] / nf, cnt[3] / nf, nf))
    print("  extract: wave 0's stop mean %.1f, frames with a helper stop %.3f, pops %.1f per frame" % (
        m[16] / fr, m[17] / fr, m[18] / fr))
if os.environ.get("CTCX_DIAG_TIES"):   # (a build with -DCTCX_PHASE_TIES: the first tied pair at rank p)
    nt = max(1.0, m[25])
    print("  ties (two new children, one label): %.3f of frames; parents: label = child's (sum of 2) %.3f,"
          " one the other's parent %.3f, siblings %.3f, same label %.3f, equal totals %.3f, blank = other's total %.3f"
          % (m[25] / fr, m[29] / nt, m[30] / nt, m[27] / nt, m[26] / nt, m[24] / nt, m[31] / nt))
if os.environ.get("CTCX_DIAG_EXTT"):   # (a build with -DCTCX_PHASE_EXTT: when the helper's stop lands)
    print("  extract: helper stop published in %.3f of frames, %.0f cycles after wave 0's extract start;"
          " asm segments %.2f per frame, %.1f pops, %.0f cycles in them (%.0f per pop), extract phase %.0f"
          % (m[26] / fr, m[25] / max(1.0, m[26]), m[17] / fr, m[18] / fr, m[23] / fr, m[23] / max(1.0, m[18]), m[3] / fr))
if os.environ.get("CTCX_DIAG_EXTT"):
    print("  helper: kCtlDone seen %.0f cycles after wave 0's extract start (all frames it ranks), rank to publish %.0f"
          % (m[24] / max(1.0, m[26]), m[27] / max(1.0, m[26])))
if os.environ.get("CTCX_DIAG_BIRTH"):   # (a build with -DCTCX_PHASE_BIRTH)
    print("  ties: frames ending without a tie %.3f; after such a frame, frames ending with one %.4f (of %.0f per item)"
          % (m[28] / fr, m[31] / max(1.0, m[30]), m[30]))
if os.environ.get("CTCX_DIAG_SET"):   # (a build with -DCTCX_PHASE_SET -DCTCX_SET_MODE=1)
    print("  set mode: frames tried %.3f, replayed on the heap %.4f (of frames); set pushes %.1f per frame, %.0f cycles"
          " each (in the set loop)" % (m[16] / fr, m[17] / fr, m[18] / fr, m[23] / max(1.0, m[18])))

