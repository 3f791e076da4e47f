"""Diagnostic: where the host-I/O path's extra time goes at cfg3 (bench.py host_io)."""
import os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ctc-beam-search-op_amd"))
import numpy as np, torch, ctcext_amd
B, T, C, W, P = 256, 1500, 29, 128, 3
x_np = np.random.default_rng(20251015).standard_normal((T, B, C), dtype=np.float32)
sl_np = np.full(B, T, np.int32)
x = torch.as_tensor(x_np, device="cuda"); sl = torch.as_tensor(sl_np, device="cuda")
def tm(f, n=2):
    f(); torch.cuda.synchronize(); t = time.perf_counter()
    for _ in range(n): f()
    torch.cuda.synchronize(); return 1e3 * (time.perf_counter() - t) / n
dev = lambda: ctcext_amd.ctc_ext_beam_search_decoder(x, sl, W, P, merge_repeated=True)
host = lambda: ctcext_amd.ctc_ext_beam_search_decoder(x_np, sl_np, W, P, merge_repeated=True)
out = dev()
tot = sum(t.numel() * 8 for f in (out.decoded_indices, out.decoded_values, out.alignment_indices, out.alignment_values) for t in f)
print("device path ms %.1f" % tm(dev))
print("host path ms %.1f" % tm(host))
print("torch H2D pageable %.1f MB ms %.2f" % (x_np.nbytes / 1e6, tm(lambda: torch.as_tensor(x_np, device="cuda"))))
print("torch D2H outputs %.1f MB ms %.2f" % (tot / 1e6, tm(lambda: [t.cpu() for f in (out.decoded_indices, out.decoded_values, out.alignment_indices, out.alignment_values) for t in f])))
# split of the host path: decode (upload + kernels + sizes) vs fetch (downloads)
d = ctcext_amd.get_decoder(0)
cls = type(d)
acc = {"decode": 0.0, "fetch": 0.0}
for name in ("decode", "fetch"):
    orig = getattr(cls, name)
    def wrap(self, *a, _o=orig, _n=name, **k):
        t = time.perf_counter(); r = _o(self, *a, **k); acc[_n] += time.perf_counter() - t; return r
    setattr(cls, name, wrap)
host(); acc.update(decode=0.0, fetch=0.0); host(); print("host split ms", {k: round(1e3 * v, 1) for k, v in acc.items()})
acc.update(decode=0.0, fetch=0.0); dev(); torch.cuda.synchronize(); print("device split ms", {k: round(1e3 * v, 1) for k, v in acc.items()})
