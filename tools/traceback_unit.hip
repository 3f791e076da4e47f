// Unit check of the traceback kernels (ctcx_traceback, ctcx_traceback_seg)
// on synthetic record streams: random chains in every record format (Rec32,
// Rec, Rec16), with and without the record ring's compacted frames, walked
// on the GPU through libctcext.so's launcher and compared with a host walk
// of the same records (the reference semantics: LabelSeq with merge_repeated,
// ctc_beam_entry.h:123-136; the alignment candidate chain, :137-152, 190-228).
// Build: hipcc --offload-arch=gfx950 -O2 -std=c++17 tools/traceback_unit.hip \
//          -Lctc-beam-search-op_amd/ctcext_amd/lib -lctcext -o tools/traceback_unit
// Run (GPU): LD_LIBRARY_PATH=ctc-beam-search-op_amd/ctcext_amd/lib tools/traceback_unit
//   (CTCEXT_TRACEBACK=0 selects the one-thread-per-walk kernel)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <random>
#include <vector>

#include "../ctc-beam-search-op_amd/csrc/ctcx_kernels.h"

namespace ctcx {
hipError_t launch_traceback(const TraceParams& tp, hipStream_t s);
}
using namespace ctcx;

#define CK(x)                                                                     \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(2);                                                                    \
    }                                                                             \
  } while (0)

struct R4 { uint32_t link; int lab; uint32_t bpb, bpn; };

static int run_case(int fmt, bool ring, int B, int T, int W, int P, int C, int merge, uint64_t seed) {
  std::mt19937_64 rng(seed);
  const int rb = fmt == kRecFmt128 ? 16 : fmt == kRecFmt32 ? 4 : 8;
  // per item: frame counts (ring: 1..W compacted records, else W), records
  std::vector<int32_t> sl(B), foff((size_t)B * T, 0);
  std::vector<std::vector<std::vector<R4>>> recs(B);
  std::vector<int32_t> top_pos((size_t)B * P), top_kind((size_t)B * P);
  std::vector<ItemOut> items(B);
  for (int b = 0; b < B; ++b) {
    sl[b] = (b % 5 == 4) ? 0 : (int)(T - (rng() % (T / 2 + 1)));
    int prevn = 1;
    recs[b].resize(sl[b]);
    std::vector<int> cnt(sl[b]);
    for (int t = 0; t < sl[b]; ++t) cnt[t] = ring ? 1 + (int)(rng() % W) : W;
    if (ring) {   // the ring's layout: flushes of 1..64 frames, each written newest frame first
      int64_t off = 0;
      for (int u_lo = 0; u_lo < sl[b];) {
        const int u_hi = std::min(sl[b] - 1, u_lo + (int)(rng() % 64));
        for (int u = u_hi; u >= u_lo; --u) {
          foff[(size_t)b * T + u] = (int32_t)off;
          off += cnt[u];
        }
        u_lo = u_hi + 1;
      }
    }
    for (int t = 0; t < sl[b]; ++t) {
      const int n = cnt[t];
      recs[b][t].resize(n);
      for (int k = 0; k < n; ++k) {
        R4& r = recs[b][t][k];
        r.link = ((uint32_t)(rng() % prevn) << 1) | (uint32_t)(rng() & 1);
        r.lab = (int)(rng() % (fmt == kRecFmt32 ? (C < 63 ? C : 63) : C));
        auto bp = [&]() -> uint32_t {
          const uint64_t u = rng() % 16;
          if (u == 0 || t == 0) return kBpRestart;
          return ((uint32_t)(rng() % prevn) << 1) | (uint32_t)(rng() & 1);
        };
        r.bpb = bp();
        r.bpn = bp();
      }
      prevn = n;
    }
    items[b] = ItemOut{};
    items[b].n_leaves = sl[b] > 0 ? P : 1;
    for (int p = 0; p < P; ++p) {
      top_pos[(size_t)b * P + p] = sl[b] > 0 ? (int)(rng() % prevn) : -1;
      top_kind[(size_t)b * P + p] = (int)(rng() % 3) - 1 >= 0 ? (int)(rng() & 1) : -1;
    }
  }
  // the record buffer: [B][T][W] records of rb bytes (ring: item b's stream at b * T * W)
  std::vector<uint8_t> rec((size_t)B * T * W * rb, 0xAB);
  for (int b = 0; b < B; ++b)
    for (int t = 0; t < sl[b]; ++t)
      for (size_t k = 0; k < recs[b][t].size(); ++k) {
        const R4& r = recs[b][t][k];
        const int64_t at = ring ? (int64_t)b * T * W + foff[(size_t)b * T + t] + (int64_t)k
                                : ((int64_t)b * T + t) * W + (int64_t)k;
        uint8_t* d = rec.data() + at * rb;
        if (fmt == kRecFmt32) {
          const uint32_t v = rec32_pack(r.link, r.lab, r.bpb, r.bpn);
          memcpy(d, &v, 4);
        } else if (fmt == kRecFmt64) {
          const Rec v = rec_pack(r.link, r.lab, r.bpb, r.bpn);
          memcpy(d, &v, 8);
        } else {
          const Rec16 v{r.link, r.lab, r.bpb, r.bpn};
          memcpy(d, &v, 16);
        }
      }
  // host walks (the reference semantics, as ctcx_traceback)
  std::vector<int32_t> want_seq((size_t)B * P * 2 * T, 0), want_len((size_t)P * 2 * B, 0);
  for (int b = 0; b < B; ++b)
    for (int p = 0; p < P; ++p)
      for (int which = 0; which < 2; ++which) {
        int len = 0, k = top_pos[(size_t)b * P + p];
        int32_t* out = want_seq.data() + (((size_t)b * P + p) * 2 + which) * T;
        if (sl[b] > 0 && k >= 0 && p < items[b].n_leaves) {
          if (which == 0) {
            int prev = -1;
            for (int t = sl[b] - 1; t >= 0; --t) {
              const R4& r = recs[b][t][k];
              if (r.link & 1u) {
                if (!merge || r.lab != prev) out[len++] = r.lab;
                prev = r.lab;
              }
              k = (int)(r.link >> 1);
            }
          } else {
            int kind = top_kind[(size_t)b * P + p];
            for (int t = sl[b] - 1; t >= 0 && kind >= 0; --t) {
              const R4& r = recs[b][t][k];
              out[len++] = kind == 0 ? -7 : r.lab;
              const uint32_t q = kind == 0 ? r.bpb : r.bpn;
              if (q >= kBpRestart) break;
              k = (int)(q >> 1);
              kind = (int)(q & 1u);
            }
          }
        }
        want_len[((size_t)p * 2 + which) * B + b] = len;
      }
  // device
  void *d_rec, *d_item, *d_sl, *d_tp, *d_tk, *d_foff, *d_seq, *d_len;
  CK(hipMalloc(&d_rec, rec.size()));
  CK(hipMalloc(&d_item, sizeof(ItemOut) * B));
  CK(hipMalloc(&d_sl, 4 * B));
  CK(hipMalloc(&d_tp, 4 * (size_t)B * P));
  CK(hipMalloc(&d_tk, 4 * (size_t)B * P));
  CK(hipMalloc(&d_foff, 4 * (size_t)B * T));
  CK(hipMalloc(&d_seq, 4 * (size_t)B * P * 2 * T));
  CK(hipMalloc(&d_len, 4 * (size_t)P * 2 * B));
  CK(hipMemcpy(d_rec, rec.data(), rec.size(), hipMemcpyHostToDevice));
  CK(hipMemcpy(d_item, items.data(), sizeof(ItemOut) * B, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_sl, sl.data(), 4 * B, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_tp, top_pos.data(), 4 * (size_t)B * P, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_tk, top_kind.data(), 4 * (size_t)B * P, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_foff, foff.data(), 4 * (size_t)B * T, hipMemcpyHostToDevice));
  CK(hipMemset(d_seq, 0, 4 * (size_t)B * P * 2 * T));
  CK(hipMemset(d_len, 0xFF, 4 * (size_t)P * 2 * B));
  TraceParams tp{};
  tp.rec = (const Rec*)d_rec; tp.item = (const ItemOut*)d_item; tp.seq_len = (const int32_t*)d_sl;
  tp.top_pos = (const int32_t*)d_tp; tp.top_kind = (const int32_t*)d_tk;
  tp.Tmax = T; tp.B = B; tp.W = W; tp.P = P; tp.merge = merge; tp.blank_label = -7;
  tp.rec_fmt = fmt; tp.foff = ring ? (const int32_t*)d_foff : nullptr;
  tp.seq = (int32_t*)d_seq; tp.len = (int32_t*)d_len; tp.len_stride = B;
  CK(launch_traceback(tp, nullptr));
  CK(hipDeviceSynchronize());
  std::vector<int32_t> got_seq(want_seq.size()), got_len(want_len.size());
  CK(hipMemcpy(got_seq.data(), d_seq, 4 * got_seq.size(), hipMemcpyDeviceToHost));
  CK(hipMemcpy(got_len.data(), d_len, 4 * got_len.size(), hipMemcpyDeviceToHost));
  int bad = 0;
  for (int b = 0; b < B && bad < 5; ++b)
    for (int p = 0; p < P; ++p)
      for (int which = 0; which < 2; ++which) {
        const int wl = want_len[((size_t)p * 2 + which) * B + b], gl = got_len[((size_t)p * 2 + which) * B + b];
        bool ok = wl == gl;
        const size_t o = (((size_t)b * P + p) * 2 + which) * T;
        for (int i = 0; ok && i < wl; ++i) ok = want_seq[o + i] == got_seq[o + i];
        if (!ok && bad++ < 5)
          fprintf(stderr, "  fmt %d ring %d: item %d path %d which %d: len %d want %d\n", fmt, ring, b, p, which, gl, wl);
      }
  hipFree(d_rec); hipFree(d_item); hipFree(d_sl); hipFree(d_tp); hipFree(d_tk); hipFree(d_foff); hipFree(d_seq);
  hipFree(d_len);
  return bad;
}

int main() {
  int fails = 0, n = 0;
  struct Shape { int B, T, W, P, C; };
  const Shape shapes[] = {{1, 8, 10, 5, 3}, {7, 300, 128, 3, 29}, {5, 700, 64, 1, 1000}, {3, 120, 256, 2, 5000},
                          {4, 2100, 16, 4, 40}, {2, 50, 1, 1, 2}, {3, 90, 33, 128, 7}};
  for (const Shape& s : shapes)
    for (int fmt : {kRecFmt32, kRecFmt64, kRecFmt128})
      for (int ring = 0; ring < 2; ++ring)
        for (int merge = 0; merge < 2; ++merge) {
          if (fmt == kRecFmt32 && (s.W > 128)) continue;   // Rec32: beams <= 128
          if (fmt == kRecFmt128 && ring) continue;          // the global-state tier writes every record
          const int bad = run_case(fmt, ring != 0, s.B, s.T, s.W, s.P, s.C, merge, 1000u * n + 17u);
          ++n;
          if (bad) {
            ++fails;
            printf("FAIL B=%d T=%d W=%d P=%d fmt=%d ring=%d merge=%d\n", s.B, s.T, s.W, s.P, fmt, ring, merge);
          }
        }
  printf("traceback unit: %d cases, %d failed (%s kernel)\n", n, fails,
         getenv("CTCEXT_TRACEBACK") && getenv("CTCEXT_TRACEBACK")[0] == '0' ? "one-thread" : "default");
  return fails ? 1 : 0;
}
