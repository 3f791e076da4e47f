// pop_probe.hip — where the cycles of one TopN sift go (one wave, W = 128):
// variants of the decode kernel's adjust step timed over a full sort_heap.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off tools/pop_probe.hip -o tools/pop_probe.bin
#include <hip/hip_runtime.h>

#include <cstdio>
#include <random>
#include <vector>

#include "../ctc-beam-search-op_amd/csrc/ctcx_decode.hip"

using namespace ctcx;

// MODE 0: as the decode kernel; 1: no chase (pf = 0); 2: chase, no stores;
// 3: branch-free unrolled chase; 4: prologue only (loads + ballots)
template <int MODE>
__device__ __forceinline__ HE<float> adj(CTCX_LDS HE<float>* he, int len, int vpos) {
  const int lane = threadIdx.x;
  len = uni(len);
  const int nint = len / 2;
  const int imax = nint > 0 ? nint - 1 : 0;
  const int i = min(lane, imax);
  HE<float> L, R;
  he_ld2(he, 2 * i + 2, L, R);
  const HE<float> vl = he_ld(he, uni(vpos) + 1);
  const bool pick_r = (2 * i + 2 < len) && !(R.v > L.v);
  const uint64_t bm = __ballot(pick_r);
  const float cv = pick_r ? R.v : L.v;
  const int cs = pick_r ? R.s : L.s;
  const uint64_t gm = __ballot(cv > vl.v);
  int p = 0;
  if (MODE == 0 || MODE == 2) {
    while (p < nint) {
      if ((gm >> p) & 1ull) break;
      p = 2 * p + 1 + (int)((bm >> p) & 1ull);
    }
  } else if (MODE == 3) {
#pragma unroll
    for (int h = 0; h < 7; ++h) {
      const bool go = (p < nint) && !((gm >> (p & 63)) & 1ull);
      const int np = 2 * p + 1 + (int)((bm >> (p & 63)) & 1ull);
      p = go ? np : p;
    }
  } else if (MODE == 4) {
    p = (int)(gm & 1ull);
  }
  if (MODE == 5) {
    // lane-parallel: node j is on the root's min path iff each ancestor's min
    // child is the one toward j (bits of bm); the stop is the first on-path
    // node whose min child is > v, or whose min child is a leaf
    const unsigned J = (unsigned)lane + 1u;
    const int dj = 31 - __builtin_clz(J);
    unsigned mis = 0;   // bit k-1: the depth-k ancestor's min child is not toward j
#pragma unroll
    for (int k = 1; k <= 6; ++k) {
      const unsigned A = J >> k;
      const unsigned dir = (J >> (k - 1)) & 1u;
      const unsigned have = (unsigned)(bm >> ((A - 1u) & 63u));
      mis |= ((have ^ dir) & 1u) << (k - 1);
    }
    mis &= (1u << dj) - 1u;
    const bool on = (mis | (unsigned)(lane >= nint)) == 0u;
    const bool gt = cv > vl.v;
    const int nxj = 2 * lane + 1 + (pick_r ? 1 : 0);
    const bool cand = on && (gt || nxj >= nint);
    const uint64_t cm = __ballot(cand);
    const int k = cm ? (int)__builtin_ctzll(cm) : -1;
    if (k < 0) {
      if (lane == 0) he_st(he, 1, vl);
    } else {
      if (on && (lane < k || (lane == k && !gt))) he_st(he, lane + 1, HE<float>{cv, cs});
      if (lane == k) he_st(he, (gt ? lane : nxj) + 1, vl);
    }
    p = (k == 0 && ((gm & 1ull) != 0)) || k < 0 ? 0 : 1;
  }
  if (MODE != 2 && MODE != 4 && MODE != 5) {
    const unsigned Q = (unsigned)p + 1u;
    const unsigned J = (unsigned)lane + 1u;
    const int d = __builtin_clz(J) - __builtin_clz(Q);
    if (J < Q && (Q >> d) == J) he_st(he, (int)J, HE<float>{cv, cs});
    if (lane == 0) he_st(he, p + 1, vl);
  }
  HE<float> res = vl;
  if (p != 0) {
    res.v = bcast(cv, 0);
    res.s = bcast(cs, 0);
  }
  return res;
}

template <int MODE>
__device__ __forceinline__ HE<float> adj_or_real(CTCX_LDS HE<float>* he, int len, int vpos) {
  if (MODE == 6) return wave_adjust_heap<float, 1>(he, heap_geo<1>(len, 131), HE<float>{0.f, 0}, vpos);
  return adj<MODE>(he, len, vpos);
}

template <int MODE>
__global__ void pop_time(const float* vals, float* out) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  CTCX_LDS HE<float>* he = (CTCX_LDS HE<float>*)lds;
  const int lane = threadIdx.x, len = 128;
  for (int i = lane; i < len; i += 64) he_st(he, i + 1, HE<float>{vals[i], i});
  __syncthreads();
  wave_make_heap(he, len);
  HE<float> front = he_ld(he, 1);
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int l = len; l > 1; --l) {
    const HE<float> old_front = front;
    front = adj_or_real<MODE>(he, l - 1, l - 1);
    if (lane == 0) he_st(he, l, old_front);
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) { out[MODE] = (float)(t1 - t0) / (len - 1); out[8 + MODE] = he[1].v; }
}

int main() {
  std::mt19937 g(3);
  std::normal_distribution<float> nd;
  std::vector<float> v(128);
  for (auto& x : v) x = nd(g);
  float *dv, *o, h[16];
  (void)hipMalloc(&dv, 4 * 128);
  (void)hipMalloc(&o, 64);
  (void)hipMemset(o, 0, 64);
  (void)hipMemcpy(dv, v.data(), 4 * 128, hipMemcpyHostToDevice);
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL(pop_time<0>, dim3(1), dim3(64), 8 * (136 + 64), 0, dv, o);
    hipLaunchKernelGGL(pop_time<1>, dim3(1), dim3(64), 8 * (136 + 64), 0, dv, o);
    hipLaunchKernelGGL(pop_time<2>, dim3(1), dim3(64), 8 * (136 + 64), 0, dv, o);
    hipLaunchKernelGGL(pop_time<3>, dim3(1), dim3(64), 8 * (136 + 64), 0, dv, o);
    hipLaunchKernelGGL(pop_time<4>, dim3(1), dim3(64), 8 * (136 + 64), 0, dv, o);
    hipLaunchKernelGGL(pop_time<5>, dim3(1), dim3(64), 8 * (136 + 64), 0, dv, o);
    hipLaunchKernelGGL(pop_time<6>, dim3(1), dim3(64), 8 * (136 + 64), 0, dv, o);
  }
  (void)hipMemcpy(h, o, 64, hipMemcpyDeviceToHost);
  const char* nm[] = {"decode kernel's pop", "no chase", "chase, no stores", "unrolled branch-free chase",
                      "loads + ballots only", "lane-parallel path", "decode kernel's (new)"};
  for (int m = 0; m < 7; ++m) printf("%-30s %7.0f cycles per pop\n", nm[m], h[m]);
  printf("final root: mode0 %g mode5 %g\n", h[8], h[13]);
  return 0;
}
