// heap_unit.hip — GPU unit test of the decode kernel's exact TopN heap
// primitives (wave_make_heap, wave_adjust_heap, sort via pop_heap) against
// libstdc++'s std::make_heap / std::pop_heap / std::sort_heap on the host,
// with tie-heavy values so the layout (not just the values) is checked.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off tools/heap_unit.hip -o /tmp/heap_unit
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <random>
#include <vector>

#include "../ctc-beam-search-op_amd/csrc/ctcx_decode.hip"

using namespace ctcx;

struct El { float v; int s; };
struct Gt { bool operator()(const El& a, const El& b) const { return a.v > b.v; } };

// one workgroup: load n = len+1 elements, make_heap(len+1), pop_heap(len+1),
// then nrep "replace root" ops (TopN HEAP push), then sort_heap(len).
template <int RN>
__global__ void heap_kernel(const float* vals, const float* reps, int len, int nrep, int* out_s, float* out_v, int stage) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  CTCX_LDS HE<float>* he = (CTCX_LDS HE<float>*)lds;
  const int lane = threadIdx.x;
  for (int i = lane; i < len + 1; i += 64) he_st(he, i + 1, HE<float>{vals[i], i});
  __syncthreads();
  if (stage == -1) {
    for (int i = lane; i < len + 1; i += 64) out_s[i] = he[i + 1].s;
    return;
  }
  if (stage == -2) {
    if (lane == 0)
      for (int pnt = (len + 1 - 2) / 2; pnt >= 0; --pnt) lane_adjust_heap(he, pnt, len + 1, he_ld(he, pnt + 1));
    __syncthreads();
    for (int i = lane; i < len + 1; i += 64) out_s[i] = he[i + 1].s;
    return;
  }
  wave_make_heap(he, len + 1);
  if (stage == 0) {
    for (int i = lane; i < len + 1; i += 64) out_s[i] = he[i + 1].s;
    return;
  }
  const HE<float> r0 = he_ld(he, 1);
  HE<float> front = wave_adjust_heap<float, RN>(he, heap_geo<RN>(len, len + 3), r0, len);
  if (lane == 0) he_st(he, len + 1, r0);
  if (stage == 1) {
    for (int i = lane; i < len; i += 64) out_s[i] = he[i + 1].s;
    return;
  }
  for (int r = 0; r < nrep; ++r) {
    HE<float> nv;
    nv.v = reps[r];
    nv.s = 1000 + r;
    front = wave_adjust_heap<float, RN>(he, heap_geo<RN>(len, len + 3), nv);
  }
  if (stage == 2) {
    for (int i = lane; i < len; i += 64) out_s[i] = he[i + 1].s;
    if (lane == 0 && (front.s != he[1].s || front.v != he[1].v)) out_s[0] = -12345;
    return;
  }
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int l = len; l > 1; --l) {
    const HE<float> old_front = front;
    front = wave_adjust_heap<float, RN>(he, heap_geo<RN>(l - 1, len + 3), front, l - 1);
    if (lane == 0) he_st(he, l, old_front);
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  for (int i = lane; i < len; i += 64) { out_s[i] = he[i + 1].s; out_v[i] = he[i + 1].v; }
  if (lane == 0 && len > 1) out_v[0] = (float)(t1 - t0) / (float)(len - 1);
}

// timing of the decode's real case: RN = 1, 128-element heap, random pushes
// then a full sort; prints cycles per push and per sort pop
__global__ void heap_time(const float* reps, int nrep, float* out) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  CTCX_LDS HE<float>* he = (CTCX_LDS HE<float>*)lds;
  const int lane = threadIdx.x, len = 128;
  for (int i = lane; i < len + 1; i += 64) he_st(he, i + 1, HE<float>{reps[i], i});
  __syncthreads();
  wave_make_heap(he, len + 1);
  const HE<float> r0 = he_ld(he, 1);
  HE<float> front = wave_adjust_heap<float, 1>(he, heap_geo<1>(len, len + 3), r0, len);
  if (lane == 0) he_st(he, len + 1, r0);
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < nrep; ++r) {
    HE<float> nv;
    nv.v = reps[r] + 3.0f;
    nv.s = 1000 + r;
    if (nv.v > front.v) front = wave_adjust_heap<float, 1>(he, heap_geo<1>(len, len + 3), nv);
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  for (int l = len; l > 1; --l) {
    const HE<float> old_front = front;
    front = wave_adjust_heap<float, 1>(he, heap_geo<1>(l - 1, len + 3), front, l - 1);
    if (lane == 0) he_st(he, l, old_front);
  }
  const uint64_t t2 = __builtin_amdgcn_s_memtime();
  if (lane == 0) { out[0] = (float)(t1 - t0) / nrep; out[1] = (float)(t2 - t1) / (len - 1); out[2] = he[1].v; }
}

int main() {
  {
    std::mt19937 g(3);
    std::normal_distribution<float> nd;
    const int nrep = 4096;
    std::vector<float> reps(nrep + 129);
    for (int i = 0; i < (int)reps.size(); ++i) reps[i] = nd(g) + 0.002f * i;
    float *dr, *o, ho[3];
    (void)hipMalloc(&dr, 4 * reps.size());
    (void)hipMalloc(&o, 16);
    (void)hipMemcpy(dr, reps.data(), 4 * reps.size(), hipMemcpyHostToDevice);
    hipLaunchKernelGGL(heap_time, dim3(1), dim3(64), 8 * (136 + 64), 0, dr, nrep, o);
    (void)hipMemcpy(ho, o, 12, hipMemcpyDeviceToHost);
    printf("RN=1 W=128: %.0f cycles per push slot, %.0f cycles per sort pop\n", ho[0], ho[1]);
    (void)hipFree(dr); (void)hipFree(o);
  }
  std::mt19937 g(7);
  int bad = 0, cases = 0;
  for (int it = 0; it < 300; ++it) {
    const int len = 1 + (int)(g() % 511);
    const int nrep = (int)(g() % 300);
    const int q = 1 + (int)(g() % 8);   // quantisation: few distinct values -> ties
    std::vector<float> vals(len + 1), reps(nrep + 1);
    for (auto& v : vals) v = (float)(g() % (q * 4)) / q;
    for (auto& v : reps) v = (float)(g() % (q * 4)) / q;
   for (int stage = -2; stage < 4; ++stage) {
    // host reference
    std::vector<El> e(len + 1);
    for (int i = 0; i <= len; ++i) e[i] = El{vals[i], i};
    if (stage != -1) std::make_heap(e.begin(), e.end(), Gt());
    if (stage >= 1) { std::pop_heap(e.begin(), e.end(), Gt()); e.pop_back(); }
    if (stage >= 2) for (int r = 0; r < nrep; ++r) {
      e.push_back(El{reps[r], 1000 + r});
      std::pop_heap(e.begin(), e.end(), Gt());     // TopN HEAP push with the front evicted
      e.pop_back();
    }
    if (stage >= 3) std::sort_heap(e.begin(), e.end(), Gt());
    const int nout = stage <= 0 ? len + 1 : len;
    float *dv, *dr, *ov;
    int* os;
    (void)hipMalloc(&dv, 4 * (len + 1));
    (void)hipMalloc(&dr, 4 * (nrep + 1));
    (void)hipMalloc(&os, 4 * (len + 1));
    (void)hipMalloc(&ov, 4 * (len + 1));
    (void)hipMemcpy(dv, vals.data(), 4 * (len + 1), hipMemcpyHostToDevice);
    (void)hipMemcpy(dr, reps.data(), 4 * (nrep + 1), hipMemcpyHostToDevice);
    if (len <= 128)
      hipLaunchKernelGGL(heap_kernel<1>, dim3(1), dim3(64), 8 * (len + 4 + 64), 0, dv, dr, len, nrep, os, ov, stage);
    else if (len <= 256)
      hipLaunchKernelGGL(heap_kernel<2>, dim3(1), dim3(64), 8 * (len + 4 + 64), 0, dv, dr, len, nrep, os, ov, stage);
    else
      hipLaunchKernelGGL(heap_kernel<4>, dim3(1), dim3(64), 8 * (len + 4 + 64), 0, dv, dr, len, nrep, os, ov, stage);
    std::vector<int> gs(nout);
    (void)hipMemcpy(gs.data(), os, 4 * nout, hipMemcpyDeviceToHost);
    if (stage == 3 && it < 12) {
      float cyc;
      (void)hipMemcpy(&cyc, ov, 4, hipMemcpyDeviceToHost);
      printf("len %d: %.0f cycles per sort pop\n", len, cyc);
    }
    int mism = 0, first = -1;
    for (int i = 0; i < nout; ++i) if (gs[i] != e[i].s) { ++mism; if (first < 0) first = i; }
    ++cases;
    if (mism) {
      if (bad < 6) printf("case %d stage %d len %d nrep %d q %d: %d mismatches (first at %d: got %d want %d)\n", it, stage, len, nrep, q, mism,
                          first, gs[first], e[first].s);
      ++bad;
    }
    (void)hipFree(dv); (void)hipFree(dr); (void)hipFree(os); (void)hipFree(ov);
   }
  }
  printf("heap_unit: %d/%d cases mismatched\n", bad, cases);
  return bad ? 1 : 0;
}
