// lat_probe.hip — one-wave dependency-chain latencies on gfx950 that bound the
// decode kernel's serial TopN operations (cycles per iteration, s_memtime).
//   hipcc --offload-arch=gfx950 -O3 tools/lat_probe.hip -o tools/lat_probe.bin
#include <hip/hip_runtime.h>

#include <cstdio>

#define LDS __attribute__((address_space(3)))

__global__ void probe(int n, float* out, int seed) {
  __shared__ __attribute__((aligned(16))) float buf[1024];
  LDS float* b = (LDS float*)buf;
  const int lane = threadIdx.x;
  for (int i = lane; i < 1024; i += 64) b[i] = (float)((i * 7 + seed) & 63);
  __syncthreads();
  float acc = 0.f;
  uint64_t t0, t1;
  // 1: dependent LDS read chain (index from the previous value)
  int idx = lane;
  t0 = __builtin_amdgcn_s_memtime();
  for (int k = 0; k < n; ++k) idx = (int)b[idx] + lane;
  t1 = __builtin_amdgcn_s_memtime();
  acc += idx;
  if (lane == 0) out[0] = (float)(t1 - t0) / n;
  // 2: VALU compare -> ballot -> scalar branch chain
  float x = (float)lane;
  int cnt = 0;
  t0 = __builtin_amdgcn_s_memtime();
  for (int k = 0; k < n; ++k) {
    const uint64_t m = __ballot(x > (float)(k & 63));
    if (m & 1ull) cnt++;
    x += (float)(m >> 60);
  }
  t1 = __builtin_amdgcn_s_memtime();
  acc += x + cnt;
  if (lane == 0) out[1] = (float)(t1 - t0) / n;
  // 3: readfirstlane chain (VALU -> SGPR -> VALU)
  int y = lane + seed;
  t0 = __builtin_amdgcn_s_memtime();
  for (int k = 0; k < n; ++k) y = __builtin_amdgcn_readfirstlane(y) + lane + 1;
  t1 = __builtin_amdgcn_s_memtime();
  acc += y;
  if (lane == 0) out[2] = (float)(t1 - t0) / n;
  // 4: LDS write then dependent read of the same word (store->load)
  t0 = __builtin_amdgcn_s_memtime();
  float z = 1.f;
  for (int k = 0; k < n; ++k) {
    b[lane] = z + 1.f;
    z = b[lane ^ 1];
  }
  t1 = __builtin_amdgcn_s_memtime();
  acc += z;
  if (lane == 0) out[3] = (float)(t1 - t0) / n;
  // 5: ds_read_b128 + wait + use per iteration, address from readfirstlane
  int p = seed & 7;
  t0 = __builtin_amdgcn_s_memtime();
  for (int k = 0; k < n; ++k) {
    typedef float f4 __attribute__((ext_vector_type(4)));
    const f4 v = *(LDS f4*)(b + 4 * ((p + lane) & 127));
    const float vx = v.x;
    p = __builtin_amdgcn_readfirstlane((int)vx) & 7;
  }
  t1 = __builtin_amdgcn_s_memtime();
  acc += p;
  if (lane == 0) out[4] = (float)(t1 - t0) / n;
  // 6: empty loop with a uniform trip count
  t0 = __builtin_amdgcn_s_memtime();
  int q = seed;
  for (int k = 0; k < n; ++k) q = __builtin_amdgcn_readfirstlane(q) * 3 + 1;
  t1 = __builtin_amdgcn_s_memtime();
  acc += q;
  if (lane == 0) out[5] = (float)(t1 - t0) / n;
  // 7: divergent lane-0 store + uniform LDS read of it
  t0 = __builtin_amdgcn_s_memtime();
  int w = seed;
  for (int k = 0; k < n; ++k) {
    if (lane == 0) b[200 + (k & 7)] = (float)w;
    w = __builtin_amdgcn_readfirstlane((int)b[200 + ((k + 3) & 7)]) + 1;
  }
  t1 = __builtin_amdgcn_s_memtime();
  acc += w;
  if (lane == 0) out[6] = (float)(t1 - t0) / n;
  // 8: ds_bpermute chain (gather from lane 2j+1, the heap child pattern)
  int g = lane;
  t0 = __builtin_amdgcn_s_memtime();
  for (int k = 0; k < n; ++k) g = __builtin_amdgcn_ds_bpermute(((2 * lane + 1 + (g & 1)) & 63) * 4, g) + 1;
  t1 = __builtin_amdgcn_s_memtime();
  acc += g;
  if (lane == 0) out[8] = (float)(t1 - t0) / n;
  // 9: the push pattern: two 8-byte stores (per-lane addresses) then a 16-byte read
  typedef unsigned u2 __attribute__((ext_vector_type(2)));
  typedef unsigned u4 __attribute__((ext_vector_type(4)));
  unsigned hv = lane;
  t0 = __builtin_amdgcn_s_memtime();
  for (int k = 0; k < n; ++k) {
    u2 a; a.x = hv; a.y = hv + 1;
    *(LDS u2*)(b + 2 * ((lane + hv) & 127)) = a;
    *(LDS u2*)(b + 2 * (128 + lane)) = a;
    const u4 r = *(LDS u4*)(b + 4 * (lane & 63));
    hv = r.x + r.w;
  }
  t1 = __builtin_amdgcn_s_memtime();
  acc += hv;
  if (lane == 0) out[9] = (float)(t1 - t0) / n;
  if (lane == 0) out[7] = acc;
}

int main() {
  float* o;
  (void)hipMalloc(&o, 256);
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, 1000, o, 0);
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, 1000, o, 1);
  float h[10];
  (void)hipMemcpy(h, o, 40, hipMemcpyDeviceToHost);
  const char* names[] = {"lds read chain", "cmp->ballot->branch", "readfirstlane chain", "lds store->load",
                         "ds_read_b128 -> readfirstlane", "salu/readfirstlane loop", "lane0 store + read",
                         "(acc)", "ds_bpermute chain", "2x ds_write_b64 + ds_read_b128"};
  for (int i = 0; i < 10; ++i) if (i != 7) printf("%-32s %7.1f cycles/iter\n", names[i], h[i]);
  return 0;
}
