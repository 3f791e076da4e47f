// Exhaustive check: ctcx::gm::{expf,logf,log1pf} vs the host glibc libm over
// every 32-bit float pattern, gm::expf_t_nonpos (the normalisers' branch-free
// expf) over every x <= 0, -inf and NaN, gm::expf_t_le0 over every x <= 0
// and -inf, and gm::expf_t_core over [the underflow bound, 0].  Built with hipcc (host pass only) and
// -ffp-contract=off, exactly like the device code.
//
//   hipcc -O2 -ffp-contract=off -std=c++17 tools/check_glibc_math.cpp -o /tmp/chk -lpthread
//   /tmp/chk            # all three functions, all 2^32 inputs
//   /tmp/chk sample     # every 97th input (CI-sized)
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <string.h>
#include <atomic>
#include <thread>
#include <vector>

#include "../ctc-beam-search-op_amd/csrc/glibc_math.h"

static bool same(float a, float b) {
  if (isnan(a) && isnan(b)) return true;
  uint32_t ua, ub;
  memcpy(&ua, &a, 4);
  memcpy(&ub, &b, 4);
  return ua == ub;
}

int main(int argc, char** argv) {
  const uint64_t stride = (argc > 1 && !strcmp(argv[1], "sample")) ? 97 : 1;
  const int nthr = (int)std::thread::hardware_concurrency();
  static uint64_t tab[32];
  for (int i = 0; i < 32; ++i) tab[i] = ctcx::gm::exp2f_tab(i);
  std::atomic<uint64_t> bad[4];
  for (auto& b : bad) b = 0;
  std::vector<std::thread> th;
  for (int w = 0; w < nthr; ++w) {
    th.emplace_back([&, w]() {
      uint64_t nb[4] = {0, 0, 0, 0};
      for (uint64_t u = (uint64_t)w * stride; u < (1ull << 32); u += (uint64_t)nthr * stride) {
        float x;
        uint32_t u32 = (uint32_t)u;
        memcpy(&x, &u32, 4);
        float r0 = ::expf(x), g0 = ctcx::gm::expf(x);
        float r1 = ::logf(x), g1 = ctcx::gm::logf(x);
        float r2 = ::log1pf(x), g2 = ctcx::gm::log1pf(x);
        if (!same(r0, g0)) { if (nb[0]++ < 4) printf("expf  %a: libm %a ours %a\n", x, r0, g0); }
        if (!same(r1, g1)) { if (nb[1]++ < 4) printf("logf  %a: libm %a ours %a\n", x, r1, g1); }
        if (!same(r2, g2)) { if (nb[2]++ < 4) printf("log1pf %a: libm %a ours %a\n", x, r2, g2); }
        if (x <= 0.0f || x != x) {
          const float g3 = ctcx::gm::expf_t_nonpos(x, tab);
          if (!same(r0, g3)) { if (nb[3]++ < 4) printf("expf_t_nonpos %a: libm %a ours %a\n", x, r0, g3); }
        }
        if (x <= 0.0f) {   // (NaN excluded: expf_t_le0's domain)
          const float g4 = ctcx::gm::expf_t_le0(x, tab);
          if (!same(r0, g4)) { if (nb[3]++ < 4) printf("expf_t_le0 %a: libm %a ours %a\n", x, r0, g4); }
        }
        if (x <= 0.0f && x >= ctcx::gm::kExpfUnder) {   // expf_t_core's domain
          const float g5 = ctcx::gm::expf_t_core(x, tab);
          if (!same(r0, g5)) { if (nb[3]++ < 4) printf("expf_t_core %a: libm %a ours %a\n", x, r0, g5); }
        }
      }
      for (int k = 0; k < 4; ++k) bad[k] += nb[k];
    });
  }
  for (auto& t : th) t.join();
  printf("stride=%llu mismatches: expf=%llu logf=%llu log1pf=%llu expf_t_nonpos=%llu\n",
         (unsigned long long)stride, (unsigned long long)bad[0].load(),
         (unsigned long long)bad[1].load(), (unsigned long long)bad[2].load(), (unsigned long long)bad[3].load());
  return (bad[0] | bad[1] | bad[2] | bad[3]) ? 1 : 0;
}
