// Check ctcx::gm::{exp,log} (double) against the host glibc libm.  2^64
// inputs cannot be enumerated, so every domain the decoder can feed them is
// sampled densely, plus uniformly random bit patterns:
//   exp: the normaliser's arguments x[j] - max <= 0 (uniform in [-50, 0],
//        [-750, 0]), |x| < 2^-50, the over/underflow boundaries, random bits;
//   log: its argument sum_j exp(...) in [1, C] (uniform in [1, 8192]), the
//        near-1 polynomial range [1 - 2^-4, 1 + 2^-4], subnormals, random bits.
//
//   hipcc -O2 -ffp-contract=off -std=c++17 tools/check_glibc_math_f64.cpp -o /tmp/chk64 -lpthread
//   /tmp/chk64 [samples_per_domain]      (default 20,000,000)
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <random>
#include <thread>
#include <vector>

#include "../ctc-beam-search-op_amd/csrc/glibc_math_f64.h"

static bool same(double a, double b) {
  if (isnan(a) && isnan(b)) return true;
  uint64_t ua, ub;
  memcpy(&ua, &a, 8);
  memcpy(&ub, &b, 8);
  return ua == ub;
}

static double bits(uint64_t u) {
  double d;
  memcpy(&d, &u, 8);
  return d;
}

int main(int argc, char** argv) {
  const uint64_t n = argc > 1 ? strtoull(argv[1], nullptr, 10) : 20000000ull;
  const int nthr = (int)std::thread::hardware_concurrency();
  struct Dom { const char* name; int fn; };   // fn 0 = exp, 1 = log
  const Dom doms[] = {{"exp [-50,0]", 0}, {"exp [-750,0]", 0}, {"exp |x|<2^-50", 0}, {"exp [-1100,1100]", 0},
                      {"exp random bits", 0}, {"log [1,8192]", 1}, {"log near 1", 1}, {"log subnormal", 1},
                      {"log random bits", 1}, {"log [0,1]", 1}};
  int fails = 0;
  for (int di = 0; di < (int)(sizeof(doms) / sizeof(doms[0])); ++di) {
    std::atomic<uint64_t> bad{0};
    std::atomic<int> shown{0};
    std::vector<std::thread> th;
    for (int w = 0; w < nthr; ++w) {
      th.emplace_back([&, w]() {
        std::mt19937_64 g(1234567 + 7919 * di + w);
        std::uniform_real_distribution<double> u01(0.0, 1.0);
        uint64_t nb = 0;
        for (uint64_t k = w; k < n; k += nthr) {
          double x;
          switch (di) {
            case 0: x = -50.0 * u01(g); break;
            case 1: x = -750.0 * u01(g); break;
            case 2: x = (u01(g) * 2 - 1) * 0x1p-50; break;
            case 3: x = (u01(g) * 2 - 1) * 1100.0; break;
            case 4: x = bits(g()); break;
            case 5: x = 1.0 + 8191.0 * u01(g); break;
            case 6: x = 1.0 + (u01(g) * 2 - 1) * 0x1.2p-4; break;
            case 7: x = bits(g() & 0x000fffffffffffffull); break;
            case 8: x = bits(g() & 0x7fffffffffffffffull); break;
            default: x = u01(g); break;
          }
          const double r = doms[di].fn == 0 ? ::exp(x) : ::log(x);
          const double m = doms[di].fn == 0 ? ctcx::gm::exp(x) : ctcx::gm::log(x);
          if (!same(r, m)) {
            ++nb;
            if (shown.fetch_add(1) < 3) printf("  %s: x=%a libm=%a ours=%a\n", doms[di].name, x, r, m);
          }
        }
        bad += nb;
      });
    }
    for (auto& t : th) t.join();
    printf("%-18s %llu samples, %llu mismatches\n", doms[di].name, (unsigned long long)n,
           (unsigned long long)bad.load());
    fails += bad.load() != 0;
  }
  return fails ? 1 : 0;
}
