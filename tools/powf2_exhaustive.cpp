// powf2_exhaustive.cpp — one-off verification (test infrastructure, host only) of the product's
// powf2() in csrc/env_math.h over EVERY float32 input:
//   1. the largest distance, in float ulps, between glibc's double-precision result before its
//      final rounding (powf2_core, itself a bit-exact restatement) and the exact square;
//   2. powf2(x) == libm powf(x, 2.0f) for all 2^32 bit patterns (called through a volatile
//      function pointer so the compiler cannot fold powf(x, 2) into x * x).
// Build + run: hipcc -O2 -std=c++17 -ffp-contract=off -fno-fast-math -I<csrc> tools/powf2_exhaustive.cpp
//              -o /tmp/powf2_exhaustive -lpthread && /tmp/powf2_exhaustive
#include <math.h>
#include <stdio.h>

#include <atomic>
#include <thread>
#include <vector>

#include "env_math.h"

static float (*volatile libm_powf)(float, float) = powf;

int main() {
  const int T = 8;
  std::vector<double> maxerr(T, 0.0);
  std::vector<uint64_t> bad(T, 0), slow(T, 0);
  std::vector<std::thread> th;
  for (int t = 0; t < T; ++t)
    th.emplace_back([&, t]() {
      for (uint64_t u = t; u <= 0xffffffffull; u += T) {
        const float x = mh::mh_asfloat((uint32_t)u);
        if (x != x) continue;  // NaN: both return NaN
        const double p = (double)x * (double)x;
        const float r = (float)p;
        const uint32_t rb = mh::mh_asuint(r);
        const uint32_t ex = (rb >> 23) & 0xffu;
        if (ex > 23u && ex < 0xfeu) {
          const double ulp = ldexp(1.0, (int)ex - 127 - 23);
          const double e = fabs(mh::powf2_core(x) - p) / ulp;
          if (e > maxerr[t]) maxerr[t] = e;
          if (0.5 * ulp - fabs(p - (double)r) <= mh::POWF2_MAX_ERR * ulp) slow[t]++;
        }
        const float a = mh::powf2(x), b = libm_powf(x, 2.0f);
        if (mh::mh_asuint(a) != mh::mh_asuint(b)) bad[t]++;
      }
    });
  for (auto& x : th) x.join();
  double m = 0;
  uint64_t nb = 0, ns = 0;
  for (int t = 0; t < T; ++t) {
    m = maxerr[t] > m ? maxerr[t] : m;
    nb += bad[t];
    ns += slow[t];
  }
  printf("max |core - x^2| = %.3e ulp (guard %.3e); slow-path inputs %llu of 2^32; mismatches vs libm %llu\n", m,
         mh::POWF2_MAX_ERR, (unsigned long long)ns, (unsigned long long)nb);
  return nb == 0 && m < mh::POWF2_MAX_ERR ? 0 : 1;
}
