// Test infrastructure (not product code): the accuracy of iqn_cos
// (d3rlpy_amd/csrc/iqn_cos.hpp) on the IQN prior's arguments x = fl(fl(pi
// (e + 1)) tau), e < 64, tau on a dense grid of [0, 1), against cos in double:
// prints the max error in ulps of the float result (and glibc cosf's, for
// scale) and the count of results that differ from the correctly rounded one.
//   g++ -O2 -ffp-contract=off oracle/iqn_cos_check.cpp -o oracle/_ref/iqn_cos_check
#include <cmath>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include "../d3rlpy_amd/csrc/iqn_cos.hpp"

static double ulp_err(float got, double ref) {
  const float rf = (float)ref;
  const double u = std::fabs((double)std::nextafter(rf, INFINITY) - (double)rf);
  return std::fabs((double)got - ref) / (u > 0 ? u : 1e-45);
}

int main(int argc, char** argv) {
  const int64_t n = argc > 1 ? atoll(argv[1]) : (1 << 20);
  double worst = 0, worst_ref = 0;
  int64_t off = 0, tot = 0;
  float wx = 0;
  const float pi_f = 3.14159265358979323846f;
  for (int e = 0; e < 64; ++e) {
    const float ps = pi_f * (float)(e + 1);
    for (int64_t i = 0; i < n; ++i) {
      const float tau = (float)((double)i / (double)n);
      const float x = ps * tau;
      const double ref = std::cos((double)x);
      const float got = iqn_cos(x);
      const double err = ulp_err(got, ref);
      if (err > worst) { worst = err; wx = x; }
      const double er = ulp_err(cosf(x), ref);
      if (er > worst_ref) worst_ref = er;
      off += got != (float)ref;
      ++tot;
    }
  }
  // wider arguments (the exact-reduction range)
  double worst_wide = 0;
  for (int64_t i = 0; i < n; ++i) {
    const float x = (float)(8192.0 * (double)i / (double)n);
    worst_wide = std::fmax(worst_wide, ulp_err(iqn_cos(x), std::cos((double)x)));
  }
  printf("{\"args\": %lld, \"max_ulp\": %.3f, \"at\": %.9g, \"glibc_cosf_max_ulp\": %.3f, "
         "\"not_correctly_rounded\": %lld, \"max_ulp_0_8192\": %.3f}\n",
         (long long)tot, worst, wx, worst_ref, (long long)off, worst_wide);
  return 0;
}
