// Host build of the product's fast-refit arithmetic (dialog_amd/csrc/exact_refit.hpp) for the CPU
// test tests/test_exact_refit.py: reads float32 points (x y z per line after a header line
// "n e a b c d"), accumulates the exact moment digits in the order given, and prints the refined
// coefficients' bit patterns.  The device runs the same header; the oracle restates it in C.
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../dialog_amd/csrc/exact_refit.hpp"

int main() {
  long long n = 0;
  int e = 0;
  float cin[4];
  if (std::scanf("%lld %d %a %a %a %a", &n, &e, &cin[0], &cin[1], &cin[2], &cin[3]) != 6) return 2;
  int64_t acc[dlg::kMomDigits] = {0};
  const double qs = dlg::pow2d(dlg::kFastBits - e);
  for (long long i = 0; i < n; ++i) {
    float x, y, z;
    if (std::scanf("%a %a %a", &x, &y, &z) != 3) return 3;
    dlg::mom_add(acc, dlg::fast_q(x, qs), dlg::fast_q(y, qs), dlg::fast_q(z, qs));
  }
  float out[4];
  dlg::refit_exact(acc, e, cin, out);
  unsigned u[4];
  std::memcpy(u, out, 16);
  std::printf("%08x %08x %08x %08x\n", u[0], u[1], u[2], u[3]);
  return 0;
}
