// Host build of the product's fast-refit arithmetic (dialog_amd/csrc/exact_refit.hpp) for the CPU
// test tests/test_exact_refit.py: reads float32 points (x y z per line after a header line
// "n e a b c d"), accumulates the exact moment digits in the order given, and prints the refined
// coefficients' bit patterns.  The device runs the same header; the oracle restates it in C.
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../dialog_amd/csrc/exact_refit.hpp"

// "B" mode: lines of six 32-bit limbs (hex, least significant first) of a 192-bit two's-complement
// integer -> the bits of big_to_double (correct rounding is checked against Python's int->float)
static int big_mode() {
  unsigned w[6];
  while (std::scanf("%x %x %x %x %x %x", &w[0], &w[1], &w[2], &w[3], &w[4], &w[5]) == 6) {
    dlg::Big b;
    for (int k = 0; k < 6; ++k) b.w[k] = w[k];
    const double d = dlg::big_to_double(b);
    unsigned long long u;
    std::memcpy(&u, &d, 8);
    std::printf("%016llx\n", u);
  }
  return 0;
}

int main(int argc, char** argv) {
  if (argc > 1 && argv[1][0] == 'B') return big_mode();
  long long n = 0;
  int e = 0;
  float cin[4];
  if (std::scanf("%lld %d %a %a %a %a", &n, &e, &cin[0], &cin[1], &cin[2], &cin[3]) != 6) return 2;
  int64_t acc[dlg::kMomDigits] = {0};
  const double qs = dlg::pow2d(dlg::kFastBits - e);
  dlg::MomAcc m;
  dlg::mom_zero(m);
  // (flushes after a varying number of points <= kMomFlush: the digits differ with the grouping,
  // the integers they stand for do not)
  int since = 0, every = 1;
  for (long long i = 0; i < n; ++i) {
    float x, y, z;
    if (std::scanf("%a %a %a", &x, &y, &z) != 3) return 3;
    dlg::mom_point(m, dlg::fast_q(x, qs), dlg::fast_q(y, qs), dlg::fast_q(z, qs));
    if (++since == every) {
      dlg::mom_flush(acc, m);
      since = 0;
      every = every % dlg::kMomFlush + 1;
    }
  }
  dlg::mom_flush(acc, m);
  float out[4];
  dlg::refit_exact(acc, e, cin, out);
  unsigned u[4];
  std::memcpy(u, out, 16);
  std::printf("%08x %08x %08x %08x\n", u[0], u[1], u[2], u[3]);
  return 0;
}
