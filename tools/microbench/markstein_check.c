/* tools/microbench/markstein_check.c -- exhaustive / randomized CPU proof of the short correctly
 * rounded reciprocal and division sequences of vr_sampling.h (rcp_cr, div_cr):
 *   y  = fma(fma(-b, y0, 1), y0, y0)        == RN(1/b)  for every y0 within 1 ulp of 1/b
 *   q  = fma(fma(-b, q0, a), y, q0)          == RN(a/b)  with y = RN(1/b), q0 = RN(a*y)
 * The hardware v_rcp_f32 is specified to 1 ulp, so every y0 it can return is covered: each of
 * RN(1/b) - 1 ulp, RN(1/b), RN(1/b) + 1 ulp is tried.  b ranges over every significand (the
 * sequences are scale-invariant away from the exponent limits, which the kernels' wave guards
 * exclude); a over 4096 random values per significand sample for the division.
 * Build: gcc -O2 -ffp-contract=off -o markstein_check markstein_check.c -lm */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

static float fb(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static uint32_t bf(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static float rn_div(float a, float b) { return (float)((double)a / (double)b); } /* innocuous double rounding */

int main(void) {
  uint64_t bad_rcp = 0, bad_div = 0, n_rcp = 0, n_div = 0;
  uint64_t rng = 0x9e3779b97f4a7c15ull;
  for (uint32_t m = 0; m < (1u << 23); ++m) {
    const float b = fb(0x3f800000u | m); /* [1, 2) */
    const float r = rn_div(1.f, b);
    for (int d = -1; d <= 1; ++d) {
      const float y0 = fb(bf(r) + (uint32_t)d);
      const float y = fmaf(fmaf(-b, y0, 1.f), y0, y0);
      ++n_rcp;
      if (bf(y) != bf(r)) {
        if (bad_rcp < 5) printf("rcp: b=%a y0=%a -> %a want %a\n", b, y0, y, r);
        ++bad_rcp;
      }
    }
    if ((m & 31u) == 0) {
      for (int k = 0; k < 4096; ++k) {
        rng ^= rng << 13; rng ^= rng >> 7; rng ^= rng << 17;
        /* a: any significand, exponent so that a/b in [2^-8, 2) -- the acos arguments, |q| <= ~1 */
        float a = fb((uint32_t)(0x3b800000u + (rng % (0x3fffffffu - 0x3b800000u))));
        if (rng & (1ull << 40)) a = -a;
        const float q0 = a * r;
        const float q = fmaf(fmaf(-b, q0, a), r, q0);
        const float want = rn_div(a, b);
        ++n_div;
        if (bf(q) != bf(want)) {
          if (bad_div < 5) printf("div: a=%a b=%a -> %a want %a\n", a, b, q, want);
          ++bad_div;
        }
      }
    }
  }
  printf("rcp: %llu checked, %llu wrong\ndiv: %llu checked, %llu wrong\n", (unsigned long long)n_rcp,
         (unsigned long long)bad_rcp, (unsigned long long)n_div, (unsigned long long)bad_div);
  return (bad_rcp || bad_div) ? 1 : 0;
}
