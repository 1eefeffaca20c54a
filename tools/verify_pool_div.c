/* Exhaustive check that the avg-pool's division by a tap count d can be
 * replaced by a reciprocal multiply with one fma correction step,
 *     q = x * r;  q' = fma(fma(-q, d, x), r, q),  r = RN(1/d),
 * is bitwise x / d for EVERY fp32 x, for every count a 3x3 'same' window
 * can have (d = ch * cw, ch, cw in 1..3), given the guards of pool_div()
 * in jr_pool.hip: q itself for q = +-0 / +-inf / NaN (the correction would
 * turn -0 into +0 and inf into NaN), and the true division for |x| <
 * 2^-100, where x / 6 can be subnormal and the correction is off by one ulp.
 * Build: gcc -O3 -mfma -fopenmp tools/verify_pool_div.c -o /tmp/verify_pool_div -lm */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static float bits(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static uint32_t ubits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }

int main(int argc, char** argv) {
  /* optional stride: a sampled run for the CPU test suite (default: all 2^32) */
  const long long stride = argc > 1 ? atoll(argv[1]) : 1;
  const float ds[] = {1.f, 2.f, 3.f, 4.f, 6.f, 9.f};
  long long bad_total = 0;
  for (int k = 0; k < 6; ++k) {
    const float d = ds[k];
    volatile float one = 1.0f;
    const float r = one / d;
    long long bad = 0;
    /* every stride-th bit pattern, plus (stride > 1) every input whose
       magnitude bits lie in [B0, B0 + BN) -- 2^-102 .. 2^-99, around the
       2^-100 guard -- both signs */
    const uint32_t B0 = 0x0C800000u, BN = 0x01800000u;
    const long long nstep = ((1LL << 32) + stride - 1) / stride;
    const long long nsmall = stride > 1 ? 2LL * BN : 0;
#pragma omp parallel for reduction(+ : bad) schedule(static)
    for (long long j = 0; j < nstep + nsmall; ++j) {
      const uint32_t u = j < nstep ? (uint32_t)(j * stride)
                                   : (B0 + (uint32_t)((j - nstep) % BN)) | ((j - nstep) >= BN ? 0x80000000u : 0u);
      const float x = bits(u);
      const float ref = x / d;
      const float q = x * r;
      const float q2 = (isinf(q) || q == 0.f || isnan(q)) ? q : fabsf(x) < 0x1p-100f ? x / d
                                                                                  : fmaf(fmaf(-q, d, x), r, q);
      if (isnan(ref) ? !isnan(q2) : ubits(q2) != ubits(ref)) ++bad;
    }
    printf("d = %g: r = %a, %lld mismatches (stride %lld)\n", d, r, bad, stride);
    bad_total += bad;
  }
  printf(bad_total ? "FAIL\n" : "OK: bitwise equal to x / d for all inputs\n");
  return bad_total != 0;
}
