/* Host check of the division used by the fused epilogues and the QSGD table build
 * (distributed_learning_simulation_lib_amd/csrc/exact_div.h, qsgd_div_level):
 *   y = RN(1/W); q0 = RN(a*y); t = RN(q0*W - a) (fma, exact); q = RN(q0 - t*y) (fma)
 * must equal the IEEE quotient RN(a/W). Three samples: random binary64 dividends / divisors
 * (incl. integer totals and all-ones significands), binary64 dividends near the midpoints of
 * the quotient grid, and binary32 dividends over the QSGD levels 1..255.
 *   gcc -O2 -march=native -ffp-contract=off scripts/check_exact_div.c -lm && ./a.out [n]
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static uint64_t s = 88172645463325252ull;
static uint64_t xr(void) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; }
static double rd(int emin, int emax) {
  uint64_t m = xr() & ((1ull << 52) - 1);
  int e = emin + (int)(xr() % (uint64_t)(emax - emin + 1));
  uint64_t b = ((xr() & 1) << 63) | ((uint64_t)(e + 1023) << 52) | m;
  double d;
  memcpy(&d, &b, 8);
  return d;
}
static double q64(double a, double w) {
  double y = 1.0 / w, q0 = a * y, t = fma(q0, w, -a);
  return fma(-t, y, q0);
}
static float q32(float a, float w) {
  float y = 1.0f / w, q0 = a * y, t = fmaf(q0, w, -a);
  return fmaf(-t, y, q0);
}

int main(int argc, char** argv) {
  long n = argc > 1 ? atol(argv[1]) : 100000000L, bad = 0;
  for (long i = 0; i < n; i++) {  // random binary64
    double a = rd(-60, 60), w = rd(-20, 40);
    if (i % 7 == 0) w = (double)(1 + xr() % 100000);
    if (i % 11 == 0) { uint64_t b; memcpy(&b, &w, 8); b |= (1ull << 52) - 1; memcpy(&w, &b, 8); }
    double q = q64(a, w), e = a / w;
    bad += memcmp(&q, &e, 8) != 0;
  }
  for (long i = 0; i < n; i++) {  // binary64 near quotient midpoints
    double w = (i & 1) ? (double)(1 + xr() % (1ull << (1 + xr() % 40))) : rd(-20, 40);
    double q = rd(-30, 30), up = nextafter(q, INFINITY);
    double a = w * q + fma(w, up - q, 0.0) * 0.5;
    if (xr() & 1) a = nextafter(a, (xr() & 1) ? INFINITY : -INFINITY);
    double r = q64(a, w), e = a / w;
    bad += memcmp(&r, &e, 8) != 0;
  }
  for (long i = 0; i < n; i++) {  // binary32 over the QSGD levels
    uint32_t b = ((uint32_t)((int)(xr() % 120) + 67) << 23) | (uint32_t)(xr() & 0x7fffff);
    float a, w = (float)(1 + xr() % 255);
    memcpy(&a, &b, 4);
    if (xr() & 1) a = -a;
    float q = q32(a, w), e = a / w;
    bad += memcmp(&q, &e, 4) != 0;
  }
  printf("%ld x 3 quotients, %ld differ from IEEE division\n", n, bad);
  return bad != 0;
}
