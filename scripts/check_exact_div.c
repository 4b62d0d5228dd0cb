/* Host check of the division used by the fused epilogues
 * (distributed_learning_simulation_lib_amd/csrc/exact_div.h):
 *   y = RN(1/W); q0 = RN(a*y); t = RN(q0*W - a) (fma, exact); q = RN(q0 - t*y) (fma)
 * must equal the IEEE quotient RN(a/W) over the whole range the kernels take the fast path for
 * (W in [2^-60, 2^60], |a| in [2^-900, 2^900] or a = +-0; negative totals take IEEE division). Two samples: random binary64 dividends /
 * divisors over that range (incl. integer totals and all-ones significands), and binary64
 * dividends near the midpoints of the quotient grid. (The QSGD tables divide with IEEE division
 * since round 3: qsgd_table_kernel builds each table once per call.)
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
  // keep -t a negation of the rounded residual: gcc would otherwise fuse it into the residual's
  // fma (vfnmsub: -(q0*w) + a), which gives +0 where -t is -0 and breaks -0 / W (the GPU code
  // negates the operand, as written; the golden signed-zero cases check it there)
  __asm__ volatile("" : "+x"(t));
  return fma(-t, y, q0);
}

int main(int argc, char** argv) {
  long n = argc > 1 ? atol(argv[1]) : 100000000L, bad = 0;
  for (long i = 0; i < n; i++) {  // random binary64 over the fast path's whole range
    double a = rd(-900, 899), w = fabs(rd(-60, 59));  // the fast path takes positive totals only
    if (i % 7 == 0) w = (double)(1 + xr() % 100000);
    if (i % 11 == 0) { uint64_t b; memcpy(&b, &w, 8); b |= (1ull << 52) - 1; memcpy(&w, &b, 8); }
    if (i % 13 == 0) a = 0.0 * ((xr() & 1) ? 1.0 : -1.0);
    double q = q64(a, w), e = a / w;
    bad += memcmp(&q, &e, 8) != 0;
  }
  for (long i = 0; i < n; i++) {  // binary64 near quotient midpoints
    double w = (i & 1) ? (double)(1 + xr() % (1ull << (1 + xr() % 40))) : fabs(rd(-60, 59));
    double q = rd(-800, 800), up = nextafter(q, INFINITY);
    double a = w * q + fma(w, up - q, 0.0) * 0.5;
    if (xr() & 1) a = nextafter(a, (xr() & 1) ? INFINITY : -INFINITY);
    if (!(fabs(a) >= 0x1p-900 && fabs(a) <= 0x1p900)) continue;
    double r = q64(a, w), e = a / w;
    bad += memcmp(&r, &e, 8) != 0;
  }
  printf("%ld x 2 quotients, %ld differ from IEEE division\n", n, bad);
  return bad != 0;
}
