// Correctly rounded division of many dividends by one divisor, for the fused epilogues
// (`parameter / total_weight`, fed_avg_algorithm.py:71-74: every element of a segment is divided
// by the segment's total weight).
//
// The compiler's IEEE fp64 division is ~11 VALU instructions per quotient (div_scale x2, a
// quarter-rate rcp, a Newton refinement, div_fmas, div_fixup). With one divisor W per segment the
// reciprocal is taken once per lane, and each quotient costs three fp64 operations:
//
//   y  = RN(1/W)                  one IEEE division per lane and W
//   q0 = RN(a*y)                  a faithful-or-better approximation of a/W
//   t  = RN(q0*W - a)             exact (fma): the residual of q0, negated
//   q  = RN(q0 - t*y)             = RN(a/W): Markstein's correction step (the same two fmas end
//                                 the compiler's IEEE sequence, there with a refined, not
//                                 correctly rounded, reciprocal)
//
// Computing the residual as -(q0*W - a) rather than a - q0*W keeps the sign of a zero quotient
// (-0 / W = -0) for W > 0. The fast path is taken only where none of a, q0, t can leave the
// normal range: W in [2^-60, 2^60] and |a| in [2^-900, 2^900] or a == 0. Everything else —
// inf / NaN accumulators, fp64 values near the under/overflow range, negative / zero / extreme
// totals — goes through the IEEE division (the callers branch wave-uniformly, so a wave with no
// such element never executes it). Checked bit-for-bit against IEEE division on 1.4e9 random
// and near-midpoint quotients on the host (gcc, hardware fma) and by every golden / property
// test of the kernels that use it.
#pragma once

#ifndef FEDAVG_FAST_DIV
#define FEDAVG_FAST_DIV 1
#endif

struct ExactDiv {
  double W;  // the divisor
  double y;  // RN(1/W)
  bool ok;   // W inside the range the fast path is proven for
};

__device__ __forceinline__ ExactDiv exact_div_prepare(double W) {
  ExactDiv d;
  d.W = W;
  d.ok = (W >= 0x1p-60) && (W <= 0x1p60);  // false for NaN, inf, zero and negative totals
  d.y = d.ok ? 1.0 / W : 1.0;
  return d;
}

// The fast quotient of a / d.W; `slow` is set when this element needs the IEEE division.
__device__ __forceinline__ double exact_div_fast(double a, const ExactDiv& d, bool& slow) {
  const double m = __builtin_fabs(a);
  slow |= !((m <= 0x1p900) && ((m >= 0x1p-900) || (a == 0.0)));
  const double q0 = a * d.y;
  const double t = __builtin_fma(q0, d.W, -a);
  return __builtin_fma(-t, d.y, q0);
}

// exact_div_prepare with the reciprocal RN(1/W) supplied by the caller (e.g. computed once on the
// host with IEEE division, the same value): the divisions per lane and divisor are skipped.
__device__ __forceinline__ ExactDiv exact_div_prepare_rcp(double W, double y) {
  ExactDiv d;
  d.W = W;
  d.ok = (W >= 0x1p-60) && (W <= 0x1p60);
  d.y = d.ok ? y : 1.0;
  return d;
}

// out[i] = in[i] / W for one lane's N elements, correctly rounded, with y = RN(1/W) given.
template <int N>
__device__ __forceinline__ void exact_div_block_rcp(const double* in, double* out, double W, double y) {
#if FEDAVG_FAST_DIV
  const ExactDiv d = exact_div_prepare_rcp(W, y);
  bool slow = !d.ok;
#pragma unroll
  for (int i = 0; i < N; ++i) out[i] = exact_div_fast(in[i], d, slow);
  if (__builtin_expect(__ballot(slow) != 0ull, 0)) {
#pragma unroll
    for (int i = 0; i < N; ++i) out[i] = in[i] / W;
  }
#else
  (void)y;
#pragma unroll
  for (int i = 0; i < N; ++i) out[i] = in[i] / W;
#endif
}

// out[i] = in[i] / W for one lane's N elements, correctly rounded. The IEEE fallback runs for
// the whole wave when any of its lanes has an element outside the fast path's range (a uniform
// branch: the common wave executes only the fast sequence). Elements a lane does not own may
// hold anything; they can only send the wave to the fallback, never change an owned quotient.
template <int N>
__device__ __forceinline__ void exact_div_block(const double* in, double* out, double W) {
#if FEDAVG_FAST_DIV
  const ExactDiv d = exact_div_prepare(W);
  bool slow = !d.ok;
#pragma unroll
  for (int i = 0; i < N; ++i) out[i] = exact_div_fast(in[i], d, slow);
  if (__builtin_expect(__ballot(slow) != 0ull, 0)) {
#pragma unroll
    for (int i = 0; i < N; ++i) out[i] = in[i] / W;
  }
#else
#pragma unroll
  for (int i = 0; i < N; ++i) out[i] = in[i] / W;
#endif
}
