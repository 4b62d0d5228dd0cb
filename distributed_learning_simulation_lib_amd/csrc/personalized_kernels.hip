// personalized_kernels.hip — gfx950 kernel of the server-side PersonalizedFedAVG reduce.
//
// What the reference computes (simulation_lib/algorithm/personalized_aggregation_algorithm.py):
//   every receiver j of worker_weights keeps its own FedAVGAlgorithm (:15-21); an arriving
//   update of worker i is deep-copied into every receiver j != i with the weight
//   worker_weights[j].get(i, 0) (:29-43), i.e. per receiver, per named tensor t:
//       acc_j[t] = round(x_i.to(f64) * w_ji)  (first)  /  acc_j[t] + round(x_i * w_ji)
//       W_j[t]  += w_ji                                   (fed_avg_algorithm.py:43-64)
//   out_j[t] = acc_j[t] / W_j[t] with the NaN assertions (fed_avg_algorithm.py:88-97), and
//   central[t] = sum over receivers j in key order of round(out_j[t] * (1/M))
//   (weighted_avg, aggregation_algorithm.py:51-76, called at :51-53).
//
// Shape: out = W · X for an [M x N] weight matrix and N client rows — but every receiver's
// sum must be the arrival-order fp64 chain with separately rounded products to stay
// bit-identical, which no MFMA instruction computes (its internal reduction order and
// rounding are not the reference's). So the contraction runs on the fp64 VALU, register-
// blocked:
//   * a workgroup owns a 256-element chunk of one segment (64 lanes x 4 elements) and up to
//     128 receivers: wave w holds the fp64 accumulators of receivers [16w, 16w+16) for the
//     lane's 4 elements (128 VGPRs);
//   * clients stream in arrival order, the next client group's 16-B loads in flight while a
//     group folds; the waves of a workgroup read the same 1 KiB per client (CU L1 / XCD L2:
//     HBM sees every client byte once per launch); weights are wave-uniform SGPR operands;
//     every 16-B load feeds 16 receivers x 4 elements = 64 fp64 folds — VALU-bound;
//   * the pairs the reference skips (a receiver's own update :31-32, absent tensors, padding)
//     fold with weight 0, which is exact except for ±0 / NaN sums — those elements alone are
//     re-folded with the pairs skipped (the loop stays branch-free);
//   * epilogue: divide by the receiver's per-segment total (IEEE division), store out_j, and
//     fold the centralized average across the waves in receiver order through LDS (one
//     barrier per wave); receivers beyond 128 run as further launches that carry the
//     centralized chain in an fp64 scratch buffer.
#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <type_traits>
#include <string>
#include <vector>

#include "../../include/fedavg_hip.h"
#include "exact_div.h"

__attribute__((visibility("hidden"))) int32_t fedavg_internal_fail(int32_t code, const char* msg);

namespace {

int32_t pfail(int32_t code, const std::string& msg) { return fedavg_internal_fail(code, msg.c_str()); }

#define PERS_HIP_TRY(expr)                                                                \
  do {                                                                                    \
    hipError_t e_ = (expr);                                                               \
    if (e_ != hipSuccess) {                                                               \
      return pfail(FEDAVG_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_));    \
    }                                                                                     \
  } while (0)

#define PERS_RET(expr)              \
  do {                              \
    int32_t r_ = (expr);            \
    if (r_ != FEDAVG_OK) return r_; \
  } while (0)

#ifndef PERS_VE
#define PERS_VE 4
#endif
constexpr int kVE = PERS_VE;           // elements per lane
constexpr int kChunk = 64 * kVE;       // elements per workgroup
#ifndef PERS_JB  // receivers per wave (8 or 16): the fp64 accumulators of a lane are kVE x kJB
#define PERS_JB 16
#endif
constexpr int kJB = PERS_JB;           // receivers per wave
constexpr int kGroup = 128;            // receivers per launch
constexpr int kMaxWaves = kGroup / kJB;  // waves per workgroup (8, or 16 at 8 receivers per wave)
static_assert(kJB == 8 || kJB == 16, "receivers per wave");
#ifndef PERS_U  // 2 keeps every dtype/fold at <= 168 VGPRs = 3 waves per SIMD (measured best)
#define PERS_U 2
#endif
constexpr int kU = PERS_U;             // clients loaded ahead per lane
#ifndef PERS_PTR_AHEAD  // register pipeline: client pointers loaded one group ahead
#define PERS_PTR_AHEAD 1
#endif
// Whole aligned fp32 / fp64 chunks of the fused (FMA) fold stream clients through an LDS-DMA ring;
// the separately rounded fold keeps the register pipeline (VALU-bound: the ring measured 3 % slower
// there). Weight rows staged through the ring, and a one-client-ahead weight prefetch, measured
// slower and are not kept.

struct PChunk {
  int32_t seg;
  int32_t count;  // elements (== kChunk except at a segment's end)
  int64_t start;  // first element, relative to the segment
};

enum CentralMode : int32_t {
  CENTRAL_NONE = 0,
  CENTRAL_FINAL = 1,     // fold this launch's receivers, write the centralized model
  CENTRAL_CARRY_OUT = 2, // ... write the fp64 chain to the carry buffer (more groups follow)
};

struct PArgs {
  const PChunk* chunks;
  const void* const* cptrs;   // [T][Npad] segment-major client pointers (NULL = absent / padding)
  const double* w;            // [Npad][waves*16] weights: receiver r of the launch at column r;
                              // 0 for the pairs the reference skips (own update, absent, padding)
  const int32_t* exmask;      // [N][waves] bit j: the wave's receiver j skips client k (own update)
  const void* zeros;          // kChunk zero doubles (loads of absent tensors and padding)
  const double* wtot;         // [kGroup][T] per-receiver, per-segment total weight
  const double* wrcp;         // [kGroup][T] RN(1 / wtot), IEEE division on the host
  void* const* outs;          // [kGroup][T] output pointers
  void* const* central;       // [T] centralized outputs (CENTRAL_FINAL)
  double* carry;              // flat fp64 carry of the centralized chain (P elements)
  const int64_t* seg_off;     // [T] segment offsets in the carry
  uint32_t* flag;             // [0] acc NaN, [1] result NaN, [2] centralized NaN
  int32_t N;                  // clients (arrivals)
  int32_t Npad;               // N rounded up to the client group size kU
  int32_t T;
  int32_t aligned;            // every client / output pointer allows the vector accesses
  int32_t M;                  // receivers of this launch (<= kGroup)
  int32_t waves;              // waves of the launch (ceil(M / 16))
  int32_t wstride;            // row stride of w (waves * 16)
  int32_t ring;               // 1 = whole aligned fp32/fp64 chunks stream through the LDS ring
  int32_t out_f32;
  int32_t central_mode;
  int32_t central_in;         // 1 = continue the chain from the carry buffer
  int32_t central_f32;
  double cw;                  // 1 / (number of receivers), the weighted_avg weight
};

#define PERS_AS_GLOBAL __attribute__((address_space(1)))
#define PERS_AS_CONST __attribute__((address_space(4)))
template <typename T>
using gp = T PERS_AS_GLOBAL*;
template <typename T>
using kp = const T PERS_AS_CONST*;

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef double f64x2 __attribute__((ext_vector_type(2)));

struct bf16_t {
  uint16_t bits;
};

__device__ __forceinline__ double h2d(uint32_t h) {
  return static_cast<double>(__half2float(__ushort_as_half(static_cast<unsigned short>(h))));
}
__device__ __forceinline__ double b2d(uint32_t b) { return static_cast<double>(__uint_as_float(b << 16)); }

// Raw (undecoded) kVE-element slice of one client chunk for one lane: loaded one client group
// ahead of the fold (software pipelining), expanded to doubles when folded.
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
template <typename T>
struct Raw;
template <>
struct Raw<float> {
  using type = f32x4;
  static constexpr int kSize = 4;
  __device__ __forceinline__ static type full(uint64_t b, int e) { return *((gp<const f32x4>)((gp<const float>)b + e)); }
  __device__ __forceinline__ static type guarded(uint64_t b, int e, int count) {
    type v;
    v.x = (e < count) ? ((gp<const float>)b)[e] : 0.f;
    v.y = (e + 1 < count) ? ((gp<const float>)b)[e + 1] : 0.f;
    v.z = (e + 2 < count) ? ((gp<const float>)b)[e + 2] : 0.f;
    v.w = (e + 3 < count) ? ((gp<const float>)b)[e + 3] : 0.f;
    return v;
  }
  __device__ __forceinline__ static void expand(type v, double* x) {
    x[0] = v.x;
    x[1] = v.y;
    x[2] = v.z;
    x[3] = v.w;
  }
};
struct f64x2x2 {
  f64x2 lo, hi;
};
template <>
struct Raw<double> {
  using type = f64x2x2;
  static constexpr int kSize = 8;
  __device__ __forceinline__ static type full(uint64_t b, int e) {
    const gp<const f64x2> p = (gp<const f64x2>)((gp<const double>)b + e);
    return type{p[0], p[1]};
  }
  __device__ __forceinline__ static type guarded(uint64_t b, int e, int count) {
    const gp<const double> p = (gp<const double>)b;
    type v;
    v.lo.x = (e < count) ? p[e] : 0.0;
    v.lo.y = (e + 1 < count) ? p[e + 1] : 0.0;
    v.hi.x = (e + 2 < count) ? p[e + 2] : 0.0;
    v.hi.y = (e + 3 < count) ? p[e + 3] : 0.0;
    return v;
  }
  __device__ __forceinline__ static void expand(type v, double* x) {
    x[0] = v.lo.x;
    x[1] = v.lo.y;
    x[2] = v.hi.x;
    x[3] = v.hi.y;
  }
};
template <typename H>
struct Raw16 {  // 2-byte inputs: two elements per dword
  using type = u32x2;
  static constexpr int kSize = 2;
  __device__ __forceinline__ static type full(uint64_t b, int e) { return *((gp<const u32x2>)((gp<const uint16_t>)b + e)); }
  __device__ __forceinline__ static type guarded(uint64_t b, int e, int count) {
    const gp<const uint16_t> p = (gp<const uint16_t>)b;
    uint32_t h[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) h[i] = (e + i < count) ? p[e + i] : 0u;
    return u32x2{h[0] | (h[1] << 16), h[2] | (h[3] << 16)};
  }
  __device__ __forceinline__ static void expand(type v, double* x) {
    x[0] = H::cvt(v.x & 0xffffu);
    x[1] = H::cvt(v.x >> 16);
    x[2] = H::cvt(v.y & 0xffffu);
    x[3] = H::cvt(v.y >> 16);
  }
};
struct HalfCvt {
  __device__ __forceinline__ static double cvt(uint32_t h) { return h2d(h); }
};
struct Bf16Cvt {
  __device__ __forceinline__ static double cvt(uint32_t h) { return b2d(h); }
};
template <>
struct Raw<__half> : Raw16<HalfCvt> {};
template <>
struct Raw<bf16_t> : Raw16<Bf16Cvt> {};
static_assert(kVE == 4, "the Raw loaders move 4 elements per lane");

enum PFold : int { PF_MULADD = 0, PF_FMA = 1 };

template <int B, int E, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(f);
  }
}

template <int FOLD>
__device__ __forceinline__ double pfold(double acc, double x, double w) {
  if constexpr (FOLD == PF_FMA) {
    return __builtin_fma(x, w, acc);  // exact products (host-proven): same rounding
  } else {
    const double p = x * w;  // tmp = x.to(float64) * w   (fed_avg_algorithm.py:54)
    return acc + p;          // acc += tmp                 (:58)
  }
}

#ifndef PERS_MA_GROUP  // receivers whose products issue before their sums (separately rounded fold)
#define PERS_MA_GROUP 1
#endif
// acc[v][J0 + j] (+)= x[v] * w[j] for the H receivers of one half. The separately rounded fold
// issues each receiver's 4 products before their 4 sums (the dependent add right behind its
// multiply stalls the wave); PIN keeps every sum in place (see fold_ring_split).
template <int FOLD, int J0, int H, bool PIN, bool BATCH = true>
__device__ __forceinline__ void fold_half(double (&acc)[kVE][kJB], const double* x, const double* w) {
  if constexpr (FOLD == PF_MULADD && !BATCH) {
#pragma unroll
    for (int j = 0; j < H; ++j)
#pragma unroll
      for (int v = 0; v < kVE; ++v) {
        acc[v][J0 + j] = pfold<FOLD>(acc[v][J0 + j], x[v], w[j]);
        if constexpr (PIN) asm volatile("" : "+v"(acc[v][J0 + j]));
      }
  } else if constexpr (FOLD == PF_FMA) {
#pragma unroll
    for (int j = 0; j < H; ++j)
#pragma unroll
      for (int v = 0; v < kVE; ++v) {
        acc[v][J0 + j] = __builtin_fma(x[v], w[j], acc[v][J0 + j]);
        if constexpr (PIN) asm volatile("" : "+v"(acc[v][J0 + j]));
      }
  } else {
#pragma unroll
    for (int j = 0; j < H; j += PERS_MA_GROUP) {
      double p[PERS_MA_GROUP][kVE];
#pragma unroll
      for (int jj = 0; jj < PERS_MA_GROUP; ++jj)
#pragma unroll
        for (int v = 0; v < kVE; ++v) p[jj][v] = x[v] * w[j + jj];  // tmp = x.to(float64) * w (:54)
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int jj = 0; jj < PERS_MA_GROUP; ++jj)
#pragma unroll
        for (int v = 0; v < kVE; ++v) {
          acc[v][J0 + j + jj] = acc[v][J0 + j + jj] + p[jj][v];  // acc += tmp (:58)
          if constexpr (PIN) asm volatile("" : "+v"(acc[v][J0 + j + jj]));
        }
      __builtin_amdgcn_sched_barrier(0);
    }
  }
}

__device__ __forceinline__ void pflag(uint32_t* flag, int word) {
  __hip_atomic_store(flag + word, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Base address of client k's slice of this chunk: an absent tensor (NULL) or a padding client
// reads the zero block instead (its weights are 0 for every receiver).
__device__ __forceinline__ uint64_t client_base(uint64_t p, int64_t start_bytes, uint64_t zeros) {
  return p ? p + start_bytes : zeros;
}

template <typename T, bool FULL>
__device__ __forceinline__ typename Raw<T>::type load_raw(uint64_t b, int e, int count) {
  if constexpr (FULL) {
    return Raw<T>::full(b, e);
  } else {
    return Raw<T>::guarded(b, e, count);
  }
}

__device__ __forceinline__ bool zero_or_nan(double v) { return v == 0.0 || v != v; }

// Store one receiver's kVE results of the lane (non-temporal vector stores on whole chunks).
template <bool FULL>
__device__ __forceinline__ void store_result(uint64_t op, int64_t start, int e, int count, bool f32, const double* r) {
  if (f32) {
    gp<float> o = (gp<float>)(reinterpret_cast<void*>(op)) + start + e;
    if (FULL) {
      __builtin_nontemporal_store(f32x4{static_cast<float>(r[0]), static_cast<float>(r[1]),
                                        static_cast<float>(r[2]), static_cast<float>(r[3])}, (gp<f32x4>)o);
    } else {
#pragma unroll
      for (int v = 0; v < kVE; ++v)
        if (e + v < count) o[v] = static_cast<float>(r[v]);
    }
  } else {
    gp<double> o = (gp<double>)(reinterpret_cast<void*>(op)) + start + e;
    if (FULL) {
      __builtin_nontemporal_store(f64x2{r[0], r[1]}, (gp<f64x2>)o);
      __builtin_nontemporal_store(f64x2{r[2], r[3]}, (gp<f64x2>)(o + 2));
    } else {
#pragma unroll
      for (int v = 0; v < kVE; ++v)
        if (e + v < count) o[v] = r[v];
    }
  }
}

// The main loop. Every receiver of the wave folds every client of the (padded) arrival list:
// the pairs the reference skips — a receiver's own update (:31-32), an absent tensor, padding —
// carry weight 0. Folding x*0 into acc is exact (acc + ±0 == acc) except when acc is -0.0 and
// the product +0.0 (the sum becomes +0.0) or x is inf/NaN (the product is NaN); both leave a
// receiver's final sum at ±0 or NaN, so those — and only those — elements are re-folded at the
// end with the skipped pairs really skipped (refold below). The loop itself has no branches
// and no per-receiver tests: 16 receivers x 4 elements fold per 16-byte load, with the next
// client group's loads in flight.
// ---- LDS-DMA client ring (whole, 16-B aligned fp32 / fp64 chunks) ---------------------------
// Clients are staged global -> LDS with global_load_lds_dwordx4 (no VGPRs): a stage is kSC
// clients; stage s+kD is issued while stage s is folded, so kD x kSC client slices per
// workgroup are in flight without costing registers. Each wave issues the same number of
// DMA instructions per stage (kSC / waves clients, or all kSC when the workgroup has fewer
// waves), waits for its own with a counted vmcnt, and one barrier per stage publishes them.
constexpr int kSC = 4;   // clients per stage (8 measured no faster, profiles/r04_pers_rcp_ab.txt)
constexpr int kD = 3;    // stages in flight ahead of the one being folded
constexpr int kRS = kD + 2;  // ring stages: the stage being written was last read two barriers ago

template <int N>
__device__ __forceinline__ void wait_vmcnt_le() {
  // s_waitcnt with vmcnt = N (bits 3:0 and 15:14), expcnt and lgkmcnt left at "no wait"
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}
__device__ __forceinline__ void wait_vmcnt(int n) {
  switch (n) {  // wave-uniform
    case 0: wait_vmcnt_le<0>(); break;
    case 1: wait_vmcnt_le<1>(); break;
    case 2: wait_vmcnt_le<2>(); break;
    case 3: wait_vmcnt_le<3>(); break;
    case 4: wait_vmcnt_le<4>(); break;
    case 5: wait_vmcnt_le<5>(); break;
    case 6: wait_vmcnt_le<6>(); break;
    case 7: wait_vmcnt_le<7>(); break;
    case 8: wait_vmcnt_le<8>(); break;
    case 9: wait_vmcnt_le<9>(); break;
    case 10: wait_vmcnt_le<10>(); break;
    case 11: wait_vmcnt_le<11>(); break;
    case 12: wait_vmcnt_le<12>(); break;
    case 13: wait_vmcnt_le<13>(); break;
    case 14: wait_vmcnt_le<14>(); break;
    case 15: wait_vmcnt_le<15>(); break;
    case 16: wait_vmcnt_le<16>(); break;
    case 17: wait_vmcnt_le<17>(); break;
    case 18: wait_vmcnt_le<18>(); break;
    case 19: wait_vmcnt_le<19>(); break;
    case 20: wait_vmcnt_le<20>(); break;
    case 21: wait_vmcnt_le<21>(); break;
    case 22: wait_vmcnt_le<22>(); break;
    case 23: wait_vmcnt_le<23>(); break;
    default: wait_vmcnt_le<24>(); break;
  }
}

template <typename T>
struct Glds;
template <>
struct Glds<float> {
  static constexpr int kIPC = 1;             // DMA instructions per client slice (1 KiB)
  static constexpr int kSlice = kChunk * 4;  // bytes
  // lane l moves its own 4 elements (16 B at l*16) to slot + l*16
  __device__ __forceinline__ static void issue(uint64_t base, int lane, char* slot) {
    __builtin_amdgcn_global_load_lds((void PERS_AS_GLOBAL*)(base + lane * 16), (void __attribute__((address_space(3)))*)slot, 16, 0, 0);
  }
  // a slice is read one client ahead and widened only after its wait
  using RawT = f32x4;
  __device__ __forceinline__ static RawT read_raw(const char* slot, int lane) {
    return *reinterpret_cast<const f32x4*>(slot + lane * 16);
  }
  __device__ __forceinline__ static void expand(RawT v, double* x) {
    x[0] = v.x;
    x[1] = v.y;
    x[2] = v.z;
    x[3] = v.w;
  }
};
template <>
struct Glds<double> {
  static constexpr int kIPC = 2;             // 2 KiB per client slice
  static constexpr int kSlice = kChunk * 8;
  // lane l's 4 elements are 32 B at l*32: the first 16 B land in half A (slot + l*16), the
  // second in half B (slot + 1 KiB + l*16) — the LDS image stays lane-linear per instruction
  __device__ __forceinline__ static void issue(uint64_t base, int lane, char* slot) {
    __builtin_amdgcn_global_load_lds((void PERS_AS_GLOBAL*)(base + lane * 32), (void __attribute__((address_space(3)))*)slot, 16, 0, 0);
    __builtin_amdgcn_global_load_lds((void PERS_AS_GLOBAL*)(base + lane * 32 + 16),
                                     (void __attribute__((address_space(3)))*)(slot + 1024), 16, 0, 0);
  }
  using RawT = f64x2x2;
  __device__ __forceinline__ static RawT read_raw(const char* slot, int lane) {
    return RawT{*reinterpret_cast<const f64x2*>(slot + lane * 16), *reinterpret_cast<const f64x2*>(slot + 1024 + lane * 16)};
  }
  __device__ __forceinline__ static void expand(RawT v, double* x) {
    x[0] = v.lo.x;
    x[1] = v.lo.y;
    x[2] = v.hi.x;
    x[3] = v.hi.y;
  }
};
template <typename T>
constexpr bool kHasGlds = std::is_same<T, float>::value || std::is_same<T, double>::value;

// The main loop on the LDS ring: acc[v][j] += x_k[v] * w_kj for every client k of the (padded)
// list, in order (whole chunks, 16-B aligned client pointers), with the weight loads hidden under
// the FMAs. Scalar loads complete out of order,
// so a wave can only wait for all of them at once (lgkmcnt(0)): loading a client's 16 weights and
// then waiting exposes the scalar-load latency once per client. Here the receivers are split in
// halves: while the low half's 32 FMAs of client c run, the high half's weights of c load; while
// the high half's FMAs run, the low half's weights and the x slice of client c + 1 load. Each wait
// then comes after 32 FMAs, with the same 32 weight SGPRs live as before (two halves of 8).
template <typename T, int FOLD>
__device__ __forceinline__ void fold_ring_split(const PArgs& a, int wave, int lane, int64_t sb, kp<uint64_t> ptrs,
                                                kp<double> wt, char* ring, double (&acc)[kVE][kJB]) {
  using G = Glds<T>;
  constexpr int H = kJB / 2;
  const uint64_t zeros = reinterpret_cast<uint64_t>(a.zeros);
  const int waves = a.waves;
  const int per = wave < kSC ? (kSC - wave + waves - 1) / waves : 0;
  const int nst = a.Npad / kSC;
  auto issue = [&](int st) {
    char* stage = ring + (st % kRS) * (kSC * G::kSlice);
    for (int i = 0; i < per; ++i) {
      const int c = wave + i * waves;
      const uint64_t p = ptrs[st * kSC + c];
      G::issue(p ? p + sb : zeros, lane, stage + c * G::kSlice);
    }
  };
  // stage st is usable once this wave's DMAs of it landed and the barrier saw every wave's
  auto enter = [&](int st) {
    if (st + kD < nst) issue(st + kD);
    const int ahead = (nst - 1 - st < kD) ? nst - 1 - st : kD;
    // the steady state (kD stages ahead; 1, 2 or 4 clients per wave and stage for 4+, 2-3 or 1
    // waves) waits on an immediate count: wait_vmcnt's compare-and-branch ladder over 25 counts
    // cost 16 % of the 4-wave integer-weight round (profiles/r04_pers_static_vmcnt_ab.txt;
    // immediates for the last stages too measured no faster)
    if (ahead == kD && per == 1)
      wait_vmcnt_le<kD * G::kIPC>();
    else if (ahead == kD && per == 2)
      wait_vmcnt_le<2 * kD * G::kIPC>();
    else if (ahead == kD && per == 4)
      wait_vmcnt_le<4 * kD * G::kIPC>();
    else
      wait_vmcnt(ahead * per * G::kIPC);
    __builtin_amdgcn_s_barrier();
  };
  for (int st = 0; st < kD && st < nst; ++st) issue(st);
  enter(0);
  // the client slot, the ring stage and the weight row advance incrementally (no per-client
  // division or 64-bit multiply in the scalar stream)
  constexpr int kStage = kSC * G::kSlice;
  const char* cur = ring;
  int c_in = 0, ring_st = 0, st = 0;
  kp<double> wk = wt;
  const int64_t wstep = a.wstride;
  typename G::RawT xr = G::read_raw(cur, lane);
  double wlo[H];
#pragma unroll
  for (int j = 0; j < H; ++j) wlo[j] = wt[j];
  const int n = a.Npad;
#pragma unroll 1
  for (int k = 0; k < n; ++k) {
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the x slice and the low weights of k
    __builtin_amdgcn_sched_barrier(0);
    double whi[H];
#pragma unroll
    for (int j = 0; j < H; ++j) whi[j] = wk[H + j];
    __builtin_amdgcn_sched_barrier(0);
    double x[kVE];
    G::expand(xr, x);
    fold_half<FOLD, 0, H, true>(acc, x, wlo);  // pinned ahead of the stage branch below
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the high weights of k
    __builtin_amdgcn_sched_barrier(0);
    // next client: the next slot of this stage, or the next stage's first (entered here); after
    // the last client, this one again
    const char* nxt = cur;
    kp<double> wn = wk;
    if (k + 1 < n) {
      wn = wk + wstep;
      if (c_in + 1 < kSC) {
        nxt = cur + G::kSlice;
        ++c_in;
      } else {
        enter(++st);
        ring_st = ring_st + 1 == kRS ? 0 : ring_st + 1;
        nxt = ring + ring_st * kStage;
        c_in = 0;
      }
    }
    xr = G::read_raw(nxt, lane);
#pragma unroll
    for (int j = 0; j < H; ++j) wlo[j] = wn[j];
    __builtin_amdgcn_sched_barrier(0);
    fold_half<FOLD, H, H, false>(acc, x, whi);
    __builtin_amdgcn_sched_barrier(0);
    cur = nxt;
    wk = wn;
  }
}

template <typename T, int FOLD, bool FULL, bool RING>
__device__ __forceinline__ void pers_body(const PArgs& a, int wave, int lane, int seg, int count, int64_t start,
                                          double* chain, char* ring) {
  using R = Raw<T>;
  using RT = typename R::type;
  const int j0 = wave * kJB;  // first receiver of this wave (within the launch)
  const int e = lane * kVE;
  const int64_t sb = start * R::kSize;
  const uint64_t zeros = reinterpret_cast<uint64_t>(a.zeros);
  const kp<uint64_t> ptrs = (kp<uint64_t>)(a.cptrs) + static_cast<int64_t>(seg) * a.Npad;
  const kp<double> wt = (kp<double>)(a.w) + j0;

  // fp64 accumulators of the wave's 16 receivers for the lane's kVE elements, started at the
  // IEEE additive identity (-0.0 + p == p: the first fold equals the reference's assignment)
  double acc[kVE][kJB];
#pragma unroll
  for (int v = 0; v < kVE; ++v)
#pragma unroll
    for (int j = 0; j < kJB; ++j) acc[v][j] = -0.0;

  if constexpr (RING) {
    fold_ring_split<T, FOLD>(a, wave, lane, sb, ptrs, wt, ring, acc);
  } else {
    // the register pipeline (client slices loaded one group ahead) with the split weight loads
    // of fold_ring_split: each lgkmcnt(0) wait comes after half a client's folds
    constexpr int H = kJB / 2;
    RT nxt[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) nxt[u] = load_raw<T, FULL>(client_base(ptrs[u], sb, zeros), e, count);
    double wlo[H];
#pragma unroll
    for (int j = 0; j < H; ++j) wlo[j] = wt[j];
    const int n = a.Npad;
    kp<double> wk = wt;  // weight row of client k + u, advanced incrementally
    const int64_t wstep = a.wstride;
#if PERS_PTR_AHEAD
    // the next group's client pointers are loaded one group ahead, with the first client's high
    // weights (a scalar load waited at once per group otherwise exposed its whole latency)
    uint64_t pn[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) pn[u] = ptrs[(kU + u < n) ? kU + u : u];
#endif
    for (int k = 0; k < n; k += kU) {
      RT cur[kU];
#pragma unroll
      for (int u = 0; u < kU; ++u) cur[u] = nxt[u];
      const int kn = (k + kU < n) ? k + kU : k;  // the last group re-loads itself (L2 hits)
#if PERS_PTR_AHEAD
#pragma unroll
      for (int u = 0; u < kU; ++u) nxt[u] = load_raw<T, FULL>(client_base(pn[u], sb, zeros), e, count);
      const int kn2 = (kn + kU < n) ? kn + kU : kn;
#else
#pragma unroll
      for (int u = 0; u < kU; ++u) nxt[u] = load_raw<T, FULL>(client_base(ptrs[kn + u], sb, zeros), e, count);
#endif
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const int kk = k + u;
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the low weights of kk
        __builtin_amdgcn_sched_barrier(0);
        double whi[H];
#pragma unroll
        for (int j = 0; j < H; ++j) whi[j] = wk[H + j];
#if PERS_PTR_AHEAD
        if (u == 0) {
#pragma unroll
          for (int q = 0; q < kU; ++q) pn[q] = ptrs[kn2 + q];
        }
#endif
        __builtin_amdgcn_sched_barrier(0);
        double x[kVE];
        R::expand(cur[u], x);
        // (fp64 inputs keep the plain order: their raw slices leave no registers for the products)
        fold_half<FOLD, 0, H, true, !std::is_same<T, double>::value>(acc, x, wlo);
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the high weights of kk
        __builtin_amdgcn_sched_barrier(0);
        const kp<double> w1 = kk + 1 < n ? wk + wstep : wk;
#pragma unroll
        for (int j = 0; j < H; ++j) wlo[j] = w1[j];
        __builtin_amdgcn_sched_barrier(0);
        fold_half<FOLD, H, H, PERS_PTR_AHEAD != 0, !std::is_same<T, double>::value>(acc, x, whi);
        __builtin_amdgcn_sched_barrier(0);
        wk = w1;
      }
    }
  }

  bool in[kVE];
#pragma unroll
  for (int v = 0; v < kVE; ++v) in[v] = e + v < count;
  // refold (rare): elements whose sum is ±0 or NaN are recomputed with the skipped pairs
  // skipped, giving the reference's exact sign of zero / its NaN-or-not verdict. One receiver
  // at a time, so the rare path adds no register pressure to the main loop.
  const kp<int32_t> exm = (kp<int32_t>)(a.exmask);
#pragma unroll
  for (int j = 0; j < kJB; ++j) {
    bool f[kVE], any = false;
#pragma unroll
    for (int v = 0; v < kVE; ++v) {
      f[v] = in[v] && zero_or_nan(acc[v][j]);
      any |= f[v];
    }
    if (__ballot(any) == 0ull) continue;
    double b[kVE];
#pragma unroll
    for (int v = 0; v < kVE; ++v) b[v] = -0.0;
    for (int k = 0; k < a.N; ++k) {
      const uint64_t p = ptrs[k];
      if (!p) continue;  // absent tensor: nobody folds it
      if ((static_cast<uint32_t>(exm[static_cast<int64_t>(k) * a.waves + wave]) >> j) & 1u) continue;  // own update
      double x[kVE];
      R::expand(load_raw<T, FULL>(p + sb, e, count), x);
      const double wj = wt[static_cast<int64_t>(k) * a.wstride + j];
#pragma unroll
      for (int v = 0; v < kVE; ++v) b[v] = pfold<FOLD>(b[v], x[v], wj);
    }
#pragma unroll
    for (int v = 0; v < kVE; ++v)
      if (f[v]) acc[v][j] = b[v];
  }

  // epilogue: out_j = acc_j / W_j with the fused NaN assertions (fed_avg_algorithm.py:92-97);
  // the quotients stay in acc for the centralized average
  bool bad_acc = false, bad_res = false;
  const kp<double> wtot = (kp<double>)(a.wtot);
  const kp<uint64_t> outs = (kp<uint64_t>)(a.outs);
#pragma unroll
  for (int j = 0; j < kJB; ++j) {
    if (j0 + j >= a.M) continue;  // (continue, not break: keeps the loop fully unrolled)
    const int64_t wi = static_cast<int64_t>(j0 + j) * a.T + seg;
    const double W = wtot[wi];
    const double Wy = ((kp<double>)(a.wrcp))[wi];
    double r[kVE], s[kVE];
#pragma unroll
    for (int v = 0; v < kVE; ++v) {
      bad_acc |= in[v] && acc[v][j] != acc[v][j];
      s[v] = acc[v][j];
    }
    exact_div_block_rcp<kVE>(s, r, W, Wy);
#pragma unroll
    for (int v = 0; v < kVE; ++v) {
      acc[v][j] = r[v];
      bad_res |= in[v] && r[v] != r[v];
    }
    store_result<FULL>(outs[static_cast<int64_t>(j0 + j) * a.T + seg], start, e, count, a.out_f32, r);
  }
  if (__ballot(bad_acc) != 0ull && lane == 0) pflag(a.flag, 0);
  if (__ballot(bad_res) != 0ull && lane == 0) pflag(a.flag, 1);
  if (a.central_mode == CENTRAL_NONE) return;

  // centralized model: fold round(out_j * cw) over receivers in key order; wave w continues
  // the chain of wave w-1 through LDS (weighted_avg, aggregation_algorithm.py:63-72)
  const int64_t coff = a.seg_off[seg] + start + e;
  for (int s = 0; s < a.waves; ++s) {
    if (wave == s) {
      double c[kVE];
#pragma unroll
      for (int v = 0; v < kVE; ++v) {
        if (s > 0) {
          c[v] = chain[lane * kVE + v];
        } else if (a.central_in) {
          c[v] = in[v] ? a.carry[coff + v] : -0.0;
        } else {
          c[v] = -0.0;
        }
      }
#pragma unroll
      for (int j = 0; j < kJB; ++j) {
        if (j0 + j >= a.M) continue;
#pragma unroll
        for (int v = 0; v < kVE; ++v) {
          const double d = acc[v][j] * a.cw;  // v.to(float64) * weight   (:65-68)
          c[v] = c[v] + d;                    // avg_data[k] += d[k]       (:72)
        }
      }
      if (s + 1 < a.waves) {
#pragma unroll
        for (int v = 0; v < kVE; ++v) chain[lane * kVE + v] = c[v];
      } else if (a.central_mode == CENTRAL_CARRY_OUT) {
#pragma unroll
        for (int v = 0; v < kVE; ++v)
          if (in[v]) a.carry[coff + v] = c[v];
      } else {
        bool bad = false;  // (:73-74)
#pragma unroll
        for (int v = 0; v < kVE; ++v) bad |= in[v] && c[v] != c[v];
        if (__ballot(bad) != 0ull && lane == 0) pflag(a.flag, 2);
        store_result<false>(((kp<uint64_t>)(a.central))[seg], start, e, count, a.central_f32, c);
      }
    }
    if (s + 1 < a.waves) __syncthreads();
  }
}

// RING: the fused fold of whole aligned fp32 / fp64 chunks streams through the LDS ring (opt-in,
// its own instantiation so the default register pipeline's allocation is its own)
template <typename T, int FOLD, bool RING = false>
// three waves per SIMD (<= 168 VGPRs): the fold hides its load latency across waves
__global__ __launch_bounds__(64 * kMaxWaves) __attribute__((amdgpu_waves_per_eu(3))) void personalized_kernel(PArgs a) {
  // dynamic LDS: the centralized chain (64 x kVE doubles), then the client ring (fp32 / fp64)
  extern __shared__ __attribute__((aligned(16))) double smem[];
  double* chain = smem;
  char* ring = reinterpret_cast<char*>(smem + 64 * kVE);
  const int wave = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x) >> 6);
  const int lane = threadIdx.x & 63;
  const kp<int32_t> cd = (kp<int32_t>)(a.chunks + blockIdx.x);
  const int seg = cd[0];
  const int count = cd[1];
  const int64_t start = ((kp<int64_t>)(a.chunks + blockIdx.x))[1];
  if (count == kChunk && a.aligned) {
    if constexpr (RING && kHasGlds<T> && FOLD == PF_FMA) {
      pers_body<T, FOLD, true, true>(a, wave, lane, seg, count, start, chain, ring);
    } else {
      pers_body<T, FOLD, true, false>(a, wave, lane, seg, count, start, chain, ring);
    }
  } else {
    pers_body<T, FOLD, false, false>(a, wave, lane, seg, count, start, chain, ring);
  }
}

// fp64 VALU ceiling probe (the roofline this kernel is priced against): every lane runs
// `iters` dependent-free chains of v_fma_f64.
__global__ __launch_bounds__(256) void fp64_fma_probe(double* out, int iters) {
  double a0 = threadIdx.x * 1e-9, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5,
         a6 = a0 + 6, a7 = a0 + 7;
  const double m = 0.999999, c = 1e-7;
  for (int i = 0; i < iters; ++i) {
    a0 = __builtin_fma(a0, m, c); a1 = __builtin_fma(a1, m, c); a2 = __builtin_fma(a2, m, c);
    a3 = __builtin_fma(a3, m, c); a4 = __builtin_fma(a4, m, c); a5 = __builtin_fma(a5, m, c);
    a6 = __builtin_fma(a6, m, c); a7 = __builtin_fma(a7, m, c);
  }
  const double s = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
  if (s == 12345.678) out[blockIdx.x] = s;  // keeps the chains live
}

int32_t elem_size(int32_t dt) {
  switch (dt) {
    case FEDAVG_F32: return 4;
    case FEDAVG_F16: return 2;
    case FEDAVG_BF16: return 2;
    case FEDAVG_F64: return 8;
    default: return 0;
  }
}

int32_t sig_bits(int32_t dt) {
  switch (dt) {
    case FEDAVG_F32: return 24;
    case FEDAVG_F16: return 11;
    case FEDAVG_BF16: return 8;
    default: return 53;
  }
}

// Significand width of a weight; -1 when a product with it could over/underflow or is not
// finite (then the separately rounded fold is used).
int weight_bits(double w) {
  if (w == 0.0) return 0;
  if (!std::isfinite(w)) return -1;
  int ex = 0;
  const double m = std::frexp(std::fabs(w), &ex);
  if (ex < -800 || ex > 800) return -1;
  const uint64_t bits = static_cast<uint64_t>(std::ldexp(m, 53));
  return 53 - __builtin_ctzll(bits);
}

constexpr size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

}  // namespace

struct fedavg_pers {
  int device = 0;
  int T = 0;
  std::vector<int64_t> seg_numel, seg_off;
  int64_t P = 0;
  std::vector<PChunk> chunks;
  PChunk* d_chunks = nullptr;
  int64_t* d_seg_off = nullptr;
  double* d_carry = nullptr;
  uint32_t* h_flag = nullptr;
  uint32_t* d_flag = nullptr;
  // per-call table staging: pinned host image + device copy, reused once the previous
  // call's copy has completed
  char* h_blob = nullptr;
  char* d_blob = nullptr;
  size_t blob_cap = 0;
  hipEvent_t blob_done = nullptr;
  bool blob_used = false;
  bool allow_fma = true;
  bool ring = false;  // FEDAVG_PERS_RING=1: the fused fold of whole fp32 / fp64 chunks streams through the LDS ring
  bool prof = false;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> prof_events;
};

namespace {

template <typename T>
hipError_t launch_pers_t(const PArgs& a, int fold, int nchunks, int threads, size_t lds, hipStream_t s) {
  if (fold == PF_FMA) {
    if constexpr (kHasGlds<T>) {
      if (a.ring) {
        hipLaunchKernelGGL((personalized_kernel<T, PF_FMA, true>), dim3(nchunks), dim3(threads), lds, s, a);
        return hipGetLastError();
      }
    }
    hipLaunchKernelGGL((personalized_kernel<T, PF_FMA>), dim3(nchunks), dim3(threads), lds, s, a);
  } else {
    hipLaunchKernelGGL((personalized_kernel<T, PF_MULADD>), dim3(nchunks), dim3(threads), lds, s, a);
  }
  return hipGetLastError();
}

hipError_t launch_pers(int32_t dt, const PArgs& a, int fold, int nchunks, int threads, size_t lds, hipStream_t s) {
  switch (dt) {
    case FEDAVG_F32: return launch_pers_t<float>(a, fold, nchunks, threads, lds, s);
    case FEDAVG_F16: return launch_pers_t<__half>(a, fold, nchunks, threads, lds, s);
    case FEDAVG_BF16: return launch_pers_t<bf16_t>(a, fold, nchunks, threads, lds, s);
    case FEDAVG_F64: return launch_pers_t<double>(a, fold, nchunks, threads, lds, s);
    default: return hipErrorInvalidValue;
  }
}

int32_t check_pers(const fedavg_pers* p) {
  if (p == nullptr) return pfail(FEDAVG_ERR_INVALID, "null personalized context");
  return FEDAVG_OK;
}

}  // namespace

// Geometry constants for fedavg_kernel_constant ("pers_*" names; test support).
extern "C" __attribute__((visibility("hidden"))) int32_t fedavg_internal_pers_constant(const char* name,
                                                                                      int64_t* out) {
  const std::string n(name);
  if (n == "pers_chunk") *out = kChunk;
  else if (n == "pers_jb") *out = kJB;
  else if (n == "pers_group") *out = kGroup;
  else if (n == "pers_u") *out = kU;
  else if (n == "pers_ring_stage") *out = kSC;
  else if (n == "pers_ring_depth") *out = kD;
  else return FEDAVG_ERR_INVALID;
  return FEDAVG_OK;
}

extern "C" {

int32_t fedavg_pers_create(fedavg_pers** out, int32_t device, const int64_t* seg_numel, int32_t num_segments) {
  if (out == nullptr) return pfail(FEDAVG_ERR_INVALID, "null out");
  *out = nullptr;
  if (num_segments <= 0 || seg_numel == nullptr) return pfail(FEDAVG_ERR_INVALID, "no segments");
  for (int t = 0; t < num_segments; ++t)
    if (seg_numel[t] <= 0 || seg_numel[t] > (int64_t(1) << 40))
      return pfail(FEDAVG_ERR_INVALID, "bad segment size");
  PERS_HIP_TRY(hipSetDevice(device));
  fedavg_pers* p = new fedavg_pers();
  p->device = device;
  p->T = num_segments;
  if (const char* e = std::getenv("FEDAVG_PERS_RING")) p->ring = std::strcmp(e, "0") != 0;
  p->seg_numel.assign(seg_numel, seg_numel + num_segments);
  p->seg_off.resize(num_segments);
  for (int t = 0; t < num_segments; ++t) {
    p->seg_off[t] = p->P;
    p->P += seg_numel[t];
    for (int64_t s = 0; s < seg_numel[t]; s += kChunk)
      p->chunks.push_back(PChunk{t, static_cast<int32_t>(std::min<int64_t>(kChunk, seg_numel[t] - s)), s});
  }
  if (p->chunks.size() > static_cast<size_t>(INT32_MAX)) {
    delete p;
    return pfail(FEDAVG_ERR_INVALID, "layout too large");
  }
  auto cleanup = [&](hipError_t e, const char* what) {
    fedavg_pers_destroy(p);
    return pfail(FEDAVG_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
  };
  hipError_t e;
  if ((e = hipMalloc(reinterpret_cast<void**>(&p->d_chunks), sizeof(PChunk) * p->chunks.size())) != hipSuccess)
    return cleanup(e, "hipMalloc chunks");
  if ((e = hipMalloc(reinterpret_cast<void**>(&p->d_seg_off), sizeof(int64_t) * num_segments)) != hipSuccess)
    return cleanup(e, "hipMalloc seg_off");
  if ((e = hipMemcpy(p->d_chunks, p->chunks.data(), sizeof(PChunk) * p->chunks.size(), hipMemcpyHostToDevice)) != hipSuccess)
    return cleanup(e, "hipMemcpy chunks");
  if ((e = hipMemcpy(p->d_seg_off, p->seg_off.data(), sizeof(int64_t) * num_segments, hipMemcpyHostToDevice)) != hipSuccess)
    return cleanup(e, "hipMemcpy seg_off");
  if ((e = hipHostMalloc(reinterpret_cast<void**>(&p->h_flag), sizeof(uint32_t) * 4,
                         hipHostMallocMapped | hipHostMallocCoherent)) != hipSuccess)
    return cleanup(e, "hipHostMalloc flag");
  if ((e = hipHostGetDevicePointer(reinterpret_cast<void**>(&p->d_flag), p->h_flag, 0)) != hipSuccess)
    return cleanup(e, "hipHostGetDevicePointer flag");
  std::memset(p->h_flag, 0, sizeof(uint32_t) * 4);
  if ((e = hipEventCreateWithFlags(&p->blob_done, hipEventDisableTiming)) != hipSuccess)
    return cleanup(e, "hipEventCreate");
  *out = p;
  return FEDAVG_OK;
}

int32_t fedavg_pers_destroy(fedavg_pers* p) {
  if (p == nullptr) return FEDAVG_OK;
  (void)hipSetDevice(p->device);
  (void)hipDeviceSynchronize();
  for (auto& pr : p->prof_events) {
    (void)hipEventDestroy(pr.first);
    (void)hipEventDestroy(pr.second);
  }
  if (p->blob_done) (void)hipEventDestroy(p->blob_done);
  if (p->h_blob) (void)hipHostFree(p->h_blob);
  if (p->d_blob) (void)hipFree(p->d_blob);
  if (p->d_chunks) (void)hipFree(p->d_chunks);
  if (p->d_seg_off) (void)hipFree(p->d_seg_off);
  if (p->d_carry) (void)hipFree(p->d_carry);
  if (p->h_flag) (void)hipHostFree(p->h_flag);
  delete p;
  return FEDAVG_OK;
}

int32_t fedavg_pers_set_fused_fold(fedavg_pers* p, int32_t enable) {
  PERS_RET(check_pers(p));
  p->allow_fma = enable != 0;
  return FEDAVG_OK;
}

int32_t fedavg_pers_aggregate(fedavg_pers* p, const void* const* client_ptrs, int32_t in_dtype, int32_t N,
                              const int64_t* client_ids, const double* weights, const int64_t* receiver_ids,
                              int32_t M, void* const* out_ptrs, int32_t out_dtype, void* const* central_ptrs,
                              int32_t central_dtype, void* stream) {
  PERS_RET(check_pers(p));
  const int T = p->T;
  if (N <= 0 || M <= 0) return pfail(FEDAVG_ERR_INVALID, "need at least one client and one receiver");
  if (!client_ptrs || !client_ids || !weights || !receiver_ids || !out_ptrs)
    return pfail(FEDAVG_ERR_INVALID, "null table");
  if (elem_size(in_dtype) == 0) return pfail(FEDAVG_ERR_INVALID, "bad input dtype");
  if (out_dtype != FEDAVG_F32 && out_dtype != FEDAVG_F64)
    return pfail(FEDAVG_ERR_INVALID, "out dtype must be FEDAVG_F32 or FEDAVG_F64");
  if (central_ptrs && central_dtype != FEDAVG_F32 && central_dtype != FEDAVG_F64)
    return pfail(FEDAVG_ERR_INVALID, "central dtype must be FEDAVG_F32 or FEDAVG_F64");
  for (int j = 0; j < M; ++j)
    for (int i = 0; i < j; ++i)
      if (receiver_ids[i] == receiver_ids[j]) return pfail(FEDAVG_ERR_INVALID, "duplicate receiver id");
  bool aligned = true;
  const size_t in_align = std::min<size_t>(16, static_cast<size_t>(elem_size(in_dtype)) * kVE);
  for (int64_t i = 0; i < static_cast<int64_t>(M) * T; ++i) {
    if (!out_ptrs[i]) return pfail(FEDAVG_ERR_INVALID, "null output pointer");
    if (reinterpret_cast<uintptr_t>(out_ptrs[i]) % 16 != 0) aligned = false;
  }
  for (int64_t i = 0; i < static_cast<int64_t>(N) * T; ++i)
    if (client_ptrs[i] && reinterpret_cast<uintptr_t>(client_ptrs[i]) % in_align != 0) aligned = false;
  if (central_ptrs)
    for (int t = 0; t < T; ++t)
      if (!central_ptrs[t]) return pfail(FEDAVG_ERR_INVALID, "null centralized output pointer");

  // receiver j folds arrival k unless it is j's own update (:31-32); per-receiver, per-segment
  // totals in arrival order (fed_avg_algorithm.py:59-62); the fused-fold proof (every folded
  // product exact in fp64)
  std::vector<int32_t> excl(N, -1);  // the receiver that skips arrival k (ids are unique)
  for (int k = 0; k < N; ++k)
    for (int j = 0; j < M; ++j)
      if (receiver_ids[j] == client_ids[k]) excl[k] = j;
  // sums start at -0.0, the additive identity: the first weight is taken as is (python `= w`)
  std::vector<double> wtot(static_cast<size_t>(M) * T, -0.0);
  std::vector<uint8_t> have(static_cast<size_t>(M) * T, 0);
  bool all_whole = true;  // every client sent every tensor (the server complete()s messages)
  for (int64_t i = 0; i < static_cast<int64_t>(N) * T && all_whole; ++i) all_whole = client_ptrs[i] != nullptr;
  int max_bits = 0;
  bool tame = true;
  std::vector<double> run(M, -0.0);  // all_whole: one arrival-order sum per receiver
  std::vector<uint8_t> any(M, 0);
  for (int k = 0; k < N; ++k) {
    for (int j = 0; j < M; ++j) {
      if (excl[k] == j) continue;
      const double w = weights[static_cast<int64_t>(j) * N + k];
      const int b = weight_bits(w);
      if (b < 0) tame = false;
      max_bits = std::max(max_bits, b);
      if (all_whole) {
        run[j] += w;
        any[j] = 1;
        continue;
      }
      for (int t = 0; t < T; ++t) {
        if (!client_ptrs[static_cast<int64_t>(k) * T + t]) continue;
        wtot[static_cast<size_t>(j) * T + t] += w;
        have[static_cast<size_t>(j) * T + t] = 1;
      }
    }
  }
  if (all_whole)
    for (int j = 0; j < M; ++j)
      for (int t = 0; t < T; ++t) {
        wtot[static_cast<size_t>(j) * T + t] = run[j];
        have[static_cast<size_t>(j) * T + t] = any[j];
      }
  for (int j = 0; j < M; ++j)
    for (int t = 0; t < T; ++t)
      if (!have[static_cast<size_t>(j) * T + t])
        return pfail(FEDAVG_ERR_STATE, "receiver " + std::to_string(j) + " has no data for segment " +
                                           std::to_string(t) + " (fed_avg_algorithm.py:88)");
  const int fold = (p->allow_fma && tame && sig_bits(in_dtype) + max_bits <= 53) ? PF_FMA : PF_MULADD;

  // one blob: [T][Npad] pointers; per receiver group g: [Npad][waves*16] weights, [N][waves]
  // skip masks, [kGroup][T] totals, [kGroup][T] outputs; then [T] centralized outputs and
  // the zero block
  const int G = (M + kGroup - 1) / kGroup;
  // a multiple of the register group (kU) and of a ring stage (kSC), both powers of two
  constexpr int kPad = kU > kSC ? kU : kSC;
  static_assert((kPad & (kPad - 1)) == 0 && kPad % kU == 0 && kPad % kSC == 0, "padding unit");
  const int Npad = (N + kPad - 1) / kPad * kPad;
  const size_t off_ptr = 0;
  const size_t sz_ptr = align_up(sizeof(void*) * T * Npad, 256);
  const size_t sz_w = align_up(sizeof(double) * Npad * kGroup, 256);
  const size_t sz_x = align_up(sizeof(int32_t) * N * kMaxWaves, 256);
  const size_t sz_t = align_up(sizeof(double) * kGroup * T, 256);
  const size_t sz_o = align_up(sizeof(void*) * kGroup * T, 256);
  const size_t per_g = sz_w + sz_x + sz_t + sz_o + sz_t;  // ... then the reciprocals of the totals
  const size_t off_g = off_ptr + sz_ptr;
  const size_t off_c = off_g + per_g * G;
  const size_t off_z = off_c + align_up(sizeof(void*) * T, 256);
  const size_t bytes = off_z + sizeof(double) * kChunk;

  PERS_HIP_TRY(hipSetDevice(p->device));
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (p->blob_used) PERS_HIP_TRY(hipEventSynchronize(p->blob_done));
  if (p->blob_cap < bytes) {
    if (p->h_blob) PERS_HIP_TRY(hipHostFree(p->h_blob));
    if (p->d_blob) {
      PERS_HIP_TRY(hipStreamSynchronize(s));
      PERS_HIP_TRY(hipFree(p->d_blob));
    }
    p->h_blob = nullptr;
    p->d_blob = nullptr;
    p->blob_cap = 0;
    const size_t cap = std::max<size_t>(bytes * 2, 64 * 1024);
    PERS_HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&p->h_blob), cap, hipHostMallocDefault));
    PERS_HIP_TRY(hipMalloc(reinterpret_cast<void**>(&p->d_blob), cap));
    p->blob_cap = cap;
  }
  char* h = p->h_blob;
  std::memset(h, 0, bytes);
  const void** hp = reinterpret_cast<const void**>(h + off_ptr);
  for (int t = 0; t < T; ++t)
    for (int k = 0; k < N; ++k) hp[static_cast<size_t>(t) * Npad + k] = client_ptrs[static_cast<int64_t>(k) * T + t];
  for (int g = 0; g < G; ++g) {
    char* b = h + off_g + per_g * g;
    double* hw = reinterpret_cast<double*>(b);
    int32_t* hx = reinterpret_cast<int32_t*>(b + sz_w);
    double* ht = reinterpret_cast<double*>(b + sz_w + sz_x);
    void** ho = reinterpret_cast<void**>(b + sz_w + sz_x + sz_t);
    double* hy = reinterpret_cast<double*>(b + sz_w + sz_x + sz_t + sz_o);
    const int Mg = std::min(kGroup, M - g * kGroup);
    const int waves = (Mg + kJB - 1) / kJB;
    const int wstride = kJB * waves;
    for (int k = 0; k < N; ++k) {
      for (int r = 0; r < Mg; ++r) {
        const int j = g * kGroup + r;
        if (excl[k] == j) {
          hx[static_cast<size_t>(k) * waves + r / kJB] |= 1 << (r % kJB);  // weight stays 0
        } else {
          hw[static_cast<size_t>(k) * wstride + r] = weights[static_cast<int64_t>(j) * N + k];
        }
      }
    }
    for (int r = 0; r < Mg; ++r)
      for (int t = 0; t < T; ++t) {
        const int j = g * kGroup + r;
        ht[static_cast<size_t>(r) * T + t] = wtot[static_cast<size_t>(j) * T + t];
        hy[static_cast<size_t>(r) * T + t] = 1.0 / wtot[static_cast<size_t>(j) * T + t];
        ho[static_cast<size_t>(r) * T + t] = out_ptrs[static_cast<int64_t>(j) * T + t];
      }
  }
  if (central_ptrs) {
    void** hc = reinterpret_cast<void**>(h + off_c);
    for (int t = 0; t < T; ++t) hc[t] = central_ptrs[t];
  }
  PERS_HIP_TRY(hipMemcpyAsync(p->d_blob, h, bytes, hipMemcpyHostToDevice, s));
  PERS_HIP_TRY(hipEventRecord(p->blob_done, s));
  p->blob_used = true;
  if (central_ptrs && G > 1 && !p->d_carry)
    PERS_HIP_TRY(hipMalloc(reinterpret_cast<void**>(&p->d_carry), sizeof(double) * p->P));

  const int nchunks = static_cast<int>(p->chunks.size());
  for (int g = 0; g < G; ++g) {
    char* b = p->d_blob + off_g + per_g * g;
    PArgs a;
    a.chunks = p->d_chunks;
    a.cptrs = reinterpret_cast<const void* const*>(p->d_blob + off_ptr);
    a.w = reinterpret_cast<const double*>(b);
    a.exmask = reinterpret_cast<const int32_t*>(b + sz_w);
    a.wtot = reinterpret_cast<const double*>(b + sz_w + sz_x);
    a.outs = reinterpret_cast<void* const*>(b + sz_w + sz_x + sz_t);
    a.wrcp = reinterpret_cast<const double*>(b + sz_w + sz_x + sz_t + sz_o);
    a.central = reinterpret_cast<void* const*>(p->d_blob + off_c);
    a.zeros = p->d_blob + off_z;
    a.carry = p->d_carry;
    a.seg_off = p->d_seg_off;
    a.flag = p->d_flag;
    a.N = N;
    a.Npad = Npad;
    a.T = T;
    a.aligned = aligned;
    a.M = std::min(kGroup, M - g * kGroup);
    a.waves = (a.M + kJB - 1) / kJB;
    a.wstride = kJB * a.waves;
    a.out_f32 = out_dtype == FEDAVG_F32;
    a.central_mode = !central_ptrs ? CENTRAL_NONE : (g + 1 < G ? CENTRAL_CARRY_OUT : CENTRAL_FINAL);
    a.central_in = g > 0;
    a.central_f32 = central_dtype == FEDAVG_F32;
    a.cw = 1.0 / static_cast<double>(M);
    const int threads = 64 * a.waves;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (p->prof) {
      PERS_HIP_TRY(hipEventCreate(&e0));
      PERS_HIP_TRY(hipEventCreate(&e1));
      PERS_HIP_TRY(hipEventRecord(e0, s));
    }
    // the LDS ring (whole aligned fp32 / fp64 chunks, fused fold only) is opt-in: with round 4's
    // register pipeline (split weight halves, incremental rows) the integer-weight round runs
    // 2.78 ms median (2.74-2.99) there against 2.89-3.40 ms medians (2.71-3.43) on the ring,
    // interleaved on one box (profiles/r04_pers_ring_vs_regs.txt)
    a.ring = p->ring && fold == PF_FMA && (in_dtype == FEDAVG_F32 || in_dtype == FEDAVG_F64);
    const size_t slice = static_cast<size_t>(kChunk) * (in_dtype == FEDAVG_F64 ? 8 : 4);
    const size_t lds = sizeof(double) * 64 * kVE +
                       (a.ring ? kRS * kSC * slice : 0);
    const hipError_t err = launch_pers(in_dtype, a, fold, nchunks, threads, lds, s);
    if (err != hipSuccess) return pfail(FEDAVG_ERR_HIP, std::string("kernel launch: ") + hipGetErrorString(err));
    if (p->prof) {
      PERS_HIP_TRY(hipEventRecord(e1, s));
      p->prof_events.emplace_back(e0, e1);
    }
  }
  return FEDAVG_OK;
}

int32_t fedavg_pers_check(fedavg_pers* p, void* stream, uint32_t* flags_out) {
  PERS_RET(check_pers(p));
  PERS_HIP_TRY(hipSetDevice(p->device));
  PERS_HIP_TRY(hipStreamSynchronize(static_cast<hipStream_t>(stream)));
  uint32_t f = 0;
  if (__atomic_load_n(&p->h_flag[0], __ATOMIC_ACQUIRE)) f |= FEDAVG_FLAG_ACC_NAN;
  if (__atomic_load_n(&p->h_flag[1], __ATOMIC_ACQUIRE)) f |= FEDAVG_FLAG_RESULT_NAN;
  if (__atomic_load_n(&p->h_flag[2], __ATOMIC_ACQUIRE)) f |= FEDAVG_FLAG_CENTRAL_NAN;
  std::memset(p->h_flag, 0, sizeof(uint32_t) * 4);
  if (flags_out) *flags_out = f;
  if (f & FEDAVG_FLAG_ACC_NAN) return pfail(FEDAVG_ERR_NAN_ACCUM, "NaN in a receiver's accumulator");
  if (f & FEDAVG_FLAG_RESULT_NAN) return pfail(FEDAVG_ERR_NAN_RESULT, "NaN in a receiver's result");
  if (f & FEDAVG_FLAG_CENTRAL_NAN) return pfail(FEDAVG_ERR_NAN_RESULT, "NaN in the centralized model");
  return FEDAVG_OK;
}

int32_t fedavg_pers_prof_enable(fedavg_pers* p, int32_t enable) {
  PERS_RET(check_pers(p));
  p->prof = enable != 0;
  return FEDAVG_OK;
}

int32_t fedavg_pers_prof_collect(fedavg_pers* p, double* total_ms, int32_t* launches) {
  PERS_RET(check_pers(p));
  double sum = 0.0;
  for (auto& pr : p->prof_events) {
    PERS_HIP_TRY(hipEventSynchronize(pr.second));
    float ms = 0.f;
    PERS_HIP_TRY(hipEventElapsedTime(&ms, pr.first, pr.second));
    sum += ms;
    (void)hipEventDestroy(pr.first);
    (void)hipEventDestroy(pr.second);
  }
  if (total_ms) *total_ms = sum;
  if (launches) *launches = static_cast<int32_t>(p->prof_events.size());
  p->prof_events.clear();
  return FEDAVG_OK;
}

int32_t fedavg_fp64_probe(int64_t waves, int32_t iters, double* tflops_out, void* stream) {
  if (waves <= 0 || iters <= 0 || !tflops_out) return pfail(FEDAVG_ERR_INVALID, "bad probe arguments");
  hipStream_t s = static_cast<hipStream_t>(stream);
  double* d = nullptr;
  const int blocks = static_cast<int>((waves + 3) / 4);
  PERS_HIP_TRY(hipMalloc(reinterpret_cast<void**>(&d), sizeof(double) * blocks));
  hipEvent_t e0, e1;
  PERS_HIP_TRY(hipEventCreate(&e0));
  PERS_HIP_TRY(hipEventCreate(&e1));
  hipLaunchKernelGGL(fp64_fma_probe, dim3(blocks), dim3(256), 0, s, d, iters);  // warm-up
  PERS_HIP_TRY(hipEventRecord(e0, s));
  hipLaunchKernelGGL(fp64_fma_probe, dim3(blocks), dim3(256), 0, s, d, iters);
  PERS_HIP_TRY(hipEventRecord(e1, s));
  PERS_HIP_TRY(hipEventSynchronize(e1));
  float ms = 0.f;
  PERS_HIP_TRY(hipEventElapsedTime(&ms, e0, e1));
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  (void)hipFree(d);
  *tflops_out = 2.0 * 8.0 * static_cast<double>(iters) * 256.0 * blocks / (ms * 1e-3) / 1e12;
  return FEDAVG_OK;
}

}  // extern "C"
