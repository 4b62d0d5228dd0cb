// fedavg_kernels.hip — gfx950 (MI355X) kernels of the server-side weighted FedAvg reduce.
//
// What the reference computes (simulation_lib/algorithm/fed_avg_algorithm.py:43-99):
//   for every arriving client k, for every named tensor t:
//       tmp = x_k[t].to(float64) * w_k          (:54)
//       acc[t] = tmp            if first else acc[t] += tmp   (:55-58)
//       W[t]  += w_k                                         (:59-62)
//   at the end: assert !isnan(acc[t]); out[t] = acc[t] / W[t]; assert !isnan(out[t]) (:92-97)
//
// How it is laid out here:
//   * A model is T segments (its named tensors). Every segment is cut into tiles of TILE
//     elements (never crossing a segment). One workgroup owns one tile and streams that
//     tile's slice of every client bucket from HBM, 16 B per lane per load, CU_LOADS clients
//     in flight per lane, accumulating in fp64 registers in client order. The fp64 product
//     and the fp64 sum are separately rounded (-ffp-contract=off), so each element's value
//     is bit-identical to the reference's torch CPU ops.
//   * SPLIT=4 variant (small-P / large-N shapes): the four waves of a workgroup take four
//     contiguous client ranges of the same 512-element tile; wave partials are staged in LDS
//     and wave 0 combines them in wave order (deterministic, but a different fp64 order).
//   * The NaN assertions are fused: one isnan per accumulated element, a wavefront ballot,
//     and one atomicOr per wave that saw a NaN.
//   * No MFMA: 0.25-0.5 flop per byte, the kernel is HBM-bound.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <hip/hip_fp16.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <mutex>
#include <string>
#include <type_traits>
#include <vector>

#include "../../include/fedavg_hip.h"
#include "exact_div.h"

namespace {

// ---------------------------------------------------------------------------------------
// error plumbing
// ---------------------------------------------------------------------------------------
thread_local std::string g_last_error;

int32_t fail(int32_t code, const std::string& msg) {
  g_last_error = msg;
  return code;
}

#define FEDAVG_HIP_TRY(expr)                                                              \
  do {                                                                                    \
    hipError_t e_ = (expr);                                                               \
    if (e_ != hipSuccess) {                                                               \
      return fail(FEDAVG_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_));     \
    }                                                                                     \
  } while (0)

// ---------------------------------------------------------------------------------------
// device-side descriptors
// ---------------------------------------------------------------------------------------
constexpr int kThreads = 256;     // 4 waves of 64 (split kernel, probes)
// Tuning knobs (compile-time; the shipped values were picked on MI355X by
// scripts/tune_kernel.py, see DESIGN.md "Kernel tuning"):
//   FEDAVG_AE        elements owned by one lane (= fp64 accumulators per lane)
//   FEDAVG_CU_BYTES  bytes of client loads in flight per lane per group
// Client loads and result stores are non-temporal (measured on MI355X, 64 x ResNet-18 fp32 ->
// fp32, interleaved A/B in one process: nt loads ~+1-2 %, nt stores +5-9 % — a read stream with
// interleaved writes loses HBM efficiency; nt stores cut that); AE 16 / CU 512 B +-1 %, load
// fence / 128-512-thread groups / fused fold within noise.
#ifndef FEDAVG_AE
#define FEDAVG_AE 16
#endif
#ifndef FEDAVG_AE_HALF  // elements per lane for 2-byte inputs (fp16 / bf16): 16 = two 16-B loads
// per client per lane, 512-lane wide tiles (interleaved A/B on MI355X against 8: 64 x ResNet-18
// fp16 one launch 0.2643 -> 0.2472 / 0.2644 -> 0.2488 ms on two boxes, 128 x GPT-2 fp16 one
// launch 5.420 -> 5.295 / 5.223 -> 5.192 ms, GPT-2 waves of 32 +0.2-0.4 %, ResNet-18 bf16 waves
// of 16 -1 %; 32 elements per lane and 96 / 128-B pipeline stages mixed)
#define FEDAVG_AE_HALF 16
#endif
#ifndef FEDAVG_AE_F64  // elements per lane for fp64 inputs (8: 512-lane tiles, see CU_BYTES_F64)
#define FEDAVG_AE_F64 8
#endif
#ifndef FEDAVG_TILE1  // elements per tile of the exact-order kernel (all dtypes)
#define FEDAVG_TILE1 4096
#endif
#ifndef FEDAVG_CU_BYTES
#define FEDAVG_CU_BYTES 256
#endif
#ifndef FEDAVG_CU_BYTES_F64  // the same for fp64 inputs: 8 clients x 64 B in flight per lane
// (64 x ResNet-18 fp64, interleaved A/B: AE 8 / 512 B 0.898-0.915 ms vs AE 16 / 256 B
// 0.974-0.984 ms; AE 8 / 768 B, AE 4, AE 32 and AE 16 / 512 B no better than the old default)
#define FEDAVG_CU_BYTES_F64 512
#endif
// Software-pipelined client loads (the next stage's loads issue before the current stage folds),
// one bit per input size: 1 = 2-byte, 2 = 4-byte, 4 = 8-byte. Interleaved A/B on MI355X
// (scripts/tune_kernel.py, 64-byte stages = 4 fp16 / bf16 clients): 64 x ResNet-18 fp16
// 0.2672 -> 0.2618 ms, bf16 0.2755 -> 0.2628 ms, 128 x GPT-2 fp16 5.443 -> 5.422 ms; 128 / 256-B
// stages no better; fp32 with 128 / 256-B stages 13 % / 10 % slower (kept grouped).
#ifndef FEDAVG_PIPE
#define FEDAVG_PIPE 1
#endif
#ifndef FEDAVG_ACC_PLAIN_STORE_HALF  // 2-byte inputs: the fp64 accumulator of a wave is stored with
// plain (not non-temporal) stores. Interleaved A/B on MI355X: 128 x GPT-2 fp16 in waves of 32
// 7.61 -> 6.84 ms (+11 %), 64 x ResNet-18 bf16 in waves of 16 +3.5 %, one-launch unchanged; the
// same for fp32 (all stores plain) cost ViT-B/16 waves 2.4 % (kept non-temporal there)
#define FEDAVG_ACC_PLAIN_STORE_HALF 1
#endif
#ifndef FEDAVG_BALANCE_DEFAULT  // balanced whole-layout tile orders (bit 0 fp32, bit 1 fp64); env FEDAVG_BALANCE
#define FEDAVG_BALANCE_DEFAULT 3
#endif
#ifndef FEDAVG_WALK_ALTERNATE  // streaming waves alternate their tile walk (env FEDAVG_WALK_ALTERNATE)
#define FEDAVG_WALK_ALTERNATE 1
#endif
#ifndef FEDAVG_PIPE_BYTES  // bytes of client loads per lane per pipeline stage
#define FEDAVG_PIPE_BYTES 64
#endif
constexpr int kAE = FEDAVG_AE;    // elements owned by one lane (fp64 accumulators per lane)
constexpr int kTile1 = FEDAVG_TILE1;          // 4096 elements, SPLIT = 1 (any dtype)
#ifndef FEDAVG_TILE_WIDE  // whole-layout exact-order launches of 2- and 4-byte inputs (0 = off)
#define FEDAVG_TILE_WIDE 8192
#endif
constexpr int kTileWide = FEDAVG_TILE_WIDE;
constexpr int kTile4 = (kThreads / 4) * kAE;  // 1024 elements, SPLIT = 4

struct TileDesc {
  int32_t seg;
  int32_t count;   // elements in this tile (== tile size except at a segment's end)
  int64_t start;   // first element, relative to the segment
};

struct SegDesc {
  int64_t acc_off;  // offset of the segment in the padded fp64 accumulator
  int64_t numel;
};

// Per-call table blob (device copy of a pinned staging slot). Segment-major so that the
// clients of one tile are contiguous for scalar loads.
struct CallTables {
  const void* const* cptrs;  // [T][K] compacted (non-null) client pointers
  const double* w;           // [T][K] weights
  const int32_t* kseg;       // [T] number of clients for the segment in this call
  const int32_t* acc_in;     // [T] 1 = accumulator holds data for the segment
  void* const* outs;         // [T] output pointers (final kernels)
  const double* wtot;        // [T] divisor (final kernels)
  const void* const* base;   // [T] fp64 base model (delta calls): x = base + delta
};

struct KArgs {
  const TileDesc* tiles;
  const SegDesc* segs;
  CallTables tab;
  double* acc;
  uint32_t* flag;
  int32_t tile_begin;
  int32_t num_tiles;   // tiles of this launch
  int32_t K;           // row stride of the [T][K] tables
  int32_t zero_init;   // start every segment at the identity -0.0, ignore acc_in (shard partials)
  int32_t walk_back;   // the first walk_back tiles of the launch are walked last to first
                       // (fedavg_ctx::walk_reverse); 0 = natural order
  const double* qtab;  // QSGD: [segments of the launch][K][256] |product| tables (qsgd_table_kernel)
  int32_t qtab_seg0;   // QSGD: the segment of qtab's first table row
  // Multi-device peer exchange (multi_device.cpp): a zero-initialised partial launch whose tiles
  // [win_edge[j], win_edge[j+1]) store into win_dst[j] (device j's receive slot for this device,
  // accumulator coordinates) instead of acc; win_n = G windows, NULL = not windowed.
  double* const* win_dst;
  const int32_t* win_edge;
  int32_t win_n;
  // Peer exchange, own window (COMB kernels): after this entry's zero-initialised chain, the
  // element's partials of the comb_n entries holding clients are summed in entry order from -0.0 —
  // comb_src[h] (device h's partial in this device's receive slot, accumulator coordinates), this
  // entry's own chain from registers at h == comb_self — then divided and stored like a final fold.
  const double* const* comb_src;
  int32_t comb_n;
  int32_t comb_self;
};

enum OutKind : int { OUT_ACC = 0, OUT_F32 = 1, OUT_F64 = 2 };

// Clang ext-vector types: builtin vector values, usable through address-space-qualified
// pointers (HIP's struct vector types are not).
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef double f64x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

// 16-byte vector of the input type
template <typename T>
struct Vec16;
template <>
struct Vec16<float> {
  using type = f32x4;
  static constexpr int n = 4;
};
template <>
struct Vec16<double> {
  using type = f64x2;
  static constexpr int n = 2;
};
template <>
struct Vec16<__half> {
  using type = u32x4;  // 8 halves
  static constexpr int n = 8;
};
struct bf16_t {
  uint16_t bits;
};
template <>
struct Vec16<bf16_t> {
  using type = u32x4;  // 8 bf16
  static constexpr int n = 8;
};

__device__ __forceinline__ double to_f64(float x) { return static_cast<double>(x); }
__device__ __forceinline__ double to_f64(double x) { return x; }
__device__ __forceinline__ double half_bits_to_f64(uint32_t h) {
  return static_cast<double>(__half2float(__ushort_as_half(static_cast<unsigned short>(h))));
}
__device__ __forceinline__ double bf16_bits_to_f64(uint32_t b) {
  return static_cast<double>(__uint_as_float(b << 16));
}

// Expand one 16-byte vector into Vec16<T>::n doubles.
template <typename T>
__device__ __forceinline__ void expand(const typename Vec16<T>::type& v, double* out);
template <>
__device__ __forceinline__ void expand<float>(const f32x4& v, double* o) {
  o[0] = v.x; o[1] = v.y; o[2] = v.z; o[3] = v.w;
}
template <>
__device__ __forceinline__ void expand<double>(const f64x2& v, double* o) {
  o[0] = v.x; o[1] = v.y;
}
template <>
__device__ __forceinline__ void expand<__half>(const u32x4& v, double* o) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    o[2 * i] = half_bits_to_f64(w[i] & 0xffffu);
    o[2 * i + 1] = half_bits_to_f64(w[i] >> 16);
  }
}
template <>
__device__ __forceinline__ void expand<bf16_t>(const u32x4& v, double* o) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    o[2 * i] = bf16_bits_to_f64(w[i] & 0xffffu);
    o[2 * i + 1] = bf16_bits_to_f64(w[i] >> 16);
  }
}

// scalar element load
template <typename T>
__device__ __forceinline__ double load_elem(const T* p, int64_t i);
template <>
__device__ __forceinline__ double load_elem<float>(const float* p, int64_t i) { return p[i]; }
template <>
__device__ __forceinline__ double load_elem<double>(const double* p, int64_t i) { return p[i]; }
template <>
__device__ __forceinline__ double load_elem<__half>(const __half* p, int64_t i) {
  return half_bits_to_f64(reinterpret_cast<const uint16_t*>(p)[i]);
}
template <>
__device__ __forceinline__ double load_elem<bf16_t>(const bf16_t* p, int64_t i) {
  return bf16_bits_to_f64(reinterpret_cast<const uint16_t*>(p)[i]);
}

// Address-space-qualified pointers. Client buffers and outputs are read and written through
// the global address space (saddr `global_load_dwordx4 v, v_off, s[base]`, never `flat_`);
// per-call tables are read through the constant address space, which makes every
// wave-uniform table read a scalar `s_load` (8 client pointers per s_load_dwordx16).
#define FEDAVG_AS_GLOBAL __attribute__((address_space(1)))
#define FEDAVG_AS_CONST __attribute__((address_space(4)))
template <typename T>
using gptr = T FEDAVG_AS_GLOBAL*;
template <typename T>
using kptr = const T FEDAVG_AS_CONST*;

template <typename T>
__device__ __forceinline__ gptr<const T> to_global(const void* p) {
  return (gptr<const T>)(p);
}
template <typename T>
__device__ __forceinline__ gptr<T> to_global_mut(void* p) {
  return (gptr<T>)(p);
}
template <typename T>
__device__ __forceinline__ kptr<T> to_const(const void* p) {
  return (kptr<T>)(p);
}

// scalar (s_load) read of a tile descriptor
__device__ __forceinline__ TileDesc load_tile(const TileDesc* tiles, int64_t i) {
  const kptr<int32_t> p = to_const<int32_t>(tiles + i);
  TileDesc d;
  d.seg = p[0];
  d.count = p[1];
  d.start = to_const<int64_t>(tiles + i)[1];
  return d;
}

template <typename T>
__device__ __forceinline__ double load_g(gptr<const T> p, int64_t i);
template <>
__device__ __forceinline__ double load_g<float>(gptr<const float> p, int64_t i) { return p[i]; }
template <>
__device__ __forceinline__ double load_g<double>(gptr<const double> p, int64_t i) { return p[i]; }
template <>
__device__ __forceinline__ double load_g<__half>(gptr<const __half> p, int64_t i) {
  return half_bits_to_f64(((gptr<const uint16_t>)p)[i]);
}
template <>
__device__ __forceinline__ double load_g<bf16_t>(gptr<const bf16_t> p, int64_t i) {
  return bf16_bits_to_f64(((gptr<const uint16_t>)p)[i]);
}

// Loads of one client's share of a tile for one lane: VPL vectors of 16 B, expanded to
// kAE doubles. Element index (within the tile) of vector v of lane li: (v*LANES + li)*N,
// so one wave-instruction reads 1 KiB contiguous.
template <typename T, int LANES, bool FULL, bool VEC, int AE>
struct LaneLoader {
  using V = typename Vec16<T>::type;
  static constexpr int N = Vec16<T>::n;
  static constexpr int VPL = AE / N;

  // raw 16-B loads (fast path: aligned buffers; a whole tile, or — nv < VPL — a tile of nv
  // whole lane-vectors, the rest zero: a wave-uniform guard, no per-lane bounds)
  __device__ __forceinline__ static void load_raw(gptr<const T> base, int li, V (&buf)[VPL], int nv = VPL) {
    const gptr<const V> vb = (gptr<const V>)base;
#pragma unroll
    for (int v = 0; v < VPL; ++v) {
      if (FULL || v < nv) {
        buf[v] = __builtin_nontemporal_load(vb + v * LANES + li);
      } else {
        buf[v] = V{};
      }
    }
  }

  // bounds-checked loads straight to doubles (segment tails, unaligned buffers)
  __device__ __forceinline__ static void load_checked(gptr<const T> base, int li, int count,
                                                      double (&x)[AE]) {
#pragma unroll
    for (int v = 0; v < VPL; ++v) {
      const int e = (v * LANES + li) * N;
      if (VEC && e + N <= count) {
        const V raw = ((gptr<const V>)base)[v * LANES + li];
        expand<T>(raw, x + v * N);
      } else {
#pragma unroll
        for (int j = 0; j < N; ++j) x[v * N + j] = (e + j < count) ? load_g<T>(base, e + j) : 0.0;
      }
    }
  }
};

// One tile of the weighted reduce. See the file header for the algorithm.
// Launch geometry. The exact-order kernel (SPLIT = 1) tiles every dtype the same way
// (kTile1 elements, so one tile table serves all calls) but gives each lane a dtype-dependent
// slice: 16 elements (fp32 / fp64: a client's tile slice is 16 KiB resp. 32 KiB contiguous,
// 4 / 2 clients in flight per group) or 8 (fp16 / bf16: 512-lane workgroups, 16 clients per
// group) — the fastest shapes measured on MI355X. The split kernel keeps kAE for all dtypes.
//
// Whole-layout launches of 2- and 4-byte inputs (no tile range: one-shot aggregates, waves,
// full partials) use a second table of kTileWide = 8192-element tiles (TILEN = kTileWide:
// 512 / 1024-lane workgroups, 32 / 16 KiB contiguous per client per tile): +1.3 % (fp32) and
// +3 % (fp16) on 64 x ResNet-18, interleaved A/B. Any partition of the elements gives the same
// per-element fold, so both tables produce identical bits; ranged launches (sharded chunks,
// finalize ranges) keep the 4096-element table their tile indices refer to. fp64 keeps 4096
// (1024-lane tiles measured -15 %).
template <typename T, int SPLIT, int TILEN = kTile1>
struct Geo {
  static constexpr int AE = (SPLIT > 1) ? kAE
                          : (sizeof(T) == 2 ? FEDAVG_AE_HALF
                             : sizeof(T) == 8 ? FEDAVG_AE_F64
                                              : kAE);
  static constexpr int LANES = (SPLIT > 1) ? 64 : TILEN / AE;
  static constexpr int THREADS = (SPLIT > 1) ? kThreads : LANES;
  static constexpr int TILE = LANES * AE;
  static_assert(SPLIT == 1 || TILE == kTile4, "split tiles");
  static_assert(SPLIT > 1 || TILE == TILEN, "tile geometry");
  static_assert(THREADS % 64 == 0 && THREADS <= 1024, "workgroup size");
};

// NaN flags live in host-coherent pinned memory, one word per condition (0: accumulator NaN,
// 1: result NaN). A wave that sees a NaN stores 1 with system scope — no atomics, every
// writer writes the same value — and the host reads the words after the stream drains.
__device__ __forceinline__ void raise_flag(uint32_t* flag, int word) {
  __hip_atomic_store(flag + word, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Non-temporal vector store of a result / accumulator slice.
template <typename V>
__device__ __forceinline__ void store_out(gptr<V> p, V v) {
  __builtin_nontemporal_store(v, p);
}

// One fp64 fold step. The reference rounds the product and the sum separately
// (`tmp = x.to(f64) * w; acc += tmp`). When the host has proven every product of the call
// exact in fp64 (FMA = true: the weight's significand fits beside the input's, e.g. integer
// dataset sizes and fp32 inputs), round(acc + x*w) == fma(x, w, acc) and one instruction does
// it; otherwise the two roundings are kept.
//
// FOLD_DELTA: the client sent a delta against the server's global model
// (DeltaParameterMessage.restore, message.py:40-61): x = base + delta in fp64 (rounded, like
// `old.to(float64) + v`), then the separately rounded product and sum.
enum FoldKind : int { FOLD_MULADD = 0, FOLD_FMA = 1, FOLD_DELTA = 2 };

template <int FOLD>
__device__ __forceinline__ double fold(double acc, double x, double w, double base) {
  if constexpr (FOLD == FOLD_FMA) {
    return __builtin_fma(x, w, acc);
  } else if constexpr (FOLD == FOLD_DELTA) {
    const double full = base + x;
    const double p = full * w;
    return acc + p;
  } else {
    const double p = x * w;
    return acc + p;
  }
}

// PARTV: a tile shorter than TILE whose count is a whole number of lane-vectors (LANES * N
// elements): the grouped / pipelined fast path with the missing vectors guarded wave-uniformly
// (the balanced tile tables end every launch with such tiles, see build_balanced_tiles).
template <typename T, int OUT, int SPLIT, bool VEC, bool FULL, int FOLD, int TILEN = kTile1, bool PARTV = false,
          bool COMB = false>
__device__ __forceinline__ void tile_body(const KArgs& a, const TileDesc& td, double* lds) {
  constexpr int AE = Geo<T, SPLIT, TILEN>::AE;
  constexpr int LANES = Geo<T, SPLIT, TILEN>::LANES;  // lanes sharing one client stream
  using LL = LaneLoader<T, LANES, FULL && VEC, VEC, AE>;
  using V = typename LL::V;
  constexpr int N = LL::N;
  constexpr int VPL = LL::VPL;
  // clients in flight per lane: 256 B of loads per lane per group
  constexpr int CU_B = sizeof(T) == 8 ? FEDAVG_CU_BYTES_F64 : FEDAVG_CU_BYTES;
  constexpr int CU_LOADS = (CU_B / (VPL * 16)) < 2 ? 2 : (CU_B / (VPL * 16));
  constexpr bool FAST = (FULL || PARTV) && VEC;

  const int seg = td.seg;
  const int count = td.count;
  const int nv = FULL ? VPL : count / (LANES * N);  // whole lane-vectors of the tile (PARTV)
  const int wave = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x) >> 6);
  const int li = (SPLIT == 1) ? static_cast<int>(threadIdx.x) : static_cast<int>(threadIdx.x & 63);

  const int kseg = to_const<int32_t>(a.tab.kseg)[seg];
  int kb = 0, ke = kseg;
  if constexpr (SPLIT > 1) {
    const int per = (kseg + SPLIT - 1) / SPLIT;
    kb = min(kseg, wave * per);
    ke = min(kseg, kb + per);
  }
  const kptr<uint64_t> cp = to_const<uint64_t>(a.tab.cptrs) + static_cast<int64_t>(seg) * a.K;
  const kptr<double> wp = to_const<double>(a.tab.w) + static_cast<int64_t>(seg) * a.K;
  const int64_t acc_base = to_const<int64_t>(a.segs)[2 * seg] + td.start;  // SegDesc::acc_off
  const int64_t elem_off = td.start * static_cast<int64_t>(sizeof(T));
  auto client = [&](int k) -> gptr<const T> {
    return to_global<T>(reinterpret_cast<const void*>(cp[k] + elem_off));
  };

  // The accumulator starts at -0.0, the additive identity of IEEE addition: -0.0 + p == p
  // for every p (including -0.0 and +0.0), and fma(x, w, -0.0) == round(x * w). Folding the
  // first client into it therefore equals the reference's assignment `acc = tmp`
  // (fed_avg_algorithm.py:55-56) bit for bit, signed zeros included, with no special case.
  double acc[AE];
#pragma unroll
  for (int i = 0; i < AE; ++i) acc[i] = -0.0;
  bool have = a.zero_init != 0;  // wave-uniform: "this wave holds a value for the tile"
  if ((SPLIT == 1 || wave == 0) && !a.zero_init && to_const<int32_t>(a.tab.acc_in)[seg]) {
    const gptr<const double> ap = to_global<double>(a.acc + acc_base);
#pragma unroll
    for (int v = 0; v < VPL; ++v) {
      const int e = (v * LANES + li) * N;
#pragma unroll
      for (int j = 0; j < N; j += 2) {
        if (FULL || e + j + 2 <= count) {
          const f64x2 d = *(gptr<const f64x2>)(ap + e + j);  // plain: non-temporal measured -14 %
          acc[v * N + j] = d.x;
          acc[v * N + j + 1] = d.y;
        } else {
          if (e + j < count) acc[v * N + j] = ap[e + j];
          if (e + j + 1 < count) acc[v * N + j + 1] = ap[e + j + 1];
        }
      }
    }
    have = true;
  }

  // delta calls: the base model's slice of this tile, fp64, read once per tile (L2-shared
  // by nothing else: one read of the base per fold, like one more client)
  double base[AE];
#pragma unroll
  for (int i = 0; i < AE; ++i) base[i] = 0.0;
  if constexpr (FOLD == FOLD_DELTA) {
    const gptr<const double> bp =
        to_global<double>(reinterpret_cast<const void*>(to_const<uint64_t>(a.tab.base)[seg])) + td.start;
#pragma unroll
    for (int v = 0; v < VPL; ++v) {
      const int e = (v * LANES + li) * N;
#pragma unroll
      for (int j = 0; j < N; j += 2) {
        if (VEC && (FULL || e + j + 2 <= count)) {
          const f64x2 d = *(gptr<const f64x2>)(bp + e + j);
          base[v * N + j] = d.x;
          base[v * N + j + 1] = d.y;
        } else {
          if (e + j < count) base[v * N + j] = bp[e + j];
          if (e + j + 1 < count) base[v * N + j + 1] = bp[e + j + 1];
        }
      }
    }
  }

  // Fold this wave's clients [kb, ke) in order, in groups of CU_LOADS clients: all loads of
  // a group are issued before any is consumed. A short last group (TAIL) re-loads its last
  // client for the missing slots (L2 hits) and masks them out of the fold with selects —
  // never with branches, which made hipcc serialise the loads.
  constexpr bool PIPE = FAST && ((FEDAVG_PIPE >> (sizeof(T) == 2 ? 0 : sizeof(T) == 4 ? 1 : 2)) & 1);
  if constexpr (PIPE) {
    // Software-pipelined form: the next stage's client loads are issued before the current
    // stage folds, so a lane keeps HBM requests in flight through its own fold work (the
    // grouped form below leaves the lane's memory pipe idle while it folds a group). Stages
    // of PG clients alternate between two register buffers; the stage after the last one
    // re-loads the last client (an L2 hit, never folded) so every stage issues the same loads
    // and the code stays branch-free.
    constexpr int PB = FEDAVG_PIPE_BYTES;
    constexpr int PG = (PB / (VPL * 16)) < 1 ? 1 : (PB / (VPL * 16));
    V bufA[PG][VPL], bufB[PG][VPL];
    double wA[PG], wB[PG];
    auto load_stage = [&](V (&buf)[PG][VPL], double (&wk)[PG], int k) {
#pragma unroll
      for (int c = 0; c < PG; ++c) {
        const int kc = min(k + c, ke - 1);
        wk[c] = wp[kc];
        LL::load_raw(client(kc), li, buf[c], nv);
      }
    };
    auto fold_stage = [&](auto tail_tag, V (&buf)[PG][VPL], const double (&wk)[PG], int n) {
      constexpr bool TAIL = decltype(tail_tag)::value;
#pragma unroll
      for (int c = 0; c < PG; ++c) {
#pragma unroll
        for (int v = 0; v < VPL; ++v) {
          double x[N];
          expand<T>(buf[c][v], x);
#pragma unroll
          for (int j = 0; j < N; ++j) {
            double& r = acc[v * N + j];
            const double nv = fold<FOLD>(r, x[j], wk[c], base[v * N + j]);
            if constexpr (TAIL) {
              r = (c < n) ? nv : r;
            } else {
              r = nv;
            }
          }
        }
      }
    };
    if (kb < ke) {
      int k = kb;
      load_stage(bufA, wA, k);
      // full stages two at a time (A folds while B loads, then B folds while A loads)
      while (k + 2 * PG <= ke) {
        load_stage(bufB, wB, k + PG);
        fold_stage(std::false_type{}, bufA, wA, PG);
        load_stage(bufA, wA, k + 2 * PG);
        fold_stage(std::false_type{}, bufB, wB, PG);
        k += 2 * PG;
      }
      // 0 < ke - k < 2 * PG clients left; bufA holds stage k
      if (k + PG < ke) {
        load_stage(bufB, wB, k + PG);
        fold_stage(std::false_type{}, bufA, wA, PG);
        fold_stage(std::true_type{}, bufB, wB, ke - k - PG);
      } else if (k < ke) {
        fold_stage(std::true_type{}, bufA, wA, ke - k);
      }
    }
  } else if constexpr (FAST) {
    auto group = [&](auto tail_tag, int k, int n) {
      constexpr bool TAIL = decltype(tail_tag)::value;
      V buf[CU_LOADS][VPL];
      double wk[CU_LOADS];
#pragma unroll
      for (int c = 0; c < CU_LOADS; ++c) {
        const int kc = TAIL ? k + min(c, n - 1) : k + c;
        wk[c] = wp[kc];
        LL::load_raw(client(kc), li, buf[c], nv);
      }
#pragma unroll
      for (int c = 0; c < CU_LOADS; ++c) {
#pragma unroll
        for (int v = 0; v < VPL; ++v) {
          double x[N];
          expand<T>(buf[c][v], x);
#pragma unroll
          for (int j = 0; j < N; ++j) {
            double& r = acc[v * N + j];
            const double nv = fold<FOLD>(r, x[j], wk[c], base[v * N + j]);
            if constexpr (TAIL) {
              r = (c < n) ? nv : r;
            } else {
              r = nv;
            }
          }
        }
      }
    };
    int k = kb;
    for (; k + CU_LOADS <= ke; k += CU_LOADS) group(std::false_type{}, k, CU_LOADS);
    if (k < ke) group(std::true_type{}, k, ke - k);
  } else {
    for (int k = kb; k < ke; ++k) {
      const double wk = wp[k];
      double x[AE];
      LL::load_checked(client(k), li, count, x);
#pragma unroll
      for (int i = 0; i < AE; ++i) acc[i] = fold<FOLD>(acc[i], x[i], wk, base[i]);
    }
  }
  have = have || (ke > kb);

  if constexpr (SPLIT > 1) {
    // stage wave partials in LDS; wave 0 folds them in wave order
    int* have_lds = reinterpret_cast<int*>(lds + (SPLIT - 1) * 64 * AE);
    if (wave > 0) {
      double* dst = lds + ((wave - 1) * 64 + li) * AE;
#pragma unroll
      for (int i = 0; i < AE; ++i) dst[i] = acc[i];
      if (li == 0) have_lds[wave - 1] = have ? 1 : 0;
    }
    __syncthreads();
    if (wave != 0) return;
#pragma unroll
    for (int w2 = 1; w2 < SPLIT; ++w2) {
      if (have_lds[w2 - 1]) {
        const double* src = lds + ((w2 - 1) * 64 + li) * AE;
        if (have) {
#pragma unroll
          for (int i = 0; i < AE; ++i) acc[i] = acc[i] + src[i];
        } else {
#pragma unroll
          for (int i = 0; i < AE; ++i) acc[i] = src[i];
        }
        have = true;
      }
    }
  }
  if (!have) return;  // nothing for this segment in this call (host prevents for finals)

  if constexpr (COMB) {
    // S_0 + S_1 + ... in entry order (multi_device.cpp's composition), this entry's chain in place
    static_assert(OUT != OUT_ACC && SPLIT == 1, "the own-window combine ends a final fold");
    double tot[AE];
#pragma unroll
    for (int i = 0; i < AE; ++i) tot[i] = -0.0;
    for (int h = 0; h < a.comb_n; ++h) {  // wave-uniform
      if (h == a.comb_self) {
#pragma unroll
        for (int i = 0; i < AE; ++i) tot[i] = tot[i] + acc[i];
      } else {
        const gptr<const double> sp =
            to_global<double>(reinterpret_cast<const void*>(to_const<uint64_t>(a.comb_src)[h])) + acc_base;
#pragma unroll
        for (int v = 0; v < VPL; ++v) {
          const int e = (v * LANES + li) * N;
#pragma unroll
          for (int j = 0; j < N; j += 2) {
            if (FULL || e + j + 2 <= count) {
              const f64x2 d = *(gptr<const f64x2>)(sp + e + j);
              tot[v * N + j] = tot[v * N + j] + d.x;
              tot[v * N + j + 1] = tot[v * N + j + 1] + d.y;
            } else {
              if (e + j < count) tot[v * N + j] = tot[v * N + j] + sp[e + j];
              if (e + j + 1 < count) tot[v * N + j + 1] = tot[v * N + j + 1] + sp[e + j + 1];
            }
          }
        }
      }
    }
#pragma unroll
    for (int i = 0; i < AE; ++i) acc[i] = tot[i];
  }

  // fused NaN check on the accumulator (fed_avg_algorithm.py:93)
  bool bad_acc = false;
#pragma unroll
  for (int v = 0; v < VPL; ++v) {
    const int e = (v * LANES + li) * N;
#pragma unroll
    for (int j = 0; j < N; ++j) {
      const bool in_range = FULL || (e + j < count);
      bad_acc |= in_range && (acc[v * N + j] != acc[v * N + j]);
    }
  }

  if constexpr (OUT == OUT_ACC) {
    const gptr<double> ap = to_global_mut<double>(a.acc + acc_base);
#pragma unroll
    for (int v = 0; v < VPL; ++v) {
      const int e = (v * LANES + li) * N;
#pragma unroll
      for (int j = 0; j < N; j += 2) {
        if (FULL || e + j + 2 <= count) {
          const f64x2 pair = f64x2{acc[v * N + j], acc[v * N + j + 1]};
          // (plain stores for fp32 / fp64 waves too measured -1.3 ... -3.7 %: kept non-temporal)
          if constexpr (sizeof(T) == 2 && FEDAVG_ACC_PLAIN_STORE_HALF) {
            *(gptr<f64x2>)(ap + e + j) = pair;  // see FEDAVG_ACC_PLAIN_STORE_HALF
          } else {
            store_out((gptr<f64x2>)(ap + e + j), pair);
          }
        } else {
          if (e + j < count) ap[e + j] = acc[v * N + j];
          if (e + j + 1 < count) ap[e + j + 1] = acc[v * N + j + 1];
        }
      }
    }
    if (__ballot(bad_acc) != 0ull && (threadIdx.x & 63) == 0) raise_flag(a.flag, 0);
  } else {
    // fused divide (_apply_total_weight, :71-74) + NaN check of the result (:97)
    const double W = to_const<double>(a.tab.wtot)[seg];
    bool bad_res = false;
    double res[AE];
    exact_div_block<AE>(acc, res, W);
#pragma unroll
    for (int v = 0; v < VPL; ++v) {
      const int e = (v * LANES + li) * N;
#pragma unroll
      for (int j = 0; j < N; ++j) {
        const bool in_range = FULL || (e + j < count);
        bad_res |= in_range && (res[v * N + j] != res[v * N + j]);
      }
    }
    void* const out_raw = reinterpret_cast<void*>(to_const<uint64_t>(a.tab.outs)[seg]);
    if constexpr (OUT == OUT_F32) {
      const gptr<float> op = to_global_mut<float>(out_raw) + td.start;
#pragma unroll
      for (int v = 0; v < VPL; ++v) {
        const int e = (v * LANES + li) * N;
        if constexpr (N >= 4) {
#pragma unroll
          for (int j = 0; j < N; j += 4) {
            if (VEC && (FULL || e + j + 4 <= count)) {
              store_out((gptr<f32x4>)(op + e + j),
                  f32x4{static_cast<float>(res[v * N + j]), static_cast<float>(res[v * N + j + 1]),
                        static_cast<float>(res[v * N + j + 2]), static_cast<float>(res[v * N + j + 3])});
            } else {
#pragma unroll
              for (int q = 0; q < 4; ++q)
                if (e + j + q < count) op[e + j + q] = static_cast<float>(res[v * N + j + q]);
            }
          }
        } else {
          if (VEC && (FULL || e + 2 <= count)) {
            store_out((gptr<f32x2>)(op + e),
                      f32x2{static_cast<float>(res[v * N]), static_cast<float>(res[v * N + 1])});
          } else {
            if (e < count) op[e] = static_cast<float>(res[v * N]);
            if (e + 1 < count) op[e + 1] = static_cast<float>(res[v * N + 1]);
          }
        }
      }
    } else {
      const gptr<double> op = to_global_mut<double>(out_raw) + td.start;
#pragma unroll
      for (int v = 0; v < VPL; ++v) {
        const int e = (v * LANES + li) * N;
#pragma unroll
        for (int j = 0; j < N; j += 2) {
          if (VEC && (FULL || e + j + 2 <= count)) {
            store_out((gptr<f64x2>)(op + e + j), f64x2{res[v * N + j], res[v * N + j + 1]});
          } else {
            if (e + j < count) op[e + j] = res[v * N + j];
            if (e + j + 1 < count) op[e + j + 1] = res[v * N + j + 1];
          }
        }
      }
    }
    const uint64_t ba = __ballot(bad_acc);
    const uint64_t br = __ballot(bad_res);
    if ((ba | br) != 0ull && (threadIdx.x & 63) == 0) {
      if (ba) raise_flag(a.flag, 0);
      if (br) raise_flag(a.flag, 1);
    }
  }
}

// PV: the launch's tile table holds tiles of whole lane-vectors shorter than a tile (the pieces of
// a balanced order, build_balanced_tiles) and they take the grouped fast path. A separate
// instantiation: compiled into every launch, that path cost the plain whole-layout launch 3-4 %
// (VGPRs 131 -> 144, twice the code; profiles/r03_ab_matrix.txt).
template <typename T, int OUT, int SPLIT, bool VEC, int FOLD, int TILEN = kTile1, bool PV = false, bool COMB = false>
__global__ __launch_bounds__((Geo<T, SPLIT, TILEN>::THREADS)) void fedavg_tile_kernel(KArgs a) {
  __shared__ double lds[(SPLIT > 1) ? ((SPLIT - 1) * 64 * kAE + 8) : 1];
  constexpr int TILE = Geo<T, SPLIT, TILEN>::TILE;
  // One workgroup per tile (a persistent grid walking the tiles measured 2 % slower and is not
  // kept). The split kernel's LDS combine ends with the non-zero waves leaving.
  const int ntiles = (SPLIT == 1) ? a.num_tiles : static_cast<int>(gridDim.x);
  if constexpr (OUT == OUT_ACC && SPLIT == 1) {
    if (a.win_dst != nullptr) {
      // windowed partial (multi-device peer exchange): the tile's window picks the destination,
      // a wave-uniform scan of at most FEDAVG_MULTI_MAX_DEVICES scalar edges
      for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const int32_t ti = a.tile_begin + t;
        const kptr<int32_t> we = to_const<int32_t>(a.win_edge);
        int j = 0;
        while (j + 1 < a.win_n && ti >= we[j + 1]) ++j;
        KArgs b = a;
        b.acc = reinterpret_cast<double*>(to_const<uint64_t>(a.win_dst)[j]);
        const TileDesc td = load_tile(a.tiles, ti);
        if (td.count == TILE) tile_body<T, OUT, SPLIT, VEC, true, FOLD, TILEN>(b, td, lds);
        else tile_body<T, OUT, SPLIT, VEC, false, FOLD, TILEN>(b, td, lds);
      }
      return;
    }
  }
  if constexpr (COMB) {
    // own-window combine launches: one tile per workgroup, exact order, no balanced pieces
    const TileDesc td = load_tile(a.tiles, a.tile_begin + static_cast<int>(blockIdx.x));
    if (td.count == TILE) tile_body<T, OUT, SPLIT, VEC, true, FOLD, TILEN, false, true>(a, td, lds);
    else tile_body<T, OUT, SPLIT, VEC, false, FOLD, TILEN, false, true>(a, td, lds);
    return;
  }
  for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const TileDesc td = load_tile(a.tiles, a.tile_begin + (t < a.walk_back ? a.walk_back - 1 - t : t));
    constexpr int LV = Geo<T, SPLIT, TILEN>::LANES * Vec16<T>::n;  // elements per lane-vector row
    if (td.count == TILE) {
      tile_body<T, OUT, SPLIT, VEC, true, FOLD, TILEN>(a, td, lds);
    } else {
      bool partv = false;
      if constexpr (PV && SPLIT == 1 && VEC && LV < TILE) partv = (td.count % LV) == 0;
      if (partv) {
        if constexpr (PV && SPLIT == 1 && VEC && LV < TILE) tile_body<T, OUT, SPLIT, VEC, false, FOLD, TILEN, true>(a, td, lds);
      } else {
        tile_body<T, OUT, SPLIT, VEC, false, FOLD, TILEN>(a, td, lds);
      }
    }
    if constexpr (SPLIT > 1) break;
  }
}

// ---------------------------------------------------------------------------------------
// Dynamic wave: the round's first wave folded while its clients are still arriving.
//
// The plugin round (FedAVGAlgorithm.process_worker_data x N, then aggregate_worker_data:
// fed_avg_algorithm.py:20-113, driven by aggregation_server.py:111-145) stages every arrival on
// the host; a wave launched only once all N are staged leaves the GPU idle for the whole
// arrival phase. This kernel is launched at the round's first arrival with an open client count:
// the host publishes staged rows into a host-coherent table (fedavg_dyn_publish) and the kernel
// folds them as they appear, in arrival order, into fp64 accumulators held in registers; the
// round's close (fedavg_dyn_close) fixes the count and either divides into the outputs (the
// fused `_apply_total_weight`, :71-97) or stores the accumulator (a partial wave the ordinary
// waves continue from). Per element the fold is the reference's chain — acc = -0.0, then
// acc + round(x * w) per client in arrival order — so the bits are those of the one-launch
// kernel.
//
// Workgroup 0 is the mirror: its thread 0 polls the host control words over PCIe; on new rows
// the whole workgroup copies them (client pointers, weights; at a final close the divisors and
// output pointers) from the host table into a device table and then republishes the row count
// in device memory, so the tile workgroups never read host memory and poll device memory only.
// The mirror also ends the wave by itself (state 2, accumulator mode) when the host publishes
// nothing for `idle` ticks or the wave outlives `life` ticks, and acknowledges every close in
// host memory — the host learns from that acknowledgement how many rows were folded. Every
// workgroup leaves once the mirror closed (tile workgroups also after `life` + a margin on their
// own): no wave spins past the wave's lifetime.
//
// Hand-off inside the launch (cdna_hip_programming.md §6 Guideline 16): the device table is
// written with system-coherent stores and read with system-coherent loads (no stale L1 / L2 copy
// of a line a consumer read before its later rows were written); every storing wave of the mirror
// drains its stores (s_waitcnt vmcnt(0)) before the workgroup barrier behind which ONE lane
// publishes the count word (8-B agent-scope store); a tile workgroup polls that word relaxed and
// needs no acquire (it reads no handed-off byte through L1 / L2). All stores are vector stores.
struct DynCtl {     // host-coherent, written by the host: ONE 8-B word, so a poll is one PCIe read
  uint64_t word;    // dyn_word(rows published, closed: the count is final, close mode, 0), release
  uint64_t pad[7];
};
struct DynAck {     // host-coherent, written by the mirror workgroup
  uint64_t word;    // state (0 running, 1 closed by the host, 2 closed by the kernel: idle /
                    // lifetime) | rows the wave folds << 32 — one 8-B store
  uint32_t error;   // 1: a tile workgroup gave up waiting for the mirror
  uint32_t polls;   // the mirror's polls of the host word (FEDAVG_DYN_TRACE)
  uint64_t t_seen;  // s_memrealtime when the mirror saw the close, and when it acknowledged it
  uint64_t t_done;
  uint64_t t_rows;  // s_memrealtime when the mirror last handed the tiles more rows
};
struct DynMirror {  // device memory, written by the mirror workgroup: one copy per XCD (kDynCopies,
  uint64_t word;    // a cache line apart), so the tile workgroups' polls spread over 8 lines
  uint64_t pad[7];
};
constexpr int kDynCopies = 8;
// poll back-off (s_sleep units of 64 clocks) of the mirror's host-word polls and of a waiting tile
// workgroup's mirror-word polls; 4x and 16x shorter measured the same (profiles/r06_dyn_poll_sleep_ab.txt)
constexpr int kDynMirrorSleep = 8;
constexpr int kDynTileSleep = 32;
// the mirror word: rows mirrored (bits 0-23), closed (bit 24), close mode (bits 25-27), the wave's
// epoch (bits 32-63: a word left by an earlier wave reads as "nothing yet", so no per-wave reset)
__host__ __device__ constexpr uint64_t dyn_word(uint32_t count, uint32_t closed, uint32_t mode, uint32_t epoch) {
  return static_cast<uint64_t>(count & 0xffffffu) | (static_cast<uint64_t>(closed & 1u) << 24) |
         (static_cast<uint64_t>(mode & 7u) << 25) | (static_cast<uint64_t>(epoch) << 32);
}
struct DynArgs {
  const TileDesc* tiles;       // body tiles (kDynTile elements each)
  const TileDesc* edge_tiles;  // edge tiles (<= kDynEdgeTile elements each)
  const SegDesc* segs;
  double* acc;
  uint32_t* flag;
  DynCtl* ctl;              // device aliases of the host-coherent block
  DynAck* ack;
  const uint64_t* h_ptab;   // host table: [T][cap] client pointers, segment-major
  const double* h_wtab;     // [cap] client weights
  const double* h_wtot;     // [T] divisors (final close)
  const uint64_t* h_outs;   // [T] output pointers (final close)
  uint64_t* ptab;           // the device copies the mirror writes
  double* wtab;
  double* wtot;
  uint64_t* outs;
  DynMirror* mir;
  uint32_t* elect;          // the mirror election word (device memory): the wave's epoch once taken
  uint64_t* tend;           // profiling: per tile (body tiles, then edge tiles) the time it finished
  int32_t edge_base;        // the first edge tile's index in tend
  int32_t num_tiles;
  int32_t num_segs;
  int32_t cap;
  uint32_t epoch;
  int32_t resume;           // 1: the accumulators start from the fp64 accumulator (a continued wave)
  uint64_t idle_ticks;      // s_memrealtime ticks (100 MHz)
  uint64_t life_ticks;
};

constexpr int kDynBatch = 64;  // rows a tile workgroup fetches per poll (one per lane of wave 0)

__device__ __forceinline__ uint64_t dyn_ld_sys64(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void dyn_st_sys64(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ double dyn_ld_sysf(const double* p) {
  return __longlong_as_double(static_cast<long long>(dyn_ld_sys64(reinterpret_cast<const uint64_t*>(p))));
}

// The mirror role goes to the first leading workgroup to arrive: each launch of the wave (body and
// edge, on two streams) starts with one candidate workgroup, the loser leaves at once. A launch's
// leading workgroup is dispatched before the rest of it, so whichever launch holds CU slots also
// holds (or held) the mirror, and no tile can spin on a mirror that waits for those slots. Were
// that ordering ever broken, the tiles' own lifetime bound still ends the wave (ack->error).
__device__ bool dyn_elect(const DynArgs& a) {
  __shared__ int32_t s_win;
  if (threadIdx.x == 0) {
    uint32_t cur = __hip_atomic_load(a.elect, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int32_t win = 0;
    while (cur != a.epoch) {
      if (__hip_atomic_compare_exchange_strong(a.elect, &cur, a.epoch, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT)) {
        win = 1;
        break;
      }
    }
    s_win = win;
  }
  __syncthreads();
  return s_win != 0;
}

__device__ void dyn_mirror(const DynArgs& a) {
  __shared__ uint32_t s_cmd[3];  // rows published, 0 running / 1 host close / 2 own close, close mode
  const int tid = static_cast<int>(threadIdx.x);
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  uint64_t last = t0, t_seen = 0, t_rows = 0;
  uint32_t mc = 0, polls = 0;  // rows mirrored so far, host polls
  for (;;) {
    if (tid == 0) {
      uint32_t hc = mc, st = 0, mode = OUT_ACC;
      for (;;) {
        const uint64_t cw = dyn_ld_sys64(&a.ctl->word);
        const uint32_t c = static_cast<uint32_t>(cw) & 0xffffffu;
        const uint64_t now = __builtin_amdgcn_s_memrealtime();
        ++polls;
        if ((cw >> 24) & 1u) {
          // no fence: the host wrote the table before releasing the word, and every read of the
          // host block is system-coherent (uncached), issued after this poll returned
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
          hc = c;
          mode = static_cast<uint32_t>(cw >> 25) & 7u;
          st = 1;
          t_seen = now;
          break;
        }
        if (c > mc) {
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
          hc = c;
          last = now;
          break;
        }
        if (now - last > a.idle_ticks || now - t0 > a.life_ticks) {
          // nothing new for too long (or too long alive): the wave ends with the rows it has
          st = 2;
          break;
        }
        __builtin_amdgcn_s_sleep(kDynMirrorSleep);
      }
      s_cmd[0] = hc;
      s_cmd[1] = st;
      s_cmd[2] = mode;
    }
    __syncthreads();
    const uint32_t hc = s_cmd[0], st = s_cmd[1], mode = s_cmd[2];
    // copy rows [mc, hc) of the host table, and at a final close the divisors and outputs
    const int rows = static_cast<int>(hc - mc);
    if (rows > 0) t_rows = __builtin_amdgcn_s_memrealtime();
    if (rows > 0) {
      const int n = rows * a.num_segs;
#pragma unroll 4
      for (int i = tid; i < n; i += static_cast<int>(blockDim.x)) {  // (4 PCIe reads in flight)
        const int t = i / rows;
        const int64_t o = static_cast<int64_t>(t) * a.cap + mc + (i - t * rows);
        dyn_st_sys64(a.ptab + o, dyn_ld_sys64(a.h_ptab + o));
      }
      for (int i = tid; i < rows; i += static_cast<int>(blockDim.x)) {
        uint64_t* d = reinterpret_cast<uint64_t*>(a.wtab) + mc + i;
        dyn_st_sys64(d, dyn_ld_sys64(reinterpret_cast<const uint64_t*>(a.h_wtab) + mc + i));
      }
    }
    if (st == 1 && mode != OUT_ACC) {
      for (int t = tid; t < a.num_segs; t += static_cast<int>(blockDim.x)) {
        dyn_st_sys64(reinterpret_cast<uint64_t*>(a.wtot) + t, dyn_ld_sys64(reinterpret_cast<const uint64_t*>(a.h_wtot) + t));
        dyn_st_sys64(a.outs + t, dyn_ld_sys64(a.h_outs + t));
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its stores
    __syncthreads();
    if (tid == 0) {
      const uint64_t w = dyn_word(hc, st != 0 ? 1u : 0u, st == 1 ? mode : static_cast<uint32_t>(OUT_ACC), a.epoch);
      for (int i = 0; i < kDynCopies; ++i)
        __hip_atomic_store(&a.mir[i].word, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (st != 0) {
        __hip_atomic_store(&a.ack->polls, polls, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(&a.ack->t_seen, t_seen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(&a.ack->t_rows, t_rows, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(&a.ack->t_done, __builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(&a.ack->word, static_cast<uint64_t>(st) | (static_cast<uint64_t>(hc) << 32), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
    if (st != 0) return;
    mc = hc;
  }
}

// Geometry: the wave's fp64 accumulators stay in registers for the whole round, so as many
// tiles as possible must be resident at once — a tile that is not waits for a resident one to
// finish, i.e. for the close, and then folds every row after the arrivals instead of during them.
// Two launches share the wave (one mirror, one protocol):
//  * body tiles — every whole kDynTile-element tile of a segment: one-wave workgroups, kDynAE
//    elements per lane (96: 192 VGPRs of accumulators, two 16-element load stages, <= 256 VGPRs
//    = 2 waves per SIMD): 256 CUs x 4 SIMDs x 2 waves x 64 lanes x 96 = 12.6 M elements
//    resident, e.g. all 1,883 body tiles of ResNet-18 (11.7 M parameters in 62 tensors);
//  * edge tiles — what is left of each segment, in kDynEdgeTile-element tiles (kDynAEEdge per
//    lane): whole 16-B vectors with clamped loads, the < 16 B past the last one by one lane with
//    its accumulators in LDS (a tensor may end anywhere: nothing past its end is read).
// Loads are double-buffered per 16 elements (8 for fp64 inputs), across client boundaries too.
#ifndef FEDAVG_DYN_AE
#define FEDAVG_DYN_AE 96
#endif
#ifndef FEDAVG_DYN_AE_EDGE
#define FEDAVG_DYN_AE_EDGE 32
#endif
constexpr int kDynAE = FEDAVG_DYN_AE;
constexpr int kDynAEEdge = FEDAVG_DYN_AE_EDGE;
constexpr int kDynLanes = 64;
constexpr int kDynTile = kDynAE * kDynLanes;
constexpr int kDynEdgeTile = kDynAEEdge * kDynLanes;
template <typename T>
using DynV = typename Vec16<T>::type;
template <typename T, int AE>
struct DynGeo {
  using V = typename Vec16<T>::type;
  static constexpr int N = Vec16<T>::n;  // elements per 16-B vector = per load stage
  static constexpr int NV = AE / N;      // vectors (stages) per lane and client
  // NB load buffers in a ring: NB - 1 vectors in flight while one is folded; NV % NB == 0 keeps
  // every client's first stage on buffer 0, so the unrolled ring indices are compile-time
  static constexpr int NB = NV % 8 == 0 ? 8 : NV % 6 == 0 ? 6 : NV % 4 == 0 ? 4 : 2;
  static_assert(AE % N == 0 && NV % NB == 0, "lane slice in whole vectors, a whole number of rings");
};

// vector v of a client's tile slice into a ring buffer. PART (edge tiles): vectors at or past
// `nfull` (the tile's whole vectors) re-read vector 0 instead; their fold adds zeros
template <typename T, bool PART>
__device__ __forceinline__ void dyn_issue(DynV<T>& b, gptr<const DynV<T>> base, int v, int li, int nfull) {
  const int idx = v * kDynLanes + li;
  b = __builtin_nontemporal_load(base + ((!PART || idx < nfull) ? idx : 0));
}
// fold vector v into the accumulators: acc = acc + round(x * w), in arrival order
template <typename T, int AE, bool PART>
__device__ __forceinline__ void dyn_fold_vec(double (&acc)[AE], const DynV<T>& b, int v, double w, int li, int nfull) {
  constexpr int N = Vec16<T>::n;
  double x[N];
  expand<T>(b, x);
  const bool in = !PART || v * kDynLanes + li < nfull;
#pragma unroll
  for (int q = 0; q < N; ++q) {
    double& r = acc[v * N + q];
    r = fold<FOLD_MULADD>(r, in ? x[q] : 0.0, w, 0.0);
  }
}

// one client's tile slice through the load ring: before vector v is folded, vector v + NB - 1 is
// issued (past the slice's end: the next client's first vectors, when NEXT). The scheduling groups
// pin that order — left alone, the scheduler hoists every load of the client to its top and runs
// out of registers beside the accumulators.
template <typename T, int AE, bool PART, bool NEXT, int NB>
__device__ __forceinline__ void dyn_fold_client(double (&acc)[AE], DynV<T> (&buf)[NB], gptr<const DynV<T>> cur,
                                                gptr<const DynV<T>> nxt, double w, int li, int nfull) {
  constexpr int NV = AE / Vec16<T>::n;
  static_assert(NV % NB == 0, "a whole number of rings per client");
  constexpr int VALU_PER_VEC = Vec16<T>::n * (sizeof(T) == 8 ? 2 : sizeof(T) == 4 ? 3 : 4);
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    const int ahead = v + NB - 1;
    if (ahead < NV) {
      dyn_issue<T, PART>(buf[ahead % NB], cur, ahead, li, nfull);
    } else if (NEXT) {
      dyn_issue<T, PART>(buf[ahead % NB], nxt, ahead - NV, li, nfull);
    }
    dyn_fold_vec<T, AE, PART>(acc, buf[v % NB], v, w, li, nfull);
    __builtin_amdgcn_sched_group_barrier(0x20, 1, 0);             // VMEM_READ: the vector ahead
    __builtin_amdgcn_sched_group_barrier(0x2, VALU_PER_VEC, 0);  // VALU: this vector's fold
  }
}
// the ring's first NB - 1 vectors of a client
template <typename T, bool PART, int NB>
__device__ __forceinline__ void dyn_prime(DynV<T> (&buf)[NB], gptr<const DynV<T>> base, int li, int nfull) {
#pragma unroll
  for (int v = 0; v + 1 < NB; ++v) dyn_issue<T, PART>(buf[v], base, v, li, nfull);
}

// While the context profiles (fedavg_prof_enable): every tile workgroup stores the time it finished
// (its result stores issued) into tend[tile] — plain stores, no atomics — and fedavg_dyn_timing
// takes the latest: the fold time after the last rows reached the tiles. One lane.
__device__ __forceinline__ void dyn_tile_done(const DynArgs& a, int tile) {
  if (a.tend) a.tend[tile] = __builtin_amdgcn_s_memrealtime();
}

// EDGE = false: the body tiles, workgroup 0 the mirror; EDGE = true: the edge tiles
template <typename T, bool EDGE>
__global__ __attribute__((amdgpu_flat_work_group_size(kDynLanes, kDynLanes), amdgpu_waves_per_eu(2, 8)))
void dyn_wave_kernel(DynArgs a) {
  if (blockIdx.x == 0) {  // the launch's mirror candidate
    if (dyn_elect(a)) dyn_mirror(a);
    return;
  }
  constexpr int AE = EDGE ? kDynAEEdge : kDynAE;
  constexpr int TILE = EDGE ? kDynEdgeTile : kDynTile;
  using G = DynGeo<T, AE>;
  using V = typename G::V;
  constexpr int N = G::N;
  // the close works in groups of CE elements (CH vectors): one exact-division block each
  constexpr int CE = sizeof(T) == 8 ? 8 : 16;
  constexpr int CH = CE / N;
  constexpr int NCH = AE / CE;
  static_assert(AE % CE == 0, "whole division groups");
  __shared__ uint64_t sp[kDynBatch];
  __shared__ double sw[kDynBatch];
  __shared__ int32_t s_n;
  __shared__ int32_t s_mode;
  __shared__ double s_W;
  __shared__ uint64_t s_out;

  __shared__ double s_tail[N];

  const TileDesc td = load_tile(EDGE ? a.edge_tiles : a.tiles, blockIdx.x - 1);
  const int seg = td.seg;
  const int count = td.count;
  const bool full = !EDGE;  // body tiles are whole (count == TILE)
  const int nfull = count / N;        // whole 16-B vectors of the tile
  const int tail = count - nfull * N; // elements past them (a segment's last tile)
  const int li = static_cast<int>(threadIdx.x);
  const int64_t elem_off = td.start * static_cast<int64_t>(sizeof(T));
  const int64_t acc_base = to_const<int64_t>(a.segs)[2 * seg] + td.start;  // SegDesc::acc_off
  const gptr<const double> acc_in = to_global<double>(a.acc + acc_base);
  if (li < N) s_tail[li] = (a.resume && li < tail) ? acc_in[static_cast<int64_t>(nfull) * N + li] : -0.0;

  double acc[AE];  // element (v * 64 + li) * N + q of the tile at acc[v * N + q]
#pragma unroll
  for (int i = 0; i < AE; ++i) acc[i] = -0.0;  // the additive identity (see tile_body)
  if (a.resume) {
    // a continued wave: the rows earlier waves of the round folded, from the fp64 accumulator the
    // previous wave's accumulator close stored (the same element order as the close below)
#pragma unroll
    for (int v = 0; v < AE / N; ++v) {
      if (full || v * kDynLanes + li < nfull) {
        const gptr<const f64x2> src = reinterpret_cast<gptr<const f64x2>>(acc_in + static_cast<int64_t>(v * kDynLanes + li) * N);
#pragma unroll
        for (int q = 0; q < N / 2; ++q) {
          const f64x2 x = src[q];
          acc[v * N + 2 * q] = x.x;
          acc[v * N + 2 * q + 1] = x.y;
        }
      }
    }
  }
  (void)TILE;

  const DynMirror* const mir = a.mir + (blockIdx.x % kDynCopies);
  int k = 0;             // rows folded
  uint32_t avail = 0;    // rows known mirrored (thread 0)
  uint32_t closed = 0;   // the mirror closed the wave (thread 0)
  uint32_t cmode = OUT_ACC;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  for (;;) {
    if (threadIdx.x == 0) {
      if (avail <= static_cast<uint32_t>(k) && !closed) {
        for (;;) {  // relaxed polls of the mirror word
          const uint64_t w = __hip_atomic_load(&mir->word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (static_cast<uint32_t>(w >> 32) == a.epoch) {
            const uint32_t c = static_cast<uint32_t>(w) & 0xffffffu;
            if ((w >> 24) & 1u) {
              closed = 1;
              cmode = static_cast<uint32_t>(w >> 25) & 7u;
              avail = c;
              break;
            }
            if (c > avail) {
              avail = c;
              break;
            }
          }
          if (__builtin_amdgcn_s_memrealtime() - t0 > a.life_ticks + 100000000ull) {  // life + 1 s
            __hip_atomic_store(&a.ack->error, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            avail = static_cast<uint32_t>(k);
            closed = 1;
            cmode = OUT_ACC;
            break;
          }
          __builtin_amdgcn_s_sleep(kDynTileSleep);
        }
        // no acquire: every handed-off byte (the mirror's table) is stored and loaded with
        // system-coherent accesses, which no L1 / L2 copy can serve stale (Guideline 16's sc1
        // form); the client tensors were complete before their rows were published
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      }
      const int n = static_cast<int>(avail) - k;
      s_n = n < 0 ? 0 : (n > kDynBatch ? kDynBatch : n);
      s_mode = static_cast<int>(cmode);
    }
    __syncthreads();
    const int n = __builtin_amdgcn_readfirstlane(s_n);
    if (n == 0) break;
    if (li < n) {  // the batch's rows of this tile's segment, from the mirror's device table
      sp[li] = dyn_ld_sys64(a.ptab + static_cast<int64_t>(seg) * a.cap + k + li);
      sw[li] = dyn_ld_sysf(a.wtab + k + li);
    }
    __syncthreads();
    auto client = [&](int i) -> gptr<const T> {
      const uint64_t p = sp[i];
      const uint32_t lo = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(p));
      const uint32_t hi = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(p >> 32));
      return to_global<T>(reinterpret_cast<const void*>(((static_cast<uint64_t>(hi) << 32) | lo) + elem_off));
    };
    if (EDGE ? nfull > 0 : true) {  // the tile's whole vectors (all of a body tile's)
      constexpr int NB = G::NB;
      V buf[NB];
      dyn_prime<T, EDGE, NB>(buf, (gptr<const V>)client(0), li, nfull);
      int i = 0;
      for (; i + 1 < n; ++i)
        dyn_fold_client<T, AE, EDGE, true, NB>(acc, buf, (gptr<const V>)client(i), (gptr<const V>)client(i + 1), sw[i], li,
                                               nfull);
      dyn_fold_client<T, AE, EDGE, false, NB>(acc, buf, (gptr<const V>)client(i), (gptr<const V>)client(i), sw[i], li, nfull);
    }
    if constexpr (EDGE) {
      if (tail > 0 && li == 0) {  // the < N elements past them, one lane, accumulators in LDS
        for (int i = 0; i < n; ++i) {
          const gptr<const T> base = client(i);
          for (int q = 0; q < tail; ++q) s_tail[q] = fold<FOLD_MULADD>(s_tail[q], load_g<T>(base, nfull * N + q), sw[i], 0.0);
        }
      }
    }
    k += n;
    __syncthreads();  // sp / sw are refilled by the next batch
  }

  // the close: the mode (read with the closing word), and for a final close the segment's
  // divisor and output from the mirror's device table
  const int mode = __builtin_amdgcn_readfirstlane(s_mode);
  if (mode != OUT_ACC) {
    if (threadIdx.x == 0) {
      s_W = dyn_ld_sysf(a.wtot + seg);
      s_out = dyn_ld_sys64(a.outs + seg);
    }
    __syncthreads();
  }
  // the close, a load stage's elements at a time: vector (c * CH + j) * 64 + li of the tile
  // (a partial tile: its whole vectors here, its tail elements from LDS below)
  bool bad_acc = false, bad_res = false;
  const bool final_close = mode != OUT_ACC;
  if (!final_close && k == 0) {  // nothing folded: the accumulator holds nothing new for this round
    if (li == 0) dyn_tile_done(a, EDGE ? a.edge_base + static_cast<int>(blockIdx.x) - 1 : static_cast<int>(blockIdx.x) - 1);
    return;
  }
  const double W = final_close ? s_W : 1.0;
  void* const out_raw = final_close ? reinterpret_cast<void*>(s_out) : reinterpret_cast<void*>(a.acc + acc_base);
  const int64_t out_off = final_close ? td.start : 0;
  const bool f32_out = mode == OUT_F32;
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    double res[CE];
    bool in[CH];
#pragma unroll
    for (int j = 0; j < CH; ++j) in[j] = full || (c * CH + j) * kDynLanes + li < nfull;
#pragma unroll
    for (int i = 0; i < CE; ++i) bad_acc |= in[i / N] && acc[c * CE + i] != acc[c * CE + i];
    if (final_close) {
      exact_div_block<CE>(acc + c * CE, res, W);  // the fused divide (_apply_total_weight, :71-74)
#pragma unroll
      for (int i = 0; i < CE; ++i) bad_res |= in[i / N] && res[i] != res[i];
    } else {
#pragma unroll
      for (int i = 0; i < CE; ++i) res[i] = acc[c * CE + i];
    }
#pragma unroll
    for (int j = 0; j < CH; ++j) {
      if (!in[j]) continue;
      const int64_t e = out_off + static_cast<int64_t>((c * CH + j) * kDynLanes + li) * N;
      const double* r = res + j * N;
      if (f32_out) {
        const gptr<float> op = to_global_mut<float>(out_raw) + e;
#pragma unroll
        for (int q = 0; q < N; q += 2)
          store_out((gptr<f32x2>)(op + q), f32x2{static_cast<float>(r[q]), static_cast<float>(r[q + 1])});
      } else {
        const gptr<double> op = to_global_mut<double>(out_raw) + e;
#pragma unroll
        for (int q = 0; q < N; q += 2) store_out((gptr<f64x2>)(op + q), f64x2{r[q], r[q + 1]});
      }
    }
    __builtin_amdgcn_sched_group_barrier(0x40, CE / 2, 0);  // VMEM_WRITE: the stage's stores
  }
  if (tail > 0 && li == 0) {  // a partial tile's last < N elements
    for (int q = 0; q < tail; ++q) {
      const double t = s_tail[q];
      double r = t;
      bad_acc |= t != t;
      if (final_close) {
        exact_div_block<1>(&t, &r, W);
        bad_res |= r != r;
      }
      const int64_t e = out_off + static_cast<int64_t>(nfull) * N + q;
      if (f32_out) {
        to_global_mut<float>(out_raw)[e] = static_cast<float>(r);
      } else {
        to_global_mut<double>(out_raw)[e] = r;
      }
    }
  }
  const uint64_t ba = __ballot(bad_acc);
  const uint64_t br = __ballot(bad_res);
  if ((ba | br) != 0ull && li == 0) {
    if (ba) raise_flag(a.flag, 0);
    if (br) raise_flag(a.flag, 1);
  }
  if (li == 0) dyn_tile_done(a, EDGE ? a.edge_base + static_cast<int>(blockIdx.x) - 1 : static_cast<int>(blockIdx.x) - 1);
}

// ---------------------------------------------------------------------------------------
// Server-side dequantisation fused into the fold.
//
// The reference's StochasticQuantServerEndpoint.get (simulation_lib/topology/
// quantized_endpoint.py:69-77, level 255 at :102-111) dequantises every arriving update on the
// host — x = norm * sign * slot / level, per tensor (the QSGD codec of the unvendored
// cyy_torch_algorithm.quantization.stochastic) — and FedAVGAlgorithm then folds the dense
// copy (fed_avg_algorithm.py:54-58). Here the quantised record itself is the client "tensor":
//
//   record (16-B aligned, fedavg_qsgd_record_bytes(n) bytes, include/fedavg_hip.h):
//     [0, 8)   norm (fp64; holds the fp32 norm exactly for FEDAVG_QSGD_F32)
//     [8, 12)  level (int32, 1..255)
//     [16, 16 + n)                          slots, one uint8 per element
//     [16 + align16(n), ... + ceil(n / 8))  signs, numpy.packbits order (element i: byte
//                                           i / 8, bit 7 - i % 8; 1 = non-negative)
//
// For one (client, tensor) the dequantised value depends only on (slot, sign), so the weighted
// product the reference folds, round(f64(x) * w), takes at most 2 x 256 values: the workgroup
// tabulates the 256 non-negative ones in LDS (one entry per lane, computed with the reference's
// operation order in the codec's dtype) and every element folds acc + (sign ? p[slot] :
// -p[slot]). The negative half is exact: every step (norm * ±1, * slot, / level, widening, * w)
// rounds symmetrically. So the fold stays bit-identical to dequantise-then-FedAvg while HBM
// carries 1.125 B per element per client instead of 4 (fp32) or 8 (fp64).
//
// Geometry: one 256-lane workgroup per 4096-element tile; lane li owns elements
// [16 li, 16 li + 16) (one 16-B slot load + one 2-B sign load per client; a wave reads 1 KiB of
// slots contiguously). Clients go in groups of QG: the group's loads are issued, its QG tables
// are built into one of two LDS buffers, one barrier, then the fold in arrival order.
// The built geometry (wider tiles, 512-entry signed tables, deeper prefetch, one-wave
// workgroups, a pipelined fold and packed loads were measured no faster and are not kept).
constexpr int kQsgdAE = 16;       // elements per lane (256-lane workgroups on 4096-element tiles)
constexpr int kQsgdGroup = 2;     // clients per group (82 VGPRs, 5 waves per SIMD)
#ifndef FEDAVG_QSGD_RB  // table reads per batch before their adds (elements of a lane)
#define FEDAVG_QSGD_RB 4
#endif
constexpr int kQsgdSlots = 256;   // slot values
constexpr int kQsgdTable = 256;   // |p| per slot value
constexpr int kQsgdBufs = 2;      // LDS table buffers: the next group's DMAs land while a group folds
constexpr int kQsgdTileLanes = 4096 / kQsgdAE;  // lanes covering one 4096-element tile
constexpr int kQsgdLanes = kQsgdTileLanes;       // lanes per workgroup (one tile each)
static_assert(kQsgdGroup * kQsgdTable / 128 == kQsgdLanes / 64, "one 1-KiB table DMA chunk per wave and group");

template <typename DQ>
__device__ __forceinline__ double qsgd_product(double norm, int level, int slot, double w) {
  // torch evaluates `norm * sign * slot / level` left to right in the codec's dtype; with
  // sign = +1 the first product is exact, so the non-negative value is (norm * slot) / level
  // (IEEE division, as the codec does it).
  const DQ n = static_cast<DQ>(norm);
  const DQ v = (n * static_cast<DQ>(slot)) / static_cast<DQ>(level);
  const double x = static_cast<double>(v);  // .to(float64), fed_avg_algorithm.py:54
  return x * w;
}

// The |product| tables of one call, built once per (client, tensor) instead of once per tile:
// table[seg][k][s] = |round(f64(x_hat(s)) * w)| for slot value s of client k's record of segment
// seg (the sign is applied per element in the fold). One 256-lane workgroup per (client, segment)
// of the segments [seg_begin, seg_begin + gridDim.y); 2 KiB per table, L2 / MALL resident for
// the tile kernel's LDS-DMA loads.
template <typename DQ>
__global__ __launch_bounds__(kQsgdSlots) void qsgd_table_kernel(CallTables tab, int32_t K, int32_t seg_begin,
                                                                double* qtab) {
  const int seg = seg_begin + static_cast<int>(blockIdx.y);
  const int k = static_cast<int>(blockIdx.x);
  if (k >= to_const<int32_t>(tab.kseg)[seg]) return;
  const int64_t row = static_cast<int64_t>(seg) * K + k;
  const int64_t trow = static_cast<int64_t>(blockIdx.y) * K + k;  // row of the launch's table block
  const void* rec = reinterpret_cast<const void*>(to_const<uint64_t>(tab.cptrs)[row]);
  const double norm = to_const<double>(rec)[0];
  const int level = to_const<int32_t>(rec)[2];
  const double w = to_const<double>(tab.w)[row];
  const int s = static_cast<int>(threadIdx.x);
  const double p = __builtin_fabs(qsgd_product<DQ>(norm, level, s, w));
  // entry 0 is a zero (or a NaN, for a non-finite norm / weight): its sign bit carries the
  // client's product sign, signbit(norm) ^ signbit(w), which the fold reads with one broadcast
  // LDS load instead of keeping norm and weight in SGPRs (the fold inserts every element's sign
  // itself, so entry 0's magnitude is all the fold takes from it)
  const bool flip = __builtin_signbit(norm) != __builtin_signbit(w);
  qtab[trow * kQsgdTable + s] = (s == 0 && flip) ? -p : p;
}

__device__ __forceinline__ void wait_vmcnt0() {
  // s_waitcnt vmcnt(0) (expcnt / lgkmcnt: no wait): every vector memory op of this wave landed,
  // LDS-DMA included (the compiler does not track those)
  __builtin_amdgcn_s_waitcnt((7 << 4) | (15 << 8));
}

// Continuing accumulator of a record tile (lane slice [e0, e0 + AE) of the tile), or the -0.0
// identity. Returns whether the accumulator held data.
template <bool FULL, int AE>
__device__ __forceinline__ bool record_tile_acc_in(const KArgs& a, int seg, int64_t acc_base, int e0, int count,
                                                   double (&acc)[AE]) {
#pragma unroll
  for (int i = 0; i < AE; ++i) acc[i] = -0.0;  // additive identity (see tile_body)
  if (a.zero_init || !to_const<int32_t>(a.tab.acc_in)[seg]) return a.zero_init != 0;
  const gptr<const double> ap = to_global<double>(a.acc + acc_base) + e0;
#pragma unroll
  for (int j = 0; j < AE; j += 2) {
    if (FULL || e0 + j + 2 <= count) {
      const f64x2 d = *(gptr<const f64x2>)(ap + j);
      acc[j] = d.x;
      acc[j + 1] = d.y;
    } else {
      if (e0 + j < count) acc[j] = ap[j];
      if (e0 + j + 1 < count) acc[j + 1] = ap[j + 1];
    }
  }
  return true;
}

// Epilogue of a record tile (QSGD / NNADQ kernels): store the lane's fp64 accumulator slice, or
// divide it by the segment's total weight (exact_div_block) into the fp32 / fp64 output; NaN
// flags as in tile_body.
template <int OUT, bool FULL, bool VEC, int AE>
__device__ __forceinline__ void record_tile_finish(const KArgs& a, const TileDesc& td, int64_t acc_base, int e0,
                                                   const double (&acc)[AE]) {
  const int seg = td.seg;
  const int count = td.count;
  bool bad_acc = false;
#pragma unroll
  for (int j = 0; j < AE; ++j) bad_acc |= (FULL || e0 + j < count) && (acc[j] != acc[j]);

  if constexpr (OUT == OUT_ACC) {
    const gptr<double> ap = to_global_mut<double>(a.acc + acc_base) + e0;
#pragma unroll
    for (int j = 0; j < AE; j += 2) {
      if (FULL || e0 + j + 2 <= count) {
        *(gptr<f64x2>)(ap + j) = f64x2{acc[j], acc[j + 1]};
      } else {
        if (e0 + j < count) ap[j] = acc[j];
        if (e0 + j + 1 < count) ap[j + 1] = acc[j + 1];
      }
    }
    if (__ballot(bad_acc) != 0ull && (threadIdx.x & 63) == 0) raise_flag(a.flag, 0);
  } else {
    const double W = to_const<double>(a.tab.wtot)[seg];
    double res[AE];
    bool bad_res = false;
    exact_div_block<AE>(acc, res, W);
#pragma unroll
    for (int j = 0; j < AE; ++j) bad_res |= (FULL || e0 + j < count) && (res[j] != res[j]);
    void* const out_raw = reinterpret_cast<void*>(to_const<uint64_t>(a.tab.outs)[seg]);
    if constexpr (OUT == OUT_F32) {
      const gptr<float> op = to_global_mut<float>(out_raw) + td.start + e0;
#pragma unroll
      for (int j = 0; j < AE; j += 4) {
        if (VEC && (FULL || e0 + j + 4 <= count)) {
          *(gptr<f32x4>)(op + j) = f32x4{static_cast<float>(res[j]), static_cast<float>(res[j + 1]),
                                          static_cast<float>(res[j + 2]), static_cast<float>(res[j + 3])};
        } else {
#pragma unroll
          for (int q = 0; q < 4; ++q)
            if (e0 + j + q < count) op[j + q] = static_cast<float>(res[j + q]);
        }
      }
    } else {
      const gptr<double> op = to_global_mut<double>(out_raw) + td.start + e0;
#pragma unroll
      for (int j = 0; j < AE; j += 2) {
        if (VEC && (FULL || e0 + j + 2 <= count)) {
          *(gptr<f64x2>)(op + j) = f64x2{res[j], res[j + 1]};
        } else {
          if (e0 + j < count) op[j] = res[j];
          if (e0 + j + 1 < count) op[j + 1] = res[j + 1];
        }
      }
    }
    const uint64_t ba = __ballot(bad_acc);
    const uint64_t br = __ballot(bad_res);
    if ((ba | br) != 0ull && (threadIdx.x & 63) == 0) {
      if (ba) raise_flag(a.flag, 0);
      if (br) raise_flag(a.flag, 1);
    }
  }
}

// f(integral_constant<int, I>) for I in [I0, N), unrolled at compile time
template <int I, int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<I + 1, N>(f);
  }
}

template <int N>
__device__ __forceinline__ void qsgd_wait_vmcnt() {
  // s_waitcnt vmcnt(N) (bits 3:0 and 15:14; expcnt / lgkmcnt: no wait)
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

template <int OUT, typename DQ, bool FULL, bool VEC>
__device__ __forceinline__ void qsgd_tile_body(const KArgs& a, const TileDesc& td, double (*lut)[kQsgdGroup][kQsgdTable]) {
  constexpr int AE = kQsgdAE;
  constexpr int G = kQsgdGroup;
  constexpr int NB = kQsgdBufs;
  const int seg = td.seg;
  const int count = td.count;
  const int li = static_cast<int>(threadIdx.x);
  const int e0 = li * AE;  // first element of this lane within the tile
  const bool lane_live = FULL || e0 < count;

  const int kseg = to_const<int32_t>(a.tab.kseg)[seg];
  const kptr<uint64_t> cp = to_const<uint64_t>(a.tab.cptrs) + static_cast<int64_t>(seg) * a.K;
  const int64_t acc_base = to_const<int64_t>(a.segs)[2 * seg] + td.start;
  const int64_t numel = to_const<int64_t>(a.segs)[2 * seg + 1];
  // a lane past the tile's end loads from the record's start instead (in bounds; its sums are
  // never stored), so every wave issues the same vector memory operations per group and the
  // counted waits below hold for every wave
  const int64_t slot_off = lane_live ? 16 + td.start + e0 : 0;
  const int64_t sign_off = lane_live ? 16 + ((numel + 15) & ~int64_t(15)) + (td.start + e0) / 8 : 0;

  double acc[AE];
  bool have = record_tile_acc_in<FULL, AE>(a, seg, acc_base, e0, count, acc);

  // Client loads of one group (slots + sign words) and its G |product| tables (global -> LDS by
  // DMA: the group's 2-KiB tables are four 1-KiB chunks, wave w moves chunk w — the last table
  // again for a short group), issued one group ahead of the group's fold into the other of two
  // LDS buffers: every wave issues the same 2 G + 1 vector memory operations per group (a wave
  // retires a group with vmcnt(0) before issuing the next one).
  struct GroupRegs {
    u32x4 slots[G];     // AE slot bytes
    uint32_t signs[G];  // AE sign bits (16-bit load)
  };
  const int wave = __builtin_amdgcn_readfirstlane(li >> 6);
  const int lane = li & 63;
  const double* const tabs = a.qtab + static_cast<int64_t>(seg - a.qtab_seg0) * a.K * kQsgdTable;
  auto issue = [&](GroupRegs& r, int buf, int k) {
    const int n = min(G, kseg - k);  // wave-uniform
#pragma unroll
    for (int c = 0; c < G; ++c) {
      const int kc = k + min(c, n - 1);
      const uint64_t rp = cp[kc];
      // inline-asm loads: the compiler does not track them, so it inserts no waits of its own
      // (its loop-carried tracking otherwise drains vmcnt to 0 between groups); the counted wait
      // at the top of each step covers every use, and no register of a pending load is reused
      // before that use (the value is live from here to the fold)
      asm volatile("global_load_dwordx4 %0, %1, off nt" : "=v"(r.slots[c]) : "v"(rp + slot_off) : "memory");
      asm volatile("global_load_ushort %0, %1, off" : "=v"(r.signs[c]) : "v"(rp + sign_off) : "memory");
    }
    // this wave's 1-KiB chunk of the group's tables
    const int cl = wave / (kQsgdTable / 128);    // client of the group
    const int part = wave % (kQsgdTable / 128);  // 128 doubles each
    const double* src = tabs + static_cast<int64_t>(k + min(cl, n - 1)) * kQsgdTable + part * 128;
    double* dst = lut[buf][cl] + part * 128;
    __builtin_amdgcn_global_load_lds((void FEDAVG_AS_GLOBAL*)(src + 2 * lane),
                                     (void __attribute__((address_space(3)))*)dst, 16, 0, 0);
  };
  // Fold of one group from LDS buffer B (compile-time, so every table read is
  // `ds_read_b64 v, v_off offset:<buffer base>`). The table holds |p|; the sign of each
  // product is sign(x_hat) ^ sign(w) = (element negative) ^ signbit(norm) ^ signbit(w)
  // (every step of the dequantisation and the product is sign-symmetric, zeros included) —
  // the client's signbit(norm) ^ signbit(w) is entry 0's sign bit (qsgd_table_kernel) — and is
  // inserted into the high word with one bit-field insert.
  auto run = [&](auto buf_tag, const GroupRegs& r, int k) {
    constexpr int B = decltype(buf_tag)::value;
    const int n = min(G, kseg - k);  // wave-uniform
#pragma unroll
    for (int c = 0; c < G; ++c) {
      if (c < n) {
        const char* tab = reinterpret_cast<const char*>(lut[B][c]);
        const int32_t t0hi = reinterpret_cast<const int32_t*>(tab)[1];  // broadcast read
        // per element: 1 = negative product
        const uint32_t neg = r.signs[c] ^ ~static_cast<uint32_t>(t0hi >> 31);
        // RB table reads in flight before their adds (all 16 by default; the compiler would
        // otherwise keep ~4 outstanding and wait on each batch); fewer per batch = fewer VGPRs
        constexpr int RB = FEDAVG_QSGD_RB < AE ? FEDAVG_QSGD_RB : AE;
#pragma unroll
        for (int j0 = 0; j0 < AE; j0 += RB) {
          double pav[RB];
#pragma unroll
          for (int jj = 0; jj < RB; ++jj) {
            const int j = j0 + jj;
            const uint32_t word = r.slots[c][j >> 2];
            const uint32_t off = ((word >> (8 * (j & 3))) & 0xffu) << 3;
            pav[jj] = *reinterpret_cast<const double*>(tab + off);
          }
          // the batch's reads are issued before its adds (the compiler would otherwise keep ~4
          // outstanding and wait on each)
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int jj = 0; jj < RB; ++jj) {
            const int j = j0 + jj;
            // numpy.packbits order: element j < 8 of this lane is bit 7 - j of the low byte of
            // the little-endian sign word, element j >= 8 bit 15 - (j - 8)
            const int bit = (j < 8) ? (7 - j) : (15 - (j - 8));
            const uint32_t sb = neg << (31 - bit);
            const uint64_t u = static_cast<uint64_t>(__double_as_longlong(pav[jj]));
            const uint32_t hi = (sb & 0x80000000u) | (static_cast<uint32_t>(u >> 32) & 0x7fffffffu);
            const double p = __longlong_as_double(static_cast<long long>((static_cast<uint64_t>(hi) << 32) | (u & 0xffffffffull)));
            acc[j] = acc[j] + p;
          }
        }
      }
    }
  };
  // Group i folds from buffer i % 2. At the top of each step a wave waits until its loads and
  // DMAs of that group landed, and the barrier publishes every wave's DMAs; only then is group
  // i + 1 issued, into buffer (i + 1) % 2 — the buffer of group i - 1, which the barrier proves
  // every wave has finished reading.
  GroupRegs r[NB];
  if (kseg > 0) issue(r[0], 0, 0);
  for (int k = 0; k < kseg; k += NB * G) {
    bool go = true;
    static_for<0, NB>([&](auto b_tag) {
      constexpr int b = decltype(b_tag)::value;
      const int kk = k + b * G;
      if (!go || kk >= kseg) {  // wave-uniform
        go = false;
        return;
      }
      // past the last group the issue repeats the last group: L2 hits into a buffer nobody reads,
      // so every step's count is the same
      __builtin_amdgcn_sched_barrier(0);
      qsgd_wait_vmcnt<0>();
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      issue(r[(b + 1) % NB], (b + 1) % NB, min(kk + G, (kseg - 1) / G * G));
      run(b_tag, r[b], kk);
    });
  }
  // the repeated issues past the last group are still in flight: no DMA may land in LDS after
  // the workgroup has left it
  qsgd_wait_vmcnt<0>();
  have = have || (kseg > 0);
  if (!have) return;
  record_tile_finish<OUT, FULL, VEC, AE>(a, td, acc_base, e0, acc);
}

// Block b runs on XCD b % 8 (round-robin dispatch); the launch's tiles are segment-ordered, so
// giving XCD x the x-th contiguous eighth of them (the bijective form for any grid size) keeps each
// segment's |p| tables in one or two XCD L2s instead of all eight: 953 -> 882 MB fetched per
// 64 x ResNet-18 launch (profiles/r04_traffic_qsgd.json). Placement affects speed only.
__device__ __forceinline__ int xcd_contiguous(int b, int n) {
  constexpr int kX = 8;
  const int q = n / kX, r = n % kX;
  const int x = b % kX, k = b / kX;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + k;
}

template <int OUT, typename DQ, bool VEC>
__global__ __launch_bounds__(kQsgdLanes) void qsgd_tile_kernel(KArgs a) {
  __shared__ double lut[kQsgdBufs][kQsgdGroup][kQsgdTable];
  const int b = xcd_contiguous(static_cast<int>(blockIdx.x), static_cast<int>(gridDim.x));
  const TileDesc td = load_tile(a.tiles, a.tile_begin + b);
  if (td.count == kTile1) {
    qsgd_tile_body<OUT, DQ, true, VEC>(a, td, lut);
  } else {
    qsgd_tile_body<OUT, DQ, false, VEC>(a, td, lut);
  }
}

// Diagnostic for quantised clients: which record dequantises to a NaN somewhere.
template <typename DQ>
__global__ __launch_bounds__(kThreads) void qsgd_nan_scan_kernel(const TileDesc* tiles, const SegDesc* segs,
                                                                const void* const* cptrs_tk, int32_t K,
                                                                int32_t* bad) {
  const TileDesc td = load_tile(tiles, blockIdx.x);
  const int k = blockIdx.y;
  const uint64_t raw = to_const<uint64_t>(cptrs_tk)[static_cast<int64_t>(td.seg) * K + k];
  if (raw == 0) return;
  const gptr<const uint8_t> rp = to_global<uint8_t>(reinterpret_cast<const void*>(raw));
  const double norm = *(gptr<const double>)rp;
  const int level = *(gptr<const int32_t>)(rp + 8);
  bool b = false;
  for (int i = threadIdx.x; i < td.count; i += kThreads) {
    const double x = qsgd_product<DQ>(norm, level, rp[16 + td.start + i], 1.0);
    b |= (x != x);
  }
  (void)segs;
  if (__ballot(b) != 0ull && (threadIdx.x & 63) == 0) atomicOr(reinterpret_cast<unsigned*>(bad + k), 1u);
}

// ---------------------------------------------------------------------------------------
// NNADQ records (NNADQServerEndpoint, simulation_lib/topology/quantized_endpoint.py:114-142:
// the deterministic codec of the unvendored cyy_torch_algorithm.quantization.deterministic,
// dequantised by QuantServerEndpoint.get, :69-77, before the fold). The record is the client
// "tensor" here too:
//
//   record (16-B aligned, fedavg_nnadq_record_bytes(n) = 32 + align16(n) bytes):
//     [0, 8)   lo (fp64; holds the fp32 value exactly for FEDAVG_NNADQ_F32)
//     [8, 16)  step (fp64, likewise)
//     [16, 20) levels (int32, 1..255; informational — codes are never above it)
//     [32, 32 + n)  codes, one uint8 per element
//
//   x_hat = code * step + lo in the codec's dtype, two roundings (-ffp-contract=off)
//
// No table: one multiply and one add in the codec's dtype is cheaper than a table read, so each
// element is dequantised in registers and folded like a dense input, FOLD kinds included (the
// fused fold when the host proves every x * w exact — fp32 codec values and integer weights).
// HBM carries 1 B per element per client. Geometry: 256-lane workgroups on the 4096-element
// tiles, lane li owns elements [16 li, 16 li + 16) (one 16-B code load per client: a wave reads
// 1 KiB contiguously); clients in groups of kNnadqGroup, group g + 1's loads issued before group
// g's fold (a register double buffer; no LDS, no barriers).
constexpr int kNnadqHeader = 32;
constexpr int kNnadqLanes = 256;
constexpr int kNnadqAE = 16;
// 2-client groups (80 VGPRs, 6 waves per SIMD); inline-asm code loads with counted waits and a
// packed fp32 dequantisation were measured slower and are not kept
constexpr int kNnadqGroup = 2;
static_assert(kNnadqLanes * kNnadqAE == kTile1, "NNADQ launches walk the 4096-element tile table");

template <typename DQ>
__device__ __forceinline__ double nnadq_value(uint32_t code, DQ step, DQ lo) {
  const DQ c = static_cast<DQ>(code);
  const DQ p = c * step;  // rounded in the codec's dtype
  const DQ v = p + lo;    // rounded again (no contraction)
  return static_cast<double>(v);  // .to(float64), fed_avg_algorithm.py:54
}

template <int OUT, typename DQ, int FOLD, bool FULL, bool VEC>
__device__ __forceinline__ void nnadq_tile_body(const KArgs& a, const TileDesc& td) {
  constexpr int AE = kNnadqAE;
  constexpr int G = kNnadqGroup;
  const int seg = td.seg;
  const int count = td.count;
  const int li = static_cast<int>(threadIdx.x);
  const int e0 = li * AE;
  const bool lane_live = FULL || e0 < count;  // a 16-B load at e0 < numel stays in the record

  const int kseg = to_const<int32_t>(a.tab.kseg)[seg];
  const kptr<uint64_t> cp = to_const<uint64_t>(a.tab.cptrs) + static_cast<int64_t>(seg) * a.K;
  const kptr<double> wp = to_const<double>(a.tab.w) + static_cast<int64_t>(seg) * a.K;
  const int64_t acc_base = to_const<int64_t>(a.segs)[2 * seg] + td.start;
  const int64_t code_off = kNnadqHeader + td.start + e0;

  double acc[AE];
  bool have = record_tile_acc_in<FULL, AE>(a, seg, acc_base, e0, count, acc);

  struct GroupRegs {
    u32x4 codes[G];
    DQ lo[G], step[G];  // wave-uniform (SGPRs): record header
    double wk[G];
  };
  auto issue = [&](GroupRegs& r, int k) {
    const int n = min(G, kseg - k);  // wave-uniform
#pragma unroll
    for (int c = 0; c < G; ++c) {
      if (c < n) {
        const uint64_t rec = cp[k + c];
        const kptr<double> hdr = to_const<double>(reinterpret_cast<const void*>(rec));
        r.lo[c] = static_cast<DQ>(hdr[0]);
        r.step[c] = static_cast<DQ>(hdr[1]);
        r.wk[c] = wp[k + c];
        if (lane_live) {
          const gptr<const uint8_t> rp = to_global<uint8_t>(reinterpret_cast<const void*>(rec));
          r.codes[c] = __builtin_nontemporal_load((gptr<const u32x4>)(rp + code_off));
        } else {
          r.codes[c] = u32x4{0u, 0u, 0u, 0u};
        }
      }
    }
  };
  auto run = [&](const GroupRegs& r, int k) {
    const int n = min(G, kseg - k);  // wave-uniform
#pragma unroll
    for (int c = 0; c < G; ++c) {
      if (c < n) {
#pragma unroll
        for (int j = 0; j < AE; ++j) {
          const uint32_t code = (r.codes[c][j >> 2] >> (8 * (j & 3))) & 0xffu;
          acc[j] = fold<FOLD>(acc[j], nnadq_value<DQ>(code, r.step[c], r.lo[c]), r.wk[c], 0.0);
        }
      }
    }
  };
  GroupRegs r0, r1;
  if (kseg > 0) issue(r0, 0);
  for (int k = 0; k < kseg; k += 2 * G) {
    const bool second = k + G < kseg;
    if (second) issue(r1, k + G);
    run(r0, k);
    if (second) {
      if (k + 2 * G < kseg) issue(r0, k + 2 * G);
      run(r1, k + G);
    }
  }
  have = have || (kseg > 0);
  if (!have) return;
  record_tile_finish<OUT, FULL, VEC, AE>(a, td, acc_base, e0, acc);
}

template <int OUT, typename DQ, int FOLD, bool VEC>
__global__ __launch_bounds__(kNnadqLanes) void nnadq_tile_kernel(KArgs a) {
  const TileDesc td = load_tile(a.tiles, a.tile_begin + static_cast<int>(blockIdx.x));
  if (td.count == kTile1) {
    nnadq_tile_body<OUT, DQ, FOLD, true, VEC>(a, td);
  } else {
    nnadq_tile_body<OUT, DQ, FOLD, false, VEC>(a, td);
  }
}

// Diagnostic for NNADQ clients: which record dequantises to a NaN somewhere.
template <typename DQ>
__global__ __launch_bounds__(kThreads) void nnadq_nan_scan_kernel(const TileDesc* tiles, const void* const* cptrs_tk,
                                                                 int32_t K, int32_t* bad) {
  const TileDesc td = load_tile(tiles, blockIdx.x);
  const int k = blockIdx.y;
  const uint64_t raw = to_const<uint64_t>(cptrs_tk)[static_cast<int64_t>(td.seg) * K + k];
  if (raw == 0) return;
  const gptr<const uint8_t> rp = to_global<uint8_t>(reinterpret_cast<const void*>(raw));
  const DQ lo = static_cast<DQ>(*(gptr<const double>)rp);
  const DQ step = static_cast<DQ>(*(gptr<const double>)(rp + 8));
  bool b = false;
  for (int i = threadIdx.x; i < td.count; i += kThreads) {
    const double x = nnadq_value<DQ>(rp[kNnadqHeader + td.start + i], step, lo);
    b |= (x != x);
  }
  if (__ballot(b) != 0ull && (threadIdx.x & 63) == 0) atomicOr(reinterpret_cast<unsigned*>(bad + k), 1u);
}

// Diagnostic: per-client "holds a NaN" flags (error path only, fed_avg_algorithm.py:35).
template <typename T>
__global__ __launch_bounds__(kThreads) void nan_scan_kernel(const TileDesc* tiles,
                                                           const void* const* cptrs_tk,
                                                           int32_t K, int32_t* bad) {
  const TileDesc td = load_tile(tiles, blockIdx.x);
  const int k = blockIdx.y;
  const uint64_t raw = to_const<uint64_t>(cptrs_tk)[static_cast<int64_t>(td.seg) * K + k];
  if (raw == 0) return;
  const gptr<const T> p = to_global<T>(reinterpret_cast<const void*>(raw)) + td.start;
  bool b = false;
  for (int i = threadIdx.x; i < td.count; i += kThreads) {
    const double x = load_g<T>(p, i);
    b |= (x != x);
  }
  if (__ballot(b) != 0ull && (threadIdx.x & 63) == 0) atomicOr(reinterpret_cast<unsigned*>(bad + k), 1u);
}

// Bandwidth probes (the measured HBM ceiling next to the roofline, and the known byte counts
// that calibrate FETCH_SIZE / WRITE_SIZE for the main kernel's access pattern): mode 0 =
// 16-B/lane copy, mode 1 = 16-B/lane read-only stream; both non-temporal like the main kernel,
// 8 loads in flight per lane.
__global__ __launch_bounds__(kThreads) void bw_copy_kernel(const f32x4* __restrict__ src,
                                                          f32x4* __restrict__ dst, int64_t n) {
  constexpr int G = 8;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kThreads * G;
  for (int64_t base = static_cast<int64_t>(blockIdx.x) * kThreads * G; base < n; base += stride) {
    f32x4 v[G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const int64_t i = base + g * kThreads + threadIdx.x;
      if (i < n) v[g] = __builtin_nontemporal_load(src + i);
    }
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const int64_t i = base + g * kThreads + threadIdx.x;
      if (i < n) __builtin_nontemporal_store(v[g], dst + i);
    }
  }
}
__global__ __launch_bounds__(kThreads) void bw_read_kernel(const f32x4* __restrict__ src,
                                                          uint32_t* __restrict__ dst, int64_t n) {
  constexpr int G = 8;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kThreads * G;
  uint32_t x = 0;
  for (int64_t base = static_cast<int64_t>(blockIdx.x) * kThreads * G; base < n; base += stride) {
    f32x4 v[G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const int64_t i = base + g * kThreads + threadIdx.x;
      v[g] = (i < n) ? __builtin_nontemporal_load(src + i) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int g = 0; g < G; ++g)
      x ^= __float_as_uint(v[g].x) ^ __float_as_uint(v[g].y) ^ __float_as_uint(v[g].z) ^ __float_as_uint(v[g].w);
  }
  if (x == 0x9e3779b9u) dst[blockIdx.x] = x;  // practically never taken; keeps loads live
}

// ---------------------------------------------------------------------------------------
// Per-element weights: a _get_weight override that returns a tensor of the parameter's shape
// (fed_avg_algorithm.py:51-62: `tmp = x.to(f64) * weight`, `acc += tmp`, `total += weight`, and
// :94-96 `acc / total`, both elementwise). The total is a per-element buffer too; the reference
// keeps it in the dtype of the first weight (torch's in-place add), so segments whose first weight
// is fp32 round it to fp32 after every add (an fp32 sum of two fp32 values, computed in fp64 and
// rounded once, is the correctly rounded fp32 sum). A NULL weight pointer takes a scalar weight
// (names whose override returns a number). One workgroup per tile, clients in arrival order.
// ---------------------------------------------------------------------------------------
struct EwArgs {
  const void* const* x;   // [T][K] compacted client pointers
  const void* const* w;   // [T][K] weight pointers (NULL = scalar)
  const double* ws;       // [T][K] scalar weights
  const int32_t* wdt;     // [T][K] weight dtype (FEDAVG_F32 / FEDAVG_F64)
  const int32_t* kseg;    // [T] clients of the segment in this call
  const int32_t* flags;   // [T] bit 0: the accumulator holds data, bit 1: totals are fp32
  int32_t stride;         // row stride of the [T][K] tables
  double* acc;
  double* tot;
};

template <typename T>
__global__ __launch_bounds__(kThreads) void ew_fold_kernel(const TileDesc* __restrict__ tiles,
                                                           const SegDesc* __restrict__ segs, EwArgs a) {
  const TileDesc td = load_tile(tiles, blockIdx.x);
  const int t = td.seg;
  const int K = a.kseg[t];
  const int f = a.flags[t];
  const int64_t base = segs[t].acc_off + td.start;
  for (int i = threadIdx.x; i < td.count; i += kThreads) {
    bool have = (f & 1) != 0;
    double s = have ? a.acc[base + i] : 0.0;
    double tw = have ? a.tot[base + i] : 0.0;
    for (int k = 0; k < K; ++k) {
      const int64_t idx = static_cast<int64_t>(t) * a.stride + k;
      const double x = load_g<T>(to_global<T>(a.x[idx]) + td.start, i);
      const void* wp = a.w[idx];
      double w = a.ws[idx];
      if (wp != nullptr)
        w = (a.wdt[idx] == FEDAVG_F32) ? static_cast<double>(static_cast<const float*>(wp)[td.start + i])
                                       : static_cast<const double*>(wp)[td.start + i];
      const double p = x * w;  // rounded, then added (no contraction: -ffp-contract=off)
      if (have) {
        s = s + p;
        tw = tw + w;
      } else {
        s = p;
        tw = w;
        have = true;
      }
      if (f & 2) tw = static_cast<double>(static_cast<float>(tw));
    }
    a.acc[base + i] = s;
    a.tot[base + i] = tw;
  }
}

template <typename O>
__global__ __launch_bounds__(kThreads) void ew_finalize_kernel(const TileDesc* __restrict__ tiles,
                                                               const SegDesc* __restrict__ segs,
                                                               const double* __restrict__ acc,
                                                               const double* __restrict__ tot, void* const* outs,
                                                               uint32_t* flag) {
  const TileDesc td = load_tile(tiles, blockIdx.x);
  const int64_t base = segs[td.seg].acc_off + td.start;
  O* out = static_cast<O*>(reinterpret_cast<void*>(to_const<uint64_t>(outs)[td.seg])) + td.start;
  bool bad_acc = false, bad_res = false;
  for (int i = threadIdx.x; i < td.count; i += kThreads) {
    const double v = acc[base + i];
    const double r = v / tot[base + i];
    bad_acc |= (v != v);
    bad_res |= (r != r);
    out[i] = static_cast<O>(r);
  }
  const uint64_t ba = __ballot(bad_acc), br = __ballot(bad_res);
  if ((ba | br) != 0ull && (threadIdx.x & 63) == 0) {
    if (ba) raise_flag(flag, 0);
    if (br) raise_flag(flag, 1);
  }
}

// ---------------------------------------------------------------------------------------
// Scatter exchange of the multi-GPU round (sharded_comm.cpp): after the fp64
// partials are reduce-scattered, rank r holds the global sums of an element window [lo, hi) of
// the accumulator (any alignment, may span segments and their padding). It divides its window by
// the per-segment total weights (_apply_total_weight, fed_avg_algorithm.py:71-74, with the :93 /
// :97 NaN checks) into a result buffer kept in accumulator coordinates; the windows are gathered
// to the root, which copies the result into the caller's per-segment outputs.
// ---------------------------------------------------------------------------------------
constexpr int kWinElems = 8;  // contiguous elements per lane of the window kernel

template <typename O>
__global__ __launch_bounds__(kThreads) void window_finalize_kernel(const double* __restrict__ src, int64_t lo,
                                                                   int64_t n, const SegDesc* __restrict__ segs,
                                                                   int32_t T, const double* __restrict__ wtot,
                                                                   O* __restrict__ res, uint32_t* flag) {
  const int64_t e0 = (static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x) * kWinElems;
  bool bad_acc = false, bad_res = false;
  if (e0 < n) {
    // segment of the first element: the last segment starting at or before it (binary search)
    const int64_t p0 = lo + e0;
    int s = 0, hi_s = T - 1;
    while (s < hi_s) {
      const int mid = (s + hi_s + 1) >> 1;
      if (segs[mid].acc_off <= p0) s = mid;
      else hi_s = mid - 1;
    }
    int64_t seg_off = segs[s].acc_off, seg_n = segs[s].numel;
    double W = wtot[s];
#pragma unroll
    for (int j = 0; j < kWinElems; ++j) {
      const int64_t e = e0 + j;
      if (e >= n) break;
      const int64_t p = lo + e;
      while (s + 1 < T && segs[s + 1].acc_off <= p) {
        ++s;
        seg_off = segs[s].acc_off;
        seg_n = segs[s].numel;
        W = wtot[s];
      }
      if (p - seg_off >= seg_n) continue;  // alignment padding between segments
      const double v = src[e];
      const double r = v / W;
      bad_acc |= (v != v);
      bad_res |= (r != r);
      res[p] = static_cast<O>(r);
    }
  }
  const uint64_t ba = __ballot(bad_acc), br = __ballot(bad_res);
  if ((ba | br) != 0ull && (threadIdx.x & 63) == 0) {
    if (ba) raise_flag(flag, 0);
    if (br) raise_flag(flag, 1);
  }
}

// Root: result (accumulator coordinates) -> the caller's per-segment outputs, one workgroup per
// tile. A NaN in the gathered result (another rank's :93 / :97 failure) raises the result flag.
template <typename O>
__global__ __launch_bounds__(kThreads) void copy_out_kernel(const TileDesc* __restrict__ tiles,
                                                            const SegDesc* __restrict__ segs,
                                                            const O* __restrict__ res, void* const* outs,
                                                            uint32_t* flag) {
  const TileDesc td = load_tile(tiles, blockIdx.x);
  const gptr<const O> src = to_global<O>(res + segs[td.seg].acc_off + td.start);
  const gptr<O> dst = to_global_mut<O>(reinterpret_cast<void*>(to_const<uint64_t>(outs)[td.seg])) + td.start;
  bool bad = false;
  for (int i = threadIdx.x; i < td.count; i += kThreads) {
    const O v = src[i];
    bad |= (v != v);
    dst[i] = v;
  }
  if (__ballot(bad) != 0ull && (threadIdx.x & 63) == 0) raise_flag(flag, 1);
}

// ---------------------------------------------------------------------------------------
// Single-process multi-device exchange (multi_device.cpp, include/fedavg_hip.h fedavg_multi_*).
// Device j owns a window of tiles; the partial kernels of every device wrote their fp64 partial
// of that window into device j's receive slots (peer stores over xGMI) or left it in their own
// accumulators (read here through the peer mapping). One workgroup per tile sums the G partials
// in device order — S = S_0; S = S + S_1; ... — divides by the segment's total weight
// (fed_avg_algorithm.py:71-99: the :93 / :97 NaN checks fused) and stores the result into the
// root's outputs, which on a non-root device is a peer store. 256 lanes x 8 fp64 pairs: one
// wave instruction moves 1 KiB of a slot contiguously.
// ---------------------------------------------------------------------------------------
constexpr int kMaxDevices = 16;
struct SlotPtrs {
  const double* p[kMaxDevices];
};
constexpr int kCombinePairs = 8;  // f64x2 per lane: 256 lanes x 16 elements = one 4096-element tile
static_assert(kCombinePairs * 2 * kThreads == kTile1, "one workgroup per exact-order tile");

template <typename O, bool VEC>
__global__ __launch_bounds__(kThreads) void multi_combine_kernel(const TileDesc* __restrict__ tiles, int32_t tile_begin,
                                                                 const SegDesc* __restrict__ segs, SlotPtrs slots,
                                                                 int32_t G, const double* wtot, void* const* outs,
                                                                 uint32_t* flag) {
  const TileDesc td = load_tile(tiles, tile_begin + static_cast<int64_t>(blockIdx.x));
  const int64_t base = to_const<int64_t>(segs)[2 * td.seg] + td.start;  // SegDesc::acc_off
  const int li = static_cast<int>(threadIdx.x);
  double acc[2 * kCombinePairs];
#pragma unroll
  for (int i = 0; i < 2 * kCombinePairs; ++i) acc[i] = 0.0;
  const bool full = td.count == kCombinePairs * 2 * kThreads;
  for (int g = 0; g < G; ++g) {
    const gptr<const double> sp = to_global<double>(slots.p[g] + base);
    double x[2 * kCombinePairs];
#pragma unroll
    for (int v = 0; v < kCombinePairs; ++v) {
      const int e = (v * kThreads + li) * 2;
      if (full || e + 2 <= td.count) {
        const f64x2 d = __builtin_nontemporal_load((gptr<const f64x2>)(sp + e));
        x[2 * v] = d.x;
        x[2 * v + 1] = d.y;
      } else {
        x[2 * v] = (e < td.count) ? sp[e] : 0.0;
        x[2 * v + 1] = 0.0;
      }
    }
#pragma unroll
    for (int i = 0; i < 2 * kCombinePairs; ++i) acc[i] = (g == 0) ? x[i] : acc[i] + x[i];
  }
  double res[2 * kCombinePairs];
  exact_div_block<2 * kCombinePairs>(acc, res, to_const<double>(wtot)[td.seg]);
  bool bad_acc = false, bad_res = false;
  void* const out_raw = reinterpret_cast<void*>(to_const<uint64_t>(outs)[td.seg]);
  const gptr<O> op = to_global_mut<O>(out_raw) + td.start;
#pragma unroll
  for (int v = 0; v < kCombinePairs; ++v) {
    const int e = (v * kThreads + li) * 2;
    const bool in0 = full || e < td.count, in1 = full || e + 1 < td.count;
    bad_acc |= (in0 && acc[2 * v] != acc[2 * v]) || (in1 && acc[2 * v + 1] != acc[2 * v + 1]);
    bad_res |= (in0 && res[2 * v] != res[2 * v]) || (in1 && res[2 * v + 1] != res[2 * v + 1]);
    if (VEC && in1) {
      if constexpr (sizeof(O) == 4) {
        store_out((gptr<f32x2>)(op + e), f32x2{static_cast<float>(res[2 * v]), static_cast<float>(res[2 * v + 1])});
      } else {
        store_out((gptr<f64x2>)(op + e), f64x2{res[2 * v], res[2 * v + 1]});
      }
    } else {
      if (in0) op[e] = static_cast<O>(res[2 * v]);
      if (in1) op[e + 1] = static_cast<O>(res[2 * v + 1]);
    }
  }
  const uint64_t ba = __ballot(bad_acc), br = __ballot(bad_res);
  if ((ba | br) != 0ull && (threadIdx.x & 63) == 0) {
    if (ba) raise_flag(flag, 0);
    if (br) raise_flag(flag, 1);
  }
}

}  // namespace

// =======================================================================================
// host side
// =======================================================================================
struct fedavg_ctx {
  int device = 0;
  int T = 0;
  std::vector<int64_t> seg_numel;
  std::vector<int64_t> seg_acc_off;
  int64_t acc_numel = 0;
  double* acc = nullptr;
  bool owns_acc = false;

  // tiles for SPLIT=1 and SPLIT=4
  std::vector<TileDesc> tiles1, tiles4, tilesw;  // + kTileWide tiles (whole-layout launches)
  TileDesc* d_tiles1 = nullptr;
  TileDesc* d_tiles4 = nullptr;
  TileDesc* d_tilesw = nullptr;
  // balanced orders of the whole-layout tables (build_balanced_tiles): fp32 on kTileWide tiles,
  // fp64 on kTile1 tiles; empty = not used (FEDAVG_BALANCE)
  std::vector<TileDesc> tilesw_bal, tiles1_bal;
  int32_t tilesw_bal_head = 0, tiles1_bal_head = 0;  // their leading whole waves of full tiles
  TileDesc* d_tilesw_bal = nullptr;
  TileDesc* d_tiles1_bal = nullptr;
  SegDesc* d_segs = nullptr;
  uint32_t* h_flag = nullptr;  // host-coherent pinned NaN words (kernels store into them)
  uint32_t* d_flag = nullptr;  // device alias of h_flag

  // accumulated state (host mirror)
  std::vector<double> wsum;     // per-segment total weight (fed_avg_algorithm.py:59-62)
  std::vector<int32_t> valid;   // accumulator holds data for the segment

  // staging ring for per-call tables
  static constexpr int kSlots = 4;
  struct Slot {
    char* host = nullptr;  // pinned
    char* dev = nullptr;
    size_t cap = 0;
    hipEvent_t done = nullptr;
    bool used = false;
  } slots[kSlots];
  int next_slot = 0;
  int last_slot = -1;             // slot holding last_blob on the device
  std::vector<char> last_blob;    // host image of the last uploaded table blob
  std::vector<char> scratch;

  int split_policy = 1;  // 1 exact client order (default), 0 auto, 2 always split
  bool allow_fma = true;  // fused fold when every product is provably exact
  // whole-layout launches use the wide tile table only when they fold at least this many clients
  // per segment (short waves keep the 4096-element tiles: two workgroups per CU instead of one)
  int wide_min_clients = 0;
  // Streaming waves alternate the direction they walk the whole layout: a wave that reads the
  // accumulator starts with the tiles the previous wave wrote last, which are still in L2 / the
  // memory-side cache. Any tile order folds every element identically (FEDAVG_WALK_ALTERNATE).
  bool walk_alternate = FEDAVG_WALK_ALTERNATE != 0;
  bool walk_reverse = false;
  // profiling
  bool prof = false;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> prof_events;
  std::vector<hipEvent_t> event_pool;
  // auxiliary per-call tables (per-element weights, NaN scans): one pinned + device buffer pair
  char* aux_host = nullptr;
  char* aux_dev = nullptr;
  size_t aux_cap = 0;
  // QSGD |product| tables of the current call ([T][K][256] fp64, qsgd_table_kernel)
  double* qtab = nullptr;
  size_t qtab_cap = 0;  // doubles
  size_t qtab_cap_bytes = size_t(64) << 20;  // FEDAVG_QSGD_TABLE_CAP: table block per launch
  size_t qtab_last_bytes = 0;                // table bytes of the last QSGD launch
  hipEvent_t aux_done = nullptr;  // the last upload out of aux_host finished
  bool aux_used = false;
  // the dynamic wave (fedavg_dyn_*): its host-coherent control block and row table, the device
  // mirror words, a private stream (the caller's stream stays free for the work producing the
  // arrivals) and the per-segment totals of the published rows
  struct Dyn {
    bool active = false;
    int32_t in_dtype = -1;
    int32_t published = 0;
    int32_t cap = 0;
    char* host = nullptr;      // DynCtl, DynAck, wtot[T], outs[T], wtab[cap], ptab[T][cap]
    char* dev_alias = nullptr;
    size_t bytes = 0;
    char* mirror = nullptr;    // kDynCopies DynMirror (device)
    char* dtab = nullptr;      // the device copy of the tables (DynLayout offsets, device memory)
    std::vector<TileDesc> tiles;       // body tiles: the whole kDynTile-element tiles of each segment
    std::vector<TileDesc> edge_tiles;  // edge tiles: the rest, in <= kDynEdgeTile-element tiles
    TileDesc* d_tiles = nullptr;
    TileDesc* d_edge_tiles = nullptr;
    hipStream_t edge_stream = nullptr;  // the edge launch runs beside the body launch
    hipEvent_t edge_done = nullptr;
    bool unjoined = false;  // a finalized wave closed with join = 0: fedavg_check waits for it
    hipEvent_t prof_start = nullptr;  // profiling: the open of the wave being timed
    std::vector<std::pair<hipEvent_t, hipEvent_t>> prof;  // (open, end of the body launch) per wave
    uint32_t epoch = 0;        // waves opened on this context (tags the mirror word)
    hipStream_t stream = nullptr;
    hipEvent_t start = nullptr, done = nullptr;
    std::vector<double> wsum;  // per segment, the published rows' weights in arrival order
    // a wave that ended itself is continued by a fresh launch (dyn_continue): rows [0, base) of the
    // caller's table are in the accumulator, wsum_base their per-segment totals in arrival order
    int32_t base = 0;
    std::vector<double> wsum_base;
    int32_t reopens = 0;   // continued waves, cumulative (fedavg_dyn_info)
    int32_t launches = 0;  // wave launches, cumulative
    uint64_t* tend = nullptr;  // profiling: each tile's finishing time (dyn_tile_done)
    bool timed = false;        // the last launch recorded them
    uint64_t idle_ticks = 0, life_ticks = 0;
  } dyn;
};

namespace {

constexpr size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

struct DynLayout {  // offsets into the host-coherent block
  size_t ctl, ack, wtot, outs, wtab, ptab, bytes;
  DynLayout(int T, int cap) {
    ctl = 0;
    ack = align_up(ctl + sizeof(DynCtl), 64);
    wtot = align_up(ack + sizeof(DynAck), 64);
    outs = align_up(wtot + sizeof(double) * T, 64);
    wtab = align_up(outs + sizeof(uint64_t) * T, 64);
    ptab = align_up(wtab + sizeof(double) * cap, 64);
    bytes = align_up(ptab + sizeof(uint64_t) * static_cast<size_t>(T) * cap, 4096);
  }
};


int32_t elem_size(int32_t dt) {
  switch (dt) {
    case FEDAVG_F32: return 4;
    case FEDAVG_F16: return 2;
    case FEDAVG_BF16: return 2;
    case FEDAVG_F64: return 8;
    case FEDAVG_QSGD_F32: return 1;  // quantised records (slots / codes are bytes)
    case FEDAVG_QSGD_F64: return 1;
    case FEDAVG_NNADQ_F32: return 1;
    case FEDAVG_NNADQ_F64: return 1;
    default: return 0;
  }
}

// A whole-layout launch runs one workgroup per tile and `slots` workgroups at a time (resident
// workgroups per CU x CUs). With every tile the same length the launch ends with a partial wave
// (64 x ResNet-18 fp32: 1427 tiles of 8192 = 5.57 waves of 256 — the last 0.57 wave leaves 43 % of
// the CUs idle; a flat layout of 5.00 / 5.08 waves runs at 6.8 / 6.2 TB/s, scripts/tail_probe.py).
// The balanced order keeps whole waves of full tiles first, then cuts the remaining full tiles into
// pieces of whole lane-vectors (`gran` elements, the PARTV fast path) sized so the remaining work
// spreads over all slots, and ends with those pieces and the segments' tail pieces sorted longest
// first (list scheduling then finishes the slots within about one piece of each other). Any
// partition of the elements folds every element identically, so the bits do not change.
// Returns the number of leading full tiles (whole waves).
int32_t build_balanced_tiles(const std::vector<int64_t>& numel, int tile, int gran, int64_t slots,
                             std::vector<TileDesc>& out) {
  std::vector<TileDesc> full, tail;
  int64_t tail_elems = 0;
  for (size_t t = 0; t < numel.size(); ++t) {
    const int64_t q = numel[t] / tile;
    for (int64_t i = 0; i < q; ++i) full.push_back(TileDesc{static_cast<int32_t>(t), tile, i * tile});
    int64_t start = q * tile, r = numel[t] - q * tile;
    const int64_t rv = r - r % gran;  // whole lane-vectors: fast path
    if (rv > 0) {
      tail.push_back(TileDesc{static_cast<int32_t>(t), static_cast<int32_t>(rv), start});
      start += rv;
      r -= rv;
      tail_elems += rv;
    }
    if (r > 0) {
      tail.push_back(TileDesc{static_cast<int32_t>(t), static_cast<int32_t>(r), start});
      tail_elems += r;
    }
  }
  slots = std::max<int64_t>(slots, 1);
  const int64_t head = (static_cast<int64_t>(full.size()) / slots) * slots;
  const int64_t rest = static_cast<int64_t>(full.size()) - head;
  const int64_t remaining = rest * tile + tail_elems;
  int64_t piece = (remaining + slots - 1) / slots;
  piece = std::min<int64_t>(tile, std::max<int64_t>(gran, (piece + gran - 1) / gran * gran));
  out.assign(full.begin(), full.begin() + head);
  std::vector<TileDesc> end;
  for (int64_t i = head; i < static_cast<int64_t>(full.size()); ++i) {
    for (int64_t s = 0; s < tile; s += piece) {
      const int64_t c = std::min<int64_t>(piece, tile - s);
      end.push_back(TileDesc{full[i].seg, static_cast<int32_t>(c), full[i].start + s});
    }
  }
  end.insert(end.end(), tail.begin(), tail.end());
  std::stable_sort(end.begin(), end.end(), [](const TileDesc& a, const TileDesc& b) { return a.count > b.count; });
  out.insert(out.end(), end.begin(), end.end());
  return static_cast<int32_t>(head);
}

void build_tiles(const std::vector<int64_t>& numel, int tile, std::vector<TileDesc>& out) {
  out.clear();
  for (size_t t = 0; t < numel.size(); ++t) {
    for (int64_t s = 0; s < numel[t]; s += tile) {
      TileDesc d;
      d.seg = static_cast<int32_t>(t);
      d.count = static_cast<int32_t>(std::min<int64_t>(tile, numel[t] - s));
      d.start = s;
      out.push_back(d);
    }
  }
}

// hipStreamQuery, asked twice: right after a synchronize, the first query of a stream that waited
// on another stream's event (a dynamic wave's close) can still report the finished wait as
// pending (ROCm 7.2, traced: each reset then enqueued a memset and the next open a dependency)
bool stream_idle(hipStream_t s) { return hipStreamQuery(s) == hipSuccess || hipStreamQuery(s) == hipSuccess; }

hipEvent_t take_event(fedavg_ctx* c) {
  if (!c->event_pool.empty()) {
    hipEvent_t e = c->event_pool.back();
    c->event_pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  if (hipEventCreate(&e) != hipSuccess) return nullptr;
  return e;
}

// Staged per-call tables, laid out in one blob.
struct Staged {
  CallTables tab;
  int32_t Kmax = 0;
  int32_t stride = 1;    // row stride of the [T][K] tables
  bool aligned = true;
  bool clients_aligned = true;  // every client pointer is 16-byte aligned
  bool delta = false;           // clients are deltas against tab.base (fp64)
  int32_t max_weight_bits = 0;  // largest significand (bits) among the call's weights
  bool weights_tame = true;     // every weight finite, zero or within [2^-800, 2^800]
  double last_weight = std::numeric_limits<double>::quiet_NaN();  // note_weight's repeat cache
  std::vector<int32_t> kseg;
};

}  // namespace

struct fedavg_plan {
  enum Kind { AGGREGATE = 0, PARTIAL = 1, FINALIZE = 2 };
  fedavg_ctx* ctx = nullptr;
  int device = -1;  // the context's device (destroy must not read a context freed before it)
  Staged st;
  std::vector<char> fin_img;  // totals + outputs last copied into the blob (own-window combine)
  char* dev = nullptr;
  int32_t in_dtype = 0;
  int out_kind = 0;
  int split = 1;
  int kind = AGGREGATE;
  int32_t zero_init = 0;
};

namespace {

// Significand width of a weight (bits between its leading and trailing one).
void note_weight(Staged& st, double w) {
  // called for every (client, tensor) entry of a call (thousands per wave): a client's weight
  // usually repeats across its tensors, and the significand width comes from the bits directly
  // (frexp / ldexp library calls cost ~20 ns per entry)
  if (w == st.last_weight) return;
  st.last_weight = w;
  if (w == 0.0) return;
  uint64_t b;
  std::memcpy(&b, &w, sizeof(b));
  const int be = static_cast<int>((b >> 52) & 0x7ff);
  if (be == 0x7ff) {  // inf / NaN
    st.weights_tame = false;
    return;
  }
  // |w| = m * 2^e with m in [0.5, 1) (frexp's convention): e = be - 1022 for normal w; a
  // subnormal is far below 2^-800 anyway
  const int e = be - 1022;
  if (be == 0 || e < -800 || e > 800) st.weights_tame = false;
  const uint64_t sig = (b & ((uint64_t(1) << 52) - 1)) | (be ? (uint64_t(1) << 52) : 0);
  const int q = sig ? 53 - __builtin_ctzll(sig) : 0;
  st.max_weight_bits = std::max(st.max_weight_bits, q);
}

int32_t significand_bits(int32_t dt) {
  switch (dt) {
    case FEDAVG_F32: return 24;
    case FEDAVG_F16: return 11;
    case FEDAVG_BF16: return 8;
    case FEDAVG_NNADQ_F32: return 24;  // dequantised values are fp32
    default: return 53;
  }
}

// Every product x * w of the call is exact in fp64 (input significand + weight significand
// <= 53 bits, no over/underflow), so fma(x, w, acc) rounds exactly like acc + round(x * w).
bool fma_exact_call(const Staged& st, int32_t in_dtype) {
  return st.weights_tame && significand_bits(in_dtype) + st.max_weight_bits <= 53;
}

// Build segment-major compacted tables in a pinned slot and enqueue their H2D copy.
// Offsets of the per-call table blob (one allocation, 16-B aligned sections).
struct BlobLayout {
  size_t off_ptr, off_w, off_kseg, off_accin, off_outs, off_wtot, off_base, bytes;
  BlobLayout(int T, int Kr) {
    off_ptr = 0;
    off_w = align_up(off_ptr + sizeof(void*) * T * Kr, 16);
    off_kseg = align_up(off_w + sizeof(double) * T * Kr, 16);
    off_accin = align_up(off_kseg + sizeof(int32_t) * T, 16);
    off_outs = align_up(off_accin + sizeof(int32_t) * T, 16);
    off_wtot = align_up(off_outs + sizeof(void*) * T, 16);
    off_base = align_up(off_wtot + sizeof(double) * T, 16);
    bytes = align_up(off_base + sizeof(void*) * T, 256);
  }
  void point(char* d, CallTables& tab) const {
    tab.cptrs = reinterpret_cast<const void* const*>(d + off_ptr);
    tab.w = reinterpret_cast<const double*>(d + off_w);
    tab.kseg = reinterpret_cast<const int32_t*>(d + off_kseg);
    tab.acc_in = reinterpret_cast<const int32_t*>(d + off_accin);
    tab.outs = reinterpret_cast<void* const*>(d + off_outs);
    tab.wtot = reinterpret_cast<const double*>(d + off_wtot);
    tab.base = reinterpret_cast<const void* const*>(d + off_base);
  }
};

// Host image of the tables: segment-major compaction of the [K][T] client table.
void build_blob(const fedavg_ctx* c, const void* const* client_ptrs, const double* weights, int32_t K,
                void* const* out_ptrs, const double* wtot, const int32_t* acc_in, Staged& st,
                std::vector<char>& blob, const BlobLayout& L, const void* const* base_ptrs = nullptr) {
  const int T = c->T;
  const int Kr = std::max(K, 1);
  blob.assign(L.bytes, 0);
  char* h = blob.data();
  const void** hp = reinterpret_cast<const void**>(h + L.off_ptr);
  double* hw = reinterpret_cast<double*>(h + L.off_w);
  int32_t* hk = reinterpret_cast<int32_t*>(h + L.off_kseg);
  int32_t* ha = reinterpret_cast<int32_t*>(h + L.off_accin);
  void** ho = reinterpret_cast<void**>(h + L.off_outs);
  double* hwt = reinterpret_cast<double*>(h + L.off_wtot);
  const void** hb = reinterpret_cast<const void**>(h + L.off_base);
  st.delta = base_ptrs != nullptr;
  st.kseg.assign(T, 0);
  st.stride = Kr;
  st.aligned = true;
  st.clients_aligned = true;
  st.Kmax = 0;
  for (int t = 0; t < T; ++t) {
    int n = 0;
    for (int k = 0; k < K; ++k) {
      const void* p = client_ptrs[static_cast<int64_t>(k) * T + t];
      if (p == nullptr) continue;
      if (reinterpret_cast<uintptr_t>(p) % 16 != 0) st.aligned = st.clients_aligned = false;
      hp[static_cast<int64_t>(t) * Kr + n] = p;
      const double wv = weights[static_cast<int64_t>(k) * T + t];
      hw[static_cast<int64_t>(t) * Kr + n] = wv;
      note_weight(st, wv);
      ++n;
    }
    hk[t] = n;
    st.kseg[t] = n;
    st.Kmax = std::max(st.Kmax, n);
    ha[t] = acc_in ? acc_in[t] : 0;
    ho[t] = out_ptrs ? out_ptrs[t] : nullptr;
    if (out_ptrs && reinterpret_cast<uintptr_t>(out_ptrs[t]) % 16 != 0) st.aligned = false;
    hwt[t] = wtot ? wtot[t] : 1.0;
    hb[t] = base_ptrs ? base_ptrs[t] : nullptr;
    if (base_ptrs && reinterpret_cast<uintptr_t>(base_ptrs[t]) % 16 != 0) st.aligned = false;
  }
}

int32_t stage_tables(fedavg_ctx* c, hipStream_t s, const void* const* client_ptrs,
                     const double* weights, int32_t K, void* const* out_ptrs,
                     const double* wtot, const int32_t* acc_in, Staged& st,
                     const void* const* base_ptrs = nullptr) {
  const BlobLayout L(c->T, std::max(K, 1));
  const size_t bytes = L.bytes;
  // Build the blob in host scratch first: when it is byte-identical to the previous call's
  // (same clients, weights, outputs — e.g. persistent client slots round after round), the
  // device copy already holds it and no upload is issued.
  std::vector<char>& blob = c->scratch;
  build_blob(c, client_ptrs, weights, K, out_ptrs, wtot, acc_in, st, blob, L, base_ptrs);

  char* d = nullptr;
  if (c->last_slot >= 0 && c->last_blob.size() == bytes &&
      std::memcmp(c->last_blob.data(), blob.data(), bytes) == 0) {
    d = c->slots[c->last_slot].dev;  // unchanged since it was uploaded on this stream
  } else {
    const int slot = c->next_slot;
    fedavg_ctx::Slot& sl = c->slots[slot];
    c->next_slot = (c->next_slot + 1) % fedavg_ctx::kSlots;
    if (sl.used) FEDAVG_HIP_TRY(hipEventSynchronize(sl.done));  // its previous copy finished
    if (sl.cap < bytes) {
      if (sl.host) FEDAVG_HIP_TRY(hipHostFree(sl.host));
      if (sl.dev) {
        FEDAVG_HIP_TRY(hipStreamSynchronize(s));  // a kernel may still read the old table
        FEDAVG_HIP_TRY(hipFree(sl.dev));
      }
      const size_t cap = std::max<size_t>(bytes * 2, 64 * 1024);
      FEDAVG_HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&sl.host), cap, hipHostMallocDefault));
      FEDAVG_HIP_TRY(hipMalloc(reinterpret_cast<void**>(&sl.dev), cap));
      sl.cap = cap;
      if (!sl.done) FEDAVG_HIP_TRY(hipEventCreateWithFlags(&sl.done, hipEventDisableTiming));
    }
    std::memcpy(sl.host, blob.data(), bytes);
    FEDAVG_HIP_TRY(hipMemcpyAsync(sl.dev, sl.host, bytes, hipMemcpyHostToDevice, s));
    FEDAVG_HIP_TRY(hipEventRecord(sl.done, s));
    sl.used = true;
    c->last_blob.swap(blob);
    c->last_slot = slot;
    d = sl.dev;
  }
  L.point(d, st.tab);
  return FEDAVG_OK;
}

// Upload a small per-call table blob through the context's auxiliary pinned buffer (the device
// copy is ordered before the kernels that read it on the same stream).
int32_t aux_upload(fedavg_ctx* c, hipStream_t s, const std::vector<char>& blob, char** dev) {
  if (c->aux_used) FEDAVG_HIP_TRY(hipEventSynchronize(c->aux_done));
  if (c->aux_cap < blob.size()) {
    FEDAVG_HIP_TRY(hipStreamSynchronize(s));  // a kernel may still read the old device table
    if (c->aux_host) FEDAVG_HIP_TRY(hipHostFree(c->aux_host));
    if (c->aux_dev) FEDAVG_HIP_TRY(hipFree(c->aux_dev));
    c->aux_host = nullptr;
    c->aux_dev = nullptr;
    c->aux_cap = 0;
    const size_t cap = std::max<size_t>(blob.size() * 2, 64 * 1024);
    FEDAVG_HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&c->aux_host), cap, hipHostMallocDefault));
    FEDAVG_HIP_TRY(hipMalloc(reinterpret_cast<void**>(&c->aux_dev), cap));
    c->aux_cap = cap;
    if (!c->aux_done) FEDAVG_HIP_TRY(hipEventCreateWithFlags(&c->aux_done, hipEventDisableTiming));
  }
  std::memcpy(c->aux_host, blob.data(), blob.size());
  FEDAVG_HIP_TRY(hipMemcpyAsync(c->aux_dev, c->aux_host, blob.size(), hipMemcpyHostToDevice, s));
  FEDAVG_HIP_TRY(hipEventRecord(c->aux_done, s));
  c->aux_used = true;
  *dev = c->aux_dev;
  return FEDAVG_OK;
}

// Launches go through hipExtLaunchKernelGGL: an optional stop event is attached to the kernel's
// own dispatch (its completion signal) instead of a separate marker packet — a marker between
// two kernels costs ~6-16 µs of queue latency (DESIGN.md §5 traces); the sharded round's
// per-chunk events use this.
template <typename T, int OUT, int SPLIT, bool VEC, int TILEN = kTile1, bool PV = false>
hipError_t launch_fold_pv(const KArgs& a, int fold, int nblocks, hipStream_t s, hipEvent_t e0, hipEvent_t e1) {
  const int threads = Geo<T, SPLIT, TILEN>::THREADS;
  if (fold == FOLD_FMA) {
    hipExtLaunchKernelGGL((fedavg_tile_kernel<T, OUT, SPLIT, VEC, FOLD_FMA, TILEN, PV>), dim3(nblocks), dim3(threads),
                          0, s, e0, e1, 0, a);
  } else if (fold == FOLD_DELTA) {
    if constexpr (SPLIT == 1) {
      hipExtLaunchKernelGGL((fedavg_tile_kernel<T, OUT, SPLIT, VEC, FOLD_DELTA, TILEN, PV>), dim3(nblocks),
                            dim3(threads), 0, s, e0, e1, 0, a);
    } else {
      return hipErrorInvalidValue;  // delta calls run the exact-order kernel only
    }
  } else {
    hipExtLaunchKernelGGL((fedavg_tile_kernel<T, OUT, SPLIT, VEC, FOLD_MULADD, TILEN, PV>), dim3(nblocks),
                          dim3(threads), 0, s, e0, e1, 0, a);
  }
  return hipGetLastError();
}

// partv: the tile table is a balanced order (pieces of whole lane-vectors: the PV instantiation)
template <typename T, int OUT, int SPLIT, bool VEC, int TILEN = kTile1>
hipError_t launch_fold(const KArgs& a, int fold, int nblocks, hipStream_t s, hipEvent_t e0, hipEvent_t e1,
                       bool partv = false) {
  if constexpr (SPLIT == 1 && VEC) {
    if (partv) return launch_fold_pv<T, OUT, SPLIT, VEC, TILEN, true>(a, fold, nblocks, s, e0, e1);
  }
  return launch_fold_pv<T, OUT, SPLIT, VEC, TILEN, false>(a, fold, nblocks, s, e0, e1);
}

// wide = a whole-layout exact-order launch over the kTileWide table (2- / 4-byte inputs only)
template <typename T, int OUT>
hipError_t launch_typed(const KArgs& a, int split, bool vec, int fold, int nblocks, hipStream_t s, hipEvent_t e0,
                        hipEvent_t e1, bool wide, bool partv) {
  if (split == 4) {
    return vec ? launch_fold<T, OUT, 4, true>(a, fold, nblocks, s, e0, e1)
               : launch_fold<T, OUT, 4, false>(a, fold, nblocks, s, e0, e1);
  }
  if constexpr (sizeof(T) < 8 && kTileWide > 0) {
    if (wide) {
      return vec ? launch_fold<T, OUT, 1, true, kTileWide>(a, fold, nblocks, s, e0, e1, partv)
                 : launch_fold<T, OUT, 1, false, kTileWide>(a, fold, nblocks, s, e0, e1);
    }
  }
  if (wide) return hipErrorInvalidValue;
  return vec ? launch_fold<T, OUT, 1, true>(a, fold, nblocks, s, e0, e1, partv)
             : launch_fold<T, OUT, 1, false>(a, fold, nblocks, s, e0, e1);
}

template <int OUT>
hipError_t launch_out(int32_t in_dtype, const KArgs& a, int split, bool vec, int fold, int nblocks, hipStream_t s,
                      hipEvent_t e0, hipEvent_t e1, bool wide, bool partv = false) {
  switch (in_dtype) {
    case FEDAVG_F32: return launch_typed<float, OUT>(a, split, vec, fold, nblocks, s, e0, e1, wide, partv);
    case FEDAVG_F16: return launch_typed<__half, OUT>(a, split, vec, fold, nblocks, s, e0, e1, wide, partv);
    case FEDAVG_BF16: return launch_typed<bf16_t, OUT>(a, split, vec, fold, nblocks, s, e0, e1, wide, partv);
    case FEDAVG_F64: return launch_typed<double, OUT>(a, split, vec, fold, nblocks, s, e0, e1, wide, partv);
    default: return hipErrorInvalidValue;
  }
}

// Own-window combine launches of the multi-device peer exchange (KArgs::comb_*): exact order,
// one tile per workgroup, scalar-weight folds only (no delta calls).
template <typename T, int OUT>
hipError_t launch_comb_typed(const KArgs& a, bool vec, int fold, hipStream_t s, hipEvent_t e1) {
  if constexpr (OUT == OUT_ACC) {
    return hipErrorInvalidValue;
  } else {
    const dim3 grid(static_cast<unsigned>(a.num_tiles)), block(Geo<T, 1, kTile1>::THREADS);
    if (fold == FOLD_FMA) {
      if (vec) hipExtLaunchKernelGGL((fedavg_tile_kernel<T, OUT, 1, true, FOLD_FMA, kTile1, false, true>), grid, block, 0, s, nullptr, e1, 0, a);
      else hipExtLaunchKernelGGL((fedavg_tile_kernel<T, OUT, 1, false, FOLD_FMA, kTile1, false, true>), grid, block, 0, s, nullptr, e1, 0, a);
    } else if (fold == FOLD_MULADD) {
      if (vec) hipExtLaunchKernelGGL((fedavg_tile_kernel<T, OUT, 1, true, FOLD_MULADD, kTile1, false, true>), grid, block, 0, s, nullptr, e1, 0, a);
      else hipExtLaunchKernelGGL((fedavg_tile_kernel<T, OUT, 1, false, FOLD_MULADD, kTile1, false, true>), grid, block, 0, s, nullptr, e1, 0, a);
    } else {
      return hipErrorInvalidValue;
    }
    return hipGetLastError();
  }
}

template <int OUT>
hipError_t launch_comb_out(int32_t in_dtype, const KArgs& a, bool vec, int fold, hipStream_t s, hipEvent_t e1) {
  switch (in_dtype) {
    case FEDAVG_F32: return launch_comb_typed<float, OUT>(a, vec, fold, s, e1);
    case FEDAVG_F16: return launch_comb_typed<__half, OUT>(a, vec, fold, s, e1);
    case FEDAVG_BF16: return launch_comb_typed<bf16_t, OUT>(a, vec, fold, s, e1);
    case FEDAVG_F64: return launch_comb_typed<double, OUT>(a, vec, fold, s, e1);
    default: return hipErrorInvalidValue;
  }
}

bool is_qsgd(int32_t dt) { return dt == FEDAVG_QSGD_F32 || dt == FEDAVG_QSGD_F64; }
bool is_nnadq(int32_t dt) { return dt == FEDAVG_NNADQ_F32 || dt == FEDAVG_NNADQ_F64; }
bool is_record(int32_t dt) { return is_qsgd(dt) || is_nnadq(dt); }

template <int OUT, typename DQ, int FOLD>
hipError_t launch_nnadq_fold(const KArgs& a, bool vec, hipStream_t s, hipEvent_t e1) {
  const dim3 grid(static_cast<unsigned>(a.num_tiles)), block(kNnadqLanes);
  if (vec) hipExtLaunchKernelGGL((nnadq_tile_kernel<OUT, DQ, FOLD, true>), grid, block, 0, s, nullptr, e1, 0, a);
  else hipExtLaunchKernelGGL((nnadq_tile_kernel<OUT, DQ, FOLD, false>), grid, block, 0, s, nullptr, e1, 0, a);
  return hipGetLastError();
}

template <int OUT>
hipError_t launch_nnadq_out(int32_t in_dtype, const KArgs& a, bool vec, bool fma, hipStream_t s, hipEvent_t e1) {
  if (in_dtype == FEDAVG_NNADQ_F32)
    return fma ? launch_nnadq_fold<OUT, float, FOLD_FMA>(a, vec, s, e1) : launch_nnadq_fold<OUT, float, FOLD_MULADD>(a, vec, s, e1);
  return fma ? launch_nnadq_fold<OUT, double, FOLD_FMA>(a, vec, s, e1) : launch_nnadq_fold<OUT, double, FOLD_MULADD>(a, vec, s, e1);
}

template <int OUT>
hipError_t launch_qsgd_out(int32_t in_dtype, const KArgs& a, bool vec, hipStream_t s, hipEvent_t e1, int32_t seg_begin,
                           int32_t seg_count) {
  // the call's |product| tables first (same stream: the tile kernel reads them by DMA)
  const dim3 tgrid(static_cast<unsigned>(a.K), static_cast<unsigned>(seg_count));
  if (in_dtype == FEDAVG_QSGD_F32)
    hipLaunchKernelGGL(qsgd_table_kernel<float>, tgrid, dim3(kQsgdSlots), 0, s, a.tab, a.K, seg_begin,
                       const_cast<double*>(a.qtab));
  else
    hipLaunchKernelGGL(qsgd_table_kernel<double>, tgrid, dim3(kQsgdSlots), 0, s, a.tab, a.K, seg_begin,
                       const_cast<double*>(a.qtab));
  const dim3 grid(static_cast<unsigned>(a.num_tiles)), block(kQsgdLanes);
  if (in_dtype == FEDAVG_QSGD_F32) {
    if (vec) hipExtLaunchKernelGGL((qsgd_tile_kernel<OUT, float, true>), grid, block, 0, s, nullptr, e1, 0, a);
    else hipExtLaunchKernelGGL((qsgd_tile_kernel<OUT, float, false>), grid, block, 0, s, nullptr, e1, 0, a);
  } else {
    if (vec) hipExtLaunchKernelGGL((qsgd_tile_kernel<OUT, double, true>), grid, block, 0, s, nullptr, e1, 0, a);
    else hipExtLaunchKernelGGL((qsgd_tile_kernel<OUT, double, false>), grid, block, 0, s, nullptr, e1, 0, a);
  }
  return hipGetLastError();
}

int choose_split(const fedavg_ctx* c, int kmax) {
  if (c->split_policy == 1) return 1;
  if (c->split_policy == 2) return kmax >= 4 ? 4 : 1;
  // auto: the exact-order kernel unless the tile grid cannot fill 256 CUs and there are
  // enough clients per tile to keep four waves busy
  if (static_cast<int64_t>(c->tiles1.size()) < 512 && kmax >= 16) return 4;
  return 1;
}

// Launch the main kernel over tiles [tb, te) of the split-specific tile table.
// done_ev (optional, in/out): an event the caller wants completed with this kernel. When
// profiling is on, the profiling stop event is handed back in its place.
int32_t launch_main(fedavg_ctx* c, hipStream_t s, const Staged& st, int32_t in_dtype, int out_kind,
                    int split, int32_t zero_init, int32_t tb_split1, int32_t te_split1,
                    hipEvent_t* done_ev = nullptr, double* acc_out = nullptr,
                    const KArgs* win = nullptr, const KArgs* comb = nullptr) {
  if (c->dyn.active)
    return fail(FEDAVG_ERR_STATE, "a dynamic wave is open on this context (fedavg_dyn_close it first)");
  if (st.delta) split = 1;  // delta folds run the exact-order kernel only
  if (comb) split = 1;
  KArgs a;
  // comb (dense final folds only): the multi-device own-window combine (KArgs::comb_*)
  a.comb_src = comb ? comb->comb_src : nullptr;
  a.comb_n = comb ? comb->comb_n : 0;
  a.comb_self = comb ? comb->comb_self : 0;
  a.segs = c->d_segs;
  a.tab = st.tab;
  // win (dense zero-initialised partials only): the multi-device window table (KArgs::win_dst)
  a.win_dst = win ? win->win_dst : nullptr;
  a.win_edge = win ? win->win_edge : nullptr;
  a.win_n = win ? win->win_n : 0;
  // acc_out: a zero-initialised partial written elsewhere in accumulator coordinates (the
  // multi-device exchange: another device's receive slot, through the peer mapping)
  a.acc = acc_out ? acc_out : c->acc;
  a.flag = c->d_flag;
  a.K = st.stride;
  a.zero_init = zero_init;
  a.walk_back = 0;
  a.qtab = nullptr;
  a.qtab_seg0 = 0;
  int tb = 0, te = 0;
  if (split == 4) {
    // whole-layout launches only (tile ranges are defined on the SPLIT=1 table)
    a.tiles = c->d_tiles4;
    tb = 0;
    te = static_cast<int>(c->tiles4.size());
  } else {
    a.tiles = c->d_tiles1;
    tb = tb_split1;
    te = te_split1;
  }
  // whole-layout exact-order launch of a 2- / 4-byte input: the wide table (same elements)
  // (a windowed launch indexes the exact-order table: no wide / balanced / reversed orders)
  const bool wide = !win && !comb && split == 1 && c->d_tilesw != nullptr && tb_split1 == 0 &&
                    st.Kmax >= c->wide_min_clients &&
                    te_split1 == static_cast<int32_t>(c->tiles1.size()) &&
                    (in_dtype == FEDAVG_F32 || in_dtype == FEDAVG_F16 || in_dtype == FEDAVG_BF16 ||
                     false);
  if (wide) {
    a.tiles = c->d_tilesw;
    tb = 0;
    te = static_cast<int>(c->tilesw.size());
    if (in_dtype == FEDAVG_F32 && c->d_tilesw_bal != nullptr) {
      a.tiles = c->d_tilesw_bal;
      te = static_cast<int>(c->tilesw_bal.size());
    }
  } else if (!win && !comb && split == 1 && in_dtype == FEDAVG_F64 && c->d_tiles1_bal != nullptr &&
             tb_split1 == 0 && te_split1 == static_cast<int32_t>(c->tiles1.size())) {
    a.tiles = c->d_tiles1_bal;  // a whole-layout fp64 launch: the balanced order of the same tiles
    tb = 0;
    te = static_cast<int>(c->tiles1_bal.size());
  }
  a.tile_begin = tb;
  a.num_tiles = te - tb;
  if (a.num_tiles <= 0) return FEDAVG_OK;
  // whole-layout waves alternate their walk (a balanced order reverses only its leading whole
  // waves: its short pieces stay at the end, where they balance the tail; ranged launches keep
  // their order)
  if (!win && !comb && c->walk_alternate && split == 1 && !is_record(in_dtype) &&
      tb_split1 == 0 && te_split1 == static_cast<int32_t>(c->tiles1.size())) {
    if (c->walk_reverse)
      a.walk_back = (a.tiles == c->d_tilesw_bal)   ? c->tilesw_bal_head
                    : (a.tiles == c->d_tiles1_bal) ? c->tiles1_bal_head
                                                   : a.num_tiles;
    if (out_kind == OUT_ACC) c->walk_reverse = !c->walk_reverse;
  }
  const int nblocks = a.num_tiles;
  // Profiling events are recorded as markers around the launch (the cheapest form measured:
  // attaching start/stop events to the dispatch cost the fused step ~6 µs more); without
  // profiling, a requested done event is attached to the dispatch itself (no marker).
  hipEvent_t e1 = done_ev ? *done_ev : nullptr;
  hipEvent_t m0 = nullptr, m1 = nullptr;
  if (c->prof) {
    m0 = take_event(c);
    m1 = take_event(c);
    if (!m0 || !m1) return fail(FEDAVG_ERR_HIP, "hipEventCreate failed");
    FEDAVG_HIP_TRY(hipEventRecord(m0, s));
    c->prof_events.emplace_back(m0, m1);
    e1 = nullptr;
  }
  hipError_t err = hipSuccess;
  if (is_record(in_dtype) && (win || comb)) return fail(FEDAVG_ERR_INVALID, "windowed launches take dense inputs");
  if (is_record(in_dtype)) {
    // quantised records: one tile per workgroup, exact client order (no split); the record layout needs 16-B aligned records; outputs may be unaligned
    if (st.delta) return fail(FEDAVG_ERR_INVALID, "quantised records cannot be delta updates");
    if (!st.clients_aligned) return fail(FEDAVG_ERR_INVALID, "quantised records must be 16-byte aligned");
    a.tiles = c->d_tiles1;
    a.tile_begin = tb_split1;
    a.num_tiles = te_split1 - tb_split1;
    if (a.num_tiles <= 0) return FEDAVG_OK;
  }
  if (is_nnadq(in_dtype)) {
    const bool fma = c->allow_fma && fma_exact_call(st, in_dtype);
    switch (out_kind) {
      case OUT_ACC: err = launch_nnadq_out<OUT_ACC>(in_dtype, a, st.aligned, fma, s, e1); break;
      case OUT_F32: err = launch_nnadq_out<OUT_F32>(in_dtype, a, st.aligned, fma, s, e1); break;
      case OUT_F64: err = launch_nnadq_out<OUT_F64>(in_dtype, a, st.aligned, fma, s, e1); break;
      default: return fail(FEDAVG_ERR_INVALID, "bad out kind");
    }
    if (err != hipSuccess) return fail(FEDAVG_ERR_HIP, std::string("kernel launch: ") + hipGetErrorString(err));
    if (m1) {
      FEDAVG_HIP_TRY(hipEventRecord(m1, s));
      if (done_ev) *done_ev = m1;
    }
    return FEDAVG_OK;
  }
  if (is_qsgd(in_dtype)) {
    // tables for the segments the launch's tiles touch ([segments][K][256] fp64, 2 KiB per
    // (segment, client)); a launch whose tables would pass the cap (FEDAVG_QSGD_TABLE_CAP bytes,
    // default 64 MiB: hundreds of clients over hundreds of tensors) runs as several launches over
    // segment runs, each building its own tables into the same buffer
    const size_t per_seg = static_cast<size_t>(a.K) * kQsgdTable;  // doubles
    const size_t seg_first = static_cast<size_t>(c->tiles1[tb_split1].seg);
    const size_t seg_span = static_cast<size_t>(c->tiles1[te_split1 - 1].seg) - seg_first + 1;
    const size_t cap_segs = std::max<size_t>(1, c->qtab_cap_bytes / (per_seg * sizeof(double)));
    const size_t need = std::min(seg_span, cap_segs) * per_seg;
    if (c->qtab_cap < need) {
      FEDAVG_HIP_TRY(hipStreamSynchronize(s));  // an earlier launch may still read the old tables
      if (c->qtab) FEDAVG_HIP_TRY(hipFree(c->qtab));
      c->qtab = nullptr;
      c->qtab_cap = 0;
      FEDAVG_HIP_TRY(hipMalloc(reinterpret_cast<void**>(&c->qtab), need * sizeof(double)));
      c->qtab_cap = need;
    }
    a.qtab = c->qtab;
    c->qtab_last_bytes = need * sizeof(double);
    for (int32_t t0 = tb_split1; t0 < te_split1;) {
      // tiles [t0, t1): whole segments' tiles while the run spans at most cap_segs segments
      const int32_t seg0 = c->tiles1[t0].seg;
      int32_t t1 = t0;
      while (t1 < te_split1 && static_cast<size_t>(c->tiles1[t1].seg - seg0) < cap_segs) ++t1;
      KArgs b = a;
      b.tile_begin = t0;
      b.num_tiles = t1 - t0;
      b.qtab_seg0 = seg0;
      const int32_t nseg = c->tiles1[t1 - 1].seg - seg0 + 1;
      hipEvent_t eb = (t1 == te_split1) ? e1 : nullptr;  // the caller's event completes with the last
      switch (out_kind) {
        case OUT_ACC: err = launch_qsgd_out<OUT_ACC>(in_dtype, b, st.aligned, s, eb, seg0, nseg); break;
        case OUT_F32: err = launch_qsgd_out<OUT_F32>(in_dtype, b, st.aligned, s, eb, seg0, nseg); break;
        case OUT_F64: err = launch_qsgd_out<OUT_F64>(in_dtype, b, st.aligned, s, eb, seg0, nseg); break;
        default: return fail(FEDAVG_ERR_INVALID, "bad out kind");
      }
      if (err != hipSuccess) return fail(FEDAVG_ERR_HIP, std::string("kernel launch: ") + hipGetErrorString(err));
      t0 = t1;
    }
    if (m1) {
      FEDAVG_HIP_TRY(hipEventRecord(m1, s));
      if (done_ev) *done_ev = m1;
    }
    return FEDAVG_OK;
  }
  const int fold = st.delta ? FOLD_DELTA
                            : (c->allow_fma && fma_exact_call(st, in_dtype)) ? FOLD_FMA : FOLD_MULADD;
  const bool partv = a.tiles == c->d_tilesw_bal || a.tiles == c->d_tiles1_bal;  // a balanced order
  if (comb) {
    if (st.delta) return fail(FEDAVG_ERR_INVALID, "the own-window combine takes scalar-weight folds");
    switch (out_kind) {
      case OUT_F32: err = launch_comb_out<OUT_F32>(in_dtype, a, st.aligned, fold, s, e1); break;
      case OUT_F64: err = launch_comb_out<OUT_F64>(in_dtype, a, st.aligned, fold, s, e1); break;
      default: return fail(FEDAVG_ERR_INVALID, "the own-window combine writes fp32 / fp64 outputs");
    }
    if (err != hipSuccess) return fail(FEDAVG_ERR_HIP, std::string("kernel launch: ") + hipGetErrorString(err));
    if (m1) {
      FEDAVG_HIP_TRY(hipEventRecord(m1, s));
      if (done_ev) *done_ev = m1;
    }
    return FEDAVG_OK;
  }
  switch (out_kind) {
    case OUT_ACC: err = launch_out<OUT_ACC>(in_dtype, a, split, st.aligned, fold, nblocks, s, nullptr, e1, wide, partv); break;
    case OUT_F32: err = launch_out<OUT_F32>(in_dtype, a, split, st.aligned, fold, nblocks, s, nullptr, e1, wide, partv); break;
    case OUT_F64: err = launch_out<OUT_F64>(in_dtype, a, split, st.aligned, fold, nblocks, s, nullptr, e1, wide, partv); break;
    default: return fail(FEDAVG_ERR_INVALID, "bad out kind");
  }
  if (err != hipSuccess) return fail(FEDAVG_ERR_HIP, std::string("kernel launch: ") + hipGetErrorString(err));
  if (m1) {
    FEDAVG_HIP_TRY(hipEventRecord(m1, s));
    if (done_ev) *done_ev = m1;
  }
  return FEDAVG_OK;
}

}  // namespace

// Shared with the other translation units of the library (personalized_kernels.hip): one
// thread-local last-error string behind fedavg_last_error().
__attribute__((visibility("hidden"))) int32_t fedavg_internal_fail(int32_t code, const char* msg) {
  return fail(code, msg);
}

// =======================================================================================
// exported C ABI (include/fedavg_hip.h)
// =======================================================================================
namespace {

int32_t check_ctx(const fedavg_ctx* c) {
  if (c == nullptr) return fail(FEDAVG_ERR_INVALID, "null context");
  return FEDAVG_OK;
}

int32_t check_clients(const fedavg_ctx* c, const void* const* client_ptrs, const double* weights,
                      int32_t K, int32_t in_dtype) {
  if (K < 0) return fail(FEDAVG_ERR_INVALID, "num_clients < 0");
  if (K > 0 && (client_ptrs == nullptr || weights == nullptr))
    return fail(FEDAVG_ERR_INVALID, "null client table or weights");
  if (K > 0 && elem_size(in_dtype) == 0) return fail(FEDAVG_ERR_INVALID, "bad input dtype");
  (void)c;
  return FEDAVG_OK;
}

int out_kind_of(int32_t out_dtype) {
  if (out_dtype == FEDAVG_F32) return OUT_F32;
  if (out_dtype == FEDAVG_F64) return OUT_F64;
  return -1;
}

#define FEDAVG_RET(expr)            \
  do {                              \
    int32_t r_ = (expr);            \
    if (r_ != FEDAVG_OK) return r_; \
  } while (0)

}  // namespace

extern "C" __attribute__((visibility("hidden"))) int32_t fedavg_internal_pers_constant(const char* name, int64_t* out);

extern "C" {

int32_t fedavg_abi_version(void) { return FEDAVG_ABI_VERSION; }

int32_t fedavg_build_flags(void) {
  return 0;  // the timing-only ablation variants are no longer part of the sources
}

int32_t fedavg_kernel_constant(const char* name, int64_t* out) {
  if (name == nullptr || out == nullptr) return fail(FEDAVG_ERR_INVALID, "null argument");
  const std::string n(name);
  int64_t v = -1;
  if (n == "tile") v = kTile1;
  else if (n == "tile_wide") v = kTileWide;
  else if (n == "split_tile") v = kTile4;
  else if (n == "qsgd_tile") v = kTile1;
  else if (n == "qsgd_ae") v = kQsgdAE;
  else if (n == "qsgd_group") v = kQsgdGroup;
  else if (n == "nnadq_tile") v = kTile1;
  else if (n == "nnadq_ae") v = kNnadqAE;
  else if (n == "nnadq_group") v = kNnadqGroup;
  else if (n == "nnadq_header") v = kNnadqHeader;
  else if (n.rfind("pers_", 0) == 0) {
    if (fedavg_internal_pers_constant(name, &v) != FEDAVG_OK) v = -1;
  } else {
    const auto dsep = n.rfind('_');
    const std::string key = dsep == std::string::npos ? n : n.substr(0, dsep);
    const std::string d = dsep == std::string::npos ? "" : n.substr(dsep + 1);
    auto pick = [&](auto tag) {
      using T = decltype(tag);
      using GW = Geo<T, 1, (sizeof(T) < 8 && kTileWide > 0) ? kTileWide : kTile1>;
      using G1 = Geo<T, 1, kTile1>;
      constexpr int VPLW = GW::AE / Vec16<T>::n;
      constexpr int CU_B = sizeof(T) == 8 ? FEDAVG_CU_BYTES_F64 : FEDAVG_CU_BYTES;
      constexpr int GROUP = (CU_B / (VPLW * 16)) < 2 ? 2 : (CU_B / (VPLW * 16));
      constexpr bool PIPE = (FEDAVG_PIPE >> (sizeof(T) == 2 ? 0 : sizeof(T) == 4 ? 1 : 2)) & 1;
      constexpr int PG = (FEDAVG_PIPE_BYTES / (VPLW * 16)) < 1 ? 1 : (FEDAVG_PIPE_BYTES / (VPLW * 16));
      if (key == "ae") v = GW::AE;
      else if (key == "lanes") v = GW::LANES;
      else if (key == "ae4096") v = G1::AE;
      else if (key == "lanes4096") v = G1::LANES;
      else if (key == "group") v = GROUP;
      else if (key == "pipe") v = PIPE ? PG : 0;
    };
    if (d == "f32") pick(float{});
    else if (d == "f16") pick(__half{});
    else if (d == "bf16") pick(bf16_t{});
    else if (d == "f64") pick(double{});
  }
  if (v < 0) return fail(FEDAVG_ERR_INVALID, std::string("unknown kernel constant ") + n);
  *out = v;
  return FEDAVG_OK;
}

int64_t fedavg_qsgd_sign_offset(int64_t numel) {
  if (numel < 0) return -1;
  return 16 + static_cast<int64_t>(align_up(static_cast<size_t>(numel), 16));
}

int64_t fedavg_qsgd_record_bytes(int64_t numel) {
  if (numel < 0) return -1;
  return fedavg_qsgd_sign_offset(numel) + static_cast<int64_t>(align_up(static_cast<size_t>((numel + 7) / 8), 16));
}

int64_t fedavg_nnadq_record_bytes(int64_t numel) {
  if (numel < 0) return -1;
  return kNnadqHeader + static_cast<int64_t>(align_up(static_cast<size_t>(numel), 16));
}

const char* fedavg_last_error(void) { return g_last_error.c_str(); }

int32_t fedavg_ctx_create(fedavg_ctx** out, int32_t device, const int64_t* seg_numel,
                          int32_t num_segments, void* accumulator) {
  if (out == nullptr) return fail(FEDAVG_ERR_INVALID, "null out");
  *out = nullptr;
  if (num_segments <= 0 || seg_numel == nullptr) return fail(FEDAVG_ERR_INVALID, "no segments");
  for (int t = 0; t < num_segments; ++t) {
    if (seg_numel[t] <= 0) return fail(FEDAVG_ERR_INVALID, "segment with no elements");
    if (seg_numel[t] > (int64_t(1) << 40)) return fail(FEDAVG_ERR_INVALID, "segment too large");
  }
  if (reinterpret_cast<uintptr_t>(accumulator) % 16 != 0)
    return fail(FEDAVG_ERR_INVALID, "accumulator must be 16-byte aligned");
  FEDAVG_HIP_TRY(hipSetDevice(device));
  fedavg_ctx* c = new fedavg_ctx();
  c->device = device;
  c->T = num_segments;
  c->seg_numel.assign(seg_numel, seg_numel + num_segments);
  c->seg_acc_off.resize(num_segments);
  int64_t off = 0;
  for (int t = 0; t < num_segments; ++t) {
    c->seg_acc_off[t] = off;
    off += static_cast<int64_t>(align_up(static_cast<size_t>(seg_numel[t]), FEDAVG_ACC_ALIGN));
  }
  c->acc_numel = off;
  c->wsum.assign(num_segments, -0.0);  // additive identity: the first weight is taken as is
  if (const char* e = std::getenv("FEDAVG_WIDE_MIN_CLIENTS")) c->wide_min_clients = std::atoi(e);
  if (const char* e = std::getenv("FEDAVG_WALK_ALTERNATE")) c->walk_alternate = std::atoi(e) != 0;
  if (const char* e = std::getenv("FEDAVG_QSGD_TABLE_CAP")) {
    const long long v = std::atoll(e);
    if (v > 0) c->qtab_cap_bytes = static_cast<size_t>(v);
  }
  c->valid.assign(num_segments, 0);
  build_tiles(c->seg_numel, kTile1, c->tiles1);
  build_tiles(c->seg_numel, kTile4, c->tiles4);
  if (kTileWide > 0) build_tiles(c->seg_numel, kTileWide, c->tilesw);
  {
    // balanced whole-layout orders (FEDAVG_BALANCE bit 0: fp32 on the wide table, bit 1: fp64 on
    // the kTile1 table), sized by the resident workgroups of the kernel that runs them
    const char* env = std::getenv("FEDAVG_BALANCE");
    const int bal = env ? std::atoi(env) : FEDAVG_BALANCE_DEFAULT;
    // FEDAVG_BALANCE_ALWAYS=1: the balanced orders for every layout (A/B and the geometry tests)
    const char* always_env = std::getenv("FEDAVG_BALANCE_ALWAYS");
    const bool always = always_env && std::atoi(always_env) != 0;
    int cus = 0;
    if (bal && hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && cus > 0) {
      int per_cu = 0;
      // only where the launch's last wave of workgroups is thin (less than half the resident
      // slots): elsewhere the plain order's tail already balances and the balanced order's PV
      // kernel is the slower one (profiles/r03_ab_matrix.txt)
      auto thin_tail = [&](size_t tiles, int64_t slots) {
        const int64_t rem = static_cast<int64_t>(tiles) % slots;
        return always || (tiles > static_cast<size_t>(slots) && rem > 0 && 2 * rem < slots);
      };
      if ((bal & 1) && kTileWide > 0 &&
          hipOccupancyMaxActiveBlocksPerMultiprocessor(
              &per_cu, reinterpret_cast<const void*>(&fedavg_tile_kernel<float, OUT_F32, 1, true, FOLD_FMA, kTileWide, true>),
              Geo<float, 1, kTileWide>::THREADS, 0) == hipSuccess && per_cu > 0 &&
          thin_tail(c->tilesw.size(), static_cast<int64_t>(per_cu) * cus))
        c->tilesw_bal_head =
            build_balanced_tiles(c->seg_numel, kTileWide, Geo<float, 1, kTileWide>::LANES * Vec16<float>::n,
                                 static_cast<int64_t>(per_cu) * cus, c->tilesw_bal);
      per_cu = 0;
      if ((bal & 2) &&
          hipOccupancyMaxActiveBlocksPerMultiprocessor(
              &per_cu, reinterpret_cast<const void*>(&fedavg_tile_kernel<double, OUT_F32, 1, true, FOLD_FMA, kTile1, true>),
              Geo<double, 1, kTile1>::THREADS, 0) == hipSuccess && per_cu > 0 &&
          thin_tail(c->tiles1.size(), static_cast<int64_t>(per_cu) * cus))
        c->tiles1_bal_head =
            build_balanced_tiles(c->seg_numel, kTile1, Geo<double, 1, kTile1>::LANES * Vec16<double>::n,
                                 static_cast<int64_t>(per_cu) * cus, c->tiles1_bal);
    }
  }
  if (c->tiles1.size() > static_cast<size_t>(INT32_MAX / 2)) {
    delete c;
    return fail(FEDAVG_ERR_INVALID, "layout too large");
  }
  std::vector<SegDesc> segs(num_segments);
  for (int t = 0; t < num_segments; ++t) segs[t] = SegDesc{c->seg_acc_off[t], c->seg_numel[t]};

  auto cleanup = [&](hipError_t e, const char* what) {
    fedavg_ctx_destroy(c);
    return fail(FEDAVG_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
  };
  hipError_t e;
  if ((e = hipMalloc(reinterpret_cast<void**>(&c->d_tiles1), sizeof(TileDesc) * c->tiles1.size())) != hipSuccess)
    return cleanup(e, "hipMalloc tiles1");
  if ((e = hipMalloc(reinterpret_cast<void**>(&c->d_tiles4), sizeof(TileDesc) * c->tiles4.size())) != hipSuccess)
    return cleanup(e, "hipMalloc tiles4");
  if ((e = hipMalloc(reinterpret_cast<void**>(&c->d_segs), sizeof(SegDesc) * segs.size())) != hipSuccess)
    return cleanup(e, "hipMalloc segs");
  if ((e = hipHostMalloc(reinterpret_cast<void**>(&c->h_flag), sizeof(uint32_t) * 4,
                         hipHostMallocMapped | hipHostMallocCoherent)) != hipSuccess)
    return cleanup(e, "hipHostMalloc flag");
  if ((e = hipHostGetDevicePointer(reinterpret_cast<void**>(&c->d_flag), c->h_flag, 0)) != hipSuccess)
    return cleanup(e, "hipHostGetDevicePointer flag");
  if ((e = hipMemcpy(c->d_tiles1, c->tiles1.data(), sizeof(TileDesc) * c->tiles1.size(), hipMemcpyHostToDevice)) != hipSuccess)
    return cleanup(e, "hipMemcpy tiles1");
  if ((e = hipMemcpy(c->d_tiles4, c->tiles4.data(), sizeof(TileDesc) * c->tiles4.size(), hipMemcpyHostToDevice)) != hipSuccess)
    return cleanup(e, "hipMemcpy tiles4");
  if (!c->tilesw.empty()) {
    if ((e = hipMalloc(reinterpret_cast<void**>(&c->d_tilesw), sizeof(TileDesc) * c->tilesw.size())) != hipSuccess)
      return cleanup(e, "hipMalloc tilesw");
    if ((e = hipMemcpy(c->d_tilesw, c->tilesw.data(), sizeof(TileDesc) * c->tilesw.size(), hipMemcpyHostToDevice)) !=
        hipSuccess)
      return cleanup(e, "hipMemcpy tilesw");
  }
  if ((e = hipMemcpy(c->d_segs, segs.data(), sizeof(SegDesc) * segs.size(), hipMemcpyHostToDevice)) != hipSuccess)
    return cleanup(e, "hipMemcpy segs");
  for (auto [host, dev] : {std::pair{&c->tilesw_bal, &c->d_tilesw_bal}, std::pair{&c->tiles1_bal, &c->d_tiles1_bal}}) {
    if (host->empty()) continue;
    if ((e = hipMalloc(reinterpret_cast<void**>(dev), sizeof(TileDesc) * host->size())) != hipSuccess)
      return cleanup(e, "hipMalloc balanced tiles");
    if ((e = hipMemcpy(*dev, host->data(), sizeof(TileDesc) * host->size(), hipMemcpyHostToDevice)) != hipSuccess)
      return cleanup(e, "hipMemcpy balanced tiles");
  }
  std::memset(c->h_flag, 0, sizeof(uint32_t) * 4);
  if (accumulator != nullptr) {
    c->acc = static_cast<double*>(accumulator);
    c->owns_acc = false;
  } else {
    if ((e = hipMalloc(reinterpret_cast<void**>(&c->acc), sizeof(double) * c->acc_numel)) != hipSuccess)
      return cleanup(e, "hipMalloc accumulator");
    c->owns_acc = true;
    if ((e = hipMemset(c->acc, 0, sizeof(double) * c->acc_numel)) != hipSuccess)
      return cleanup(e, "hipMemset accumulator");
  }
  *out = c;
  return FEDAVG_OK;
}

int32_t fedavg_ctx_destroy(fedavg_ctx* c) {
  if (c == nullptr) return FEDAVG_OK;
  (void)hipSetDevice(c->device);
  if (c->dyn.active) {
    // an open dynamic wave ends with the rows it has (its ACK arrives within a mirror poll)
    const DynLayout L(c->T, c->dyn.cap);
    DynCtl* ctl = reinterpret_cast<DynCtl*>(c->dyn.host + L.ctl);
    __atomic_store_n(&ctl->word, dyn_word(static_cast<uint32_t>(c->dyn.published - c->dyn.base), 1u, OUT_ACC, 0u),
                     __ATOMIC_RELEASE);
    c->dyn.active = false;
  }
  if (c->dyn.stream) (void)hipStreamSynchronize(c->dyn.stream);
  if (c->dyn.edge_stream) (void)hipStreamSynchronize(c->dyn.edge_stream);
  (void)hipDeviceSynchronize();
  if (c->dyn.host) (void)hipHostFree(c->dyn.host);
  if (c->dyn.mirror) (void)hipFree(c->dyn.mirror);
  if (c->dyn.tend) (void)hipFree(c->dyn.tend);
  if (c->dyn.dtab) (void)hipFree(c->dyn.dtab);
  if (c->dyn.d_tiles) (void)hipFree(c->dyn.d_tiles);
  if (c->dyn.d_edge_tiles) (void)hipFree(c->dyn.d_edge_tiles);
  if (c->dyn.edge_done) (void)hipEventDestroy(c->dyn.edge_done);
  if (c->dyn.edge_stream) (void)hipStreamDestroy(c->dyn.edge_stream);
  if (c->dyn.start) (void)hipEventDestroy(c->dyn.start);
  if (c->dyn.done) (void)hipEventDestroy(c->dyn.done);
  if (c->dyn.stream) (void)hipStreamDestroy(c->dyn.stream);
  for (auto& sl : c->slots) {
    if (sl.host) (void)hipHostFree(sl.host);
    if (sl.dev) (void)hipFree(sl.dev);
    if (sl.done) (void)hipEventDestroy(sl.done);
  }
  for (auto& pr : c->prof_events) {
    (void)hipEventDestroy(pr.first);
    (void)hipEventDestroy(pr.second);
  }
  for (auto& pr : c->dyn.prof) {
    (void)hipEventDestroy(pr.first);
    (void)hipEventDestroy(pr.second);
  }
  if (c->dyn.prof_start) (void)hipEventDestroy(c->dyn.prof_start);
  for (auto e : c->event_pool) (void)hipEventDestroy(e);
  if (c->d_tiles1) (void)hipFree(c->d_tiles1);
  if (c->d_tiles4) (void)hipFree(c->d_tiles4);
  if (c->d_tilesw) (void)hipFree(c->d_tilesw);
  if (c->d_tilesw_bal) (void)hipFree(c->d_tilesw_bal);
  if (c->d_tiles1_bal) (void)hipFree(c->d_tiles1_bal);
  if (c->d_segs) (void)hipFree(c->d_segs);
  if (c->qtab) (void)hipFree(c->qtab);
  if (c->h_flag) (void)hipHostFree(c->h_flag);
  if (c->owns_acc && c->acc) (void)hipFree(c->acc);
  if (c->aux_host) (void)hipHostFree(c->aux_host);
  if (c->aux_dev) (void)hipFree(c->aux_dev);
  if (c->aux_done) (void)hipEventDestroy(c->aux_done);
  delete c;
  return FEDAVG_OK;
}

int64_t fedavg_acc_numel(const fedavg_ctx* c) { return c ? c->acc_numel : -1; }

int64_t fedavg_segment_offset(const fedavg_ctx* c, int32_t seg) {
  if (!c || seg < 0 || seg >= c->T) return -1;
  return c->seg_acc_off[seg];
}

void* fedavg_accumulator(const fedavg_ctx* c) { return c ? c->acc : nullptr; }

int32_t fedavg_set_split_policy(fedavg_ctx* c, int32_t policy) {
  FEDAVG_RET(check_ctx(c));
  if (policy < 0 || policy > 2) return fail(FEDAVG_ERR_INVALID, "split policy must be 0, 1 or 2");
  c->split_policy = policy;
  return FEDAVG_OK;
}

int32_t fedavg_set_fused_fold(fedavg_ctx* c, int32_t enable) {
  FEDAVG_RET(check_ctx(c));
  c->allow_fma = enable != 0;
  return FEDAVG_OK;
}

int32_t fedavg_dyn_close(fedavg_ctx* c, void* const* out_ptrs, int32_t out_dtype, int32_t join, void* stream,
                         int32_t* folded_out, int32_t* finalized_out);

int32_t fedavg_reset(fedavg_ctx* c, void* stream) {
  FEDAVG_RET(check_ctx(c));
  FEDAVG_HIP_TRY(hipSetDevice(c->device));
  if (c->dyn.active) {  // an abandoned round's dynamic wave: ended and drained before the reset
    FEDAVG_RET(fedavg_dyn_close(c, nullptr, FEDAVG_F64, 1, stream, nullptr, nullptr));
    FEDAVG_HIP_TRY(hipStreamSynchronize(c->dyn.stream));
    FEDAVG_HIP_TRY(hipStreamSynchronize(c->dyn.edge_stream));
  }
  if (c->dyn.unjoined) {  // a finalized wave never checked: it may still raise a flag
    FEDAVG_HIP_TRY(hipEventSynchronize(c->dyn.done));
    FEDAVG_HIP_TRY(hipEventSynchronize(c->dyn.edge_done));
    c->dyn.unjoined = false;
  }
  std::fill(c->wsum.begin(), c->wsum.end(), -0.0);
  std::fill(c->valid.begin(), c->valid.end(), 0);
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (stream_idle(s)) {
    // idle stream (the usual case: the previous round ended on the host): clear the host-coherent
    // flag words directly — an async memset is a blit kernel plus ~15 µs of queue latency per round
    for (int i = 0; i < 4; ++i) __atomic_store_n(&c->h_flag[i], 0u, __ATOMIC_RELEASE);
  } else {
    if (const char* v = std::getenv("FEDAVG_DYN_TRACE"); v && *v == '1') std::fprintf(stderr, "[reset] busy stream: memset\n");
    FEDAVG_HIP_TRY(hipMemsetAsync(c->d_flag, 0, sizeof(uint32_t) * 4, s));
  }
  return FEDAVG_OK;
}

int32_t fedavg_total_weights(const fedavg_ctx* c, double* out) {
  FEDAVG_RET(check_ctx(c));
  if (!out) return fail(FEDAVG_ERR_INVALID, "null out");
  for (int t = 0; t < c->T; ++t) out[t] = c->wsum[t];
  return FEDAVG_OK;
}

int32_t fedavg_accumulate(fedavg_ctx* c, const void* const* client_ptrs, int32_t in_dtype,
                          const double* weights, int32_t K, void* stream) {
  FEDAVG_RET(check_ctx(c));
  FEDAVG_RET(check_clients(c, client_ptrs, weights, K, in_dtype));
  if (K == 0) return FEDAVG_OK;
  FEDAVG_HIP_TRY(hipSetDevice(c->device));
  hipStream_t s = static_cast<hipStream_t>(stream);
  Staged st;
  FEDAVG_RET(stage_tables(c, s, client_ptrs, weights, K, nullptr, nullptr, c->valid.data(), st));
  const int split = choose_split(c, st.Kmax);
  FEDAVG_RET(launch_main(c, s, st, in_dtype, OUT_ACC, split, 0, 0, static_cast<int32_t>(c->tiles1.size())));
  // host mirror: total weights in arrival order (fed_avg_algorithm.py:59-62)
  for (int k = 0; k < K; ++k)
    for (int t = 0; t < c->T; ++t)
      if (client_ptrs[static_cast<int64_t>(k) * c->T + t] != nullptr) {
        c->wsum[t] += weights[static_cast<int64_t>(k) * c->T + t];
        c->valid[t] = 1;
      }
  return FEDAVG_OK;
}

int32_t fedavg_aggregate(fedavg_ctx* c, const void* const* client_ptrs, int32_t in_dtype,
                         const double* weights, int32_t K, void* const* out_ptrs, int32_t out_dtype,
                         void* stream) {
  FEDAVG_RET(check_ctx(c));
  FEDAVG_RET(check_clients(c, client_ptrs, weights, K, in_dtype));
  const int ok = out_kind_of(out_dtype);
  if (ok < 0) return fail(FEDAVG_ERR_INVALID, "out dtype must be FEDAVG_F32 or FEDAVG_F64");
  if (out_ptrs == nullptr) return fail(FEDAVG_ERR_INVALID, "null out table");
  for (int t = 0; t < c->T; ++t)
    if (out_ptrs[t] == nullptr) return fail(FEDAVG_ERR_INVALID, "null output pointer");
  // totals including this last wave, in arrival order
  std::vector<double> wtot(c->wsum);
  std::vector<int32_t> will_have(c->valid);
  for (int k = 0; k < K; ++k)
    for (int t = 0; t < c->T; ++t)
      if (client_ptrs[static_cast<int64_t>(k) * c->T + t] != nullptr) {
        wtot[t] += weights[static_cast<int64_t>(k) * c->T + t];
        will_have[t] = 1;
      }
  for (int t = 0; t < c->T; ++t)
    if (!will_have[t])
      return fail(FEDAVG_ERR_STATE, "segment " + std::to_string(t) +
                                        " has no accumulated data (fed_avg_algorithm.py:88)");
  FEDAVG_HIP_TRY(hipSetDevice(c->device));
  hipStream_t s = static_cast<hipStream_t>(stream);
  Staged st;
  FEDAVG_RET(stage_tables(c, s, K > 0 ? client_ptrs : nullptr, weights, K, out_ptrs, wtot.data(),
                          c->valid.data(), st));
  const int split = choose_split(c, st.Kmax);
  FEDAVG_RET(launch_main(c, s, st, K > 0 ? in_dtype : FEDAVG_F32, ok, split, 0, 0,
                         static_cast<int32_t>(c->tiles1.size())));
  // _aggregate_parameter resets the accumulator (fed_avg_algorithm.py:90,98)
  std::fill(c->wsum.begin(), c->wsum.end(), -0.0);
  std::fill(c->valid.begin(), c->valid.end(), 0);
  return FEDAVG_OK;
}

int32_t fedavg_accumulate_delta(fedavg_ctx* c, const void* const* client_ptrs, int32_t in_dtype,
                                const double* weights, int32_t K, const void* const* base_ptrs,
                                void* stream) {
  FEDAVG_RET(check_ctx(c));
  FEDAVG_RET(check_clients(c, client_ptrs, weights, K, in_dtype));
  if (!base_ptrs) return fail(FEDAVG_ERR_INVALID, "null base table");
  for (int t = 0; t < c->T; ++t)
    if (!base_ptrs[t]) return fail(FEDAVG_ERR_INVALID, "null base pointer");
  if (K == 0) return FEDAVG_OK;
  FEDAVG_HIP_TRY(hipSetDevice(c->device));
  hipStream_t s = static_cast<hipStream_t>(stream);
  Staged st;
  FEDAVG_RET(stage_tables(c, s, client_ptrs, weights, K, nullptr, nullptr, c->valid.data(), st, base_ptrs));
  FEDAVG_RET(launch_main(c, s, st, in_dtype, OUT_ACC, 1, 0, 0, static_cast<int32_t>(c->tiles1.size())));
  for (int k = 0; k < K; ++k)
    for (int t = 0; t < c->T; ++t)
      if (client_ptrs[static_cast<int64_t>(k) * c->T + t] != nullptr) {
        c->wsum[t] += weights[static_cast<int64_t>(k) * c->T + t];
        c->valid[t] = 1;
      }
  return FEDAVG_OK;
}

int32_t fedavg_aggregate_delta(fedavg_ctx* c, const void* const* client_ptrs, int32_t in_dtype,
                               const double* weights, int32_t K, const void* const* base_ptrs,
                               void* const* out_ptrs, int32_t out_dtype, void* stream) {
  FEDAVG_RET(check_ctx(c));
  FEDAVG_RET(check_clients(c, client_ptrs, weights, K, in_dtype));
  if (!base_ptrs) return fail(FEDAVG_ERR_INVALID, "null base table");
  for (int t = 0; t < c->T; ++t)
    if (!base_ptrs[t]) return fail(FEDAVG_ERR_INVALID, "null base pointer");
  const int ok = out_kind_of(out_dtype);
  if (ok < 0) return fail(FEDAVG_ERR_INVALID, "out dtype must be FEDAVG_F32 or FEDAVG_F64");
  if (out_ptrs == nullptr) return fail(FEDAVG_ERR_INVALID, "null out table");
  std::vector<double> wtot(c->wsum);
  std::vector<int32_t> will_have(c->valid);
  for (int k = 0; k < K; ++k)
    for (int t = 0; t < c->T; ++t)
      if (client_ptrs[static_cast<int64_t>(k) * c->T + t] != nullptr) {
        wtot[t] += weights[static_cast<int64_t>(k) * c->T + t];
        will_have[t] = 1;
      }
  for (int t = 0; t < c->T; ++t) {
    if (!will_have[t])
      return fail(FEDAVG_ERR_STATE, "segment " + std::to_string(t) + " has no accumulated data");
    if (out_ptrs[t] == nullptr) return fail(FEDAVG_ERR_INVALID, "null output pointer");
  }
  FEDAVG_HIP_TRY(hipSetDevice(c->device));
  hipStream_t s = static_cast<hipStream_t>(stream);
  Staged st;
  FEDAVG_RET(stage_tables(c, s, K > 0 ? client_ptrs : nullptr, weights, K, out_ptrs, wtot.data(),
                          c->valid.data(), st, base_ptrs));
  FEDAVG_RET(launch_main(c, s, st, K > 0 ? in_dtype : FEDAVG_F32, ok, 1, 0, 0,
                         static_cast<int32_t>(c->tiles1.size())));
  std::fill(c->wsum.begin(), c->wsum.end(), -0.0);
  std::fill(c->valid.begin(), c->valid.end(), 0);
  return FEDAVG_OK;
}

int32_t fedavg_weighted_avg(fedavg_ctx* c, const void* const* client_ptrs, int32_t in_dtype,
                            const double* ratios, int32_t K, void* const* out_ptrs, int32_t out_dtype,
                            void* stream) {
  FEDAVG_RET(check_ctx(c));
  FEDAVG_RET(check_clients(c, client_ptrs, ratios, K, in_dtype));
  if (K == 0) return fail(FEDAVG_ERR_STATE, "weighted_avg of no clients (aggregation_algorithm.py:57)");
  const int ok = out_kind_of(out_dtype);
  if (ok < 0) return fail(FEDAVG_ERR_INVALID, "out dtype must be FEDAVG_F32 or FEDAVG_F64");
  if (out_ptrs == nullptr) return fail(FEDAVG_ERR_INVALID, "null out table");
  for (int t = 0; t < c->T; ++t) {
    if (out_ptrs[t] == nullptr) return fail(FEDAVG_ERR_INVALID, "null output pointer");
    bool any = false;
    for (int k = 0; k < K && !any; ++k) any = client_ptrs[static_cast<int64_t>(k) * c->T + t] != nullptr;
    if (!any) return fail(FEDAVG_ERR_STATE, "segment " + std::to_string(t) + " has no client data");
  }
  FEDAVG_HIP_TRY(hipSetDevice(c->device));
  hipStream_t s = static_cast<hipStream_t>(stream);
  std::vector<int32_t> no_acc(c->T, 0);
  std::vector<double> ones(c->T, 1.0);  // x / 1.0 == x exactly: no division on this path
  Staged st;
  FEDAVG_RET(stage_tables(c, s, client_ptrs, ratios, K, out_ptrs, ones.data(), no_acc.data(), st));
  const int split = choose_split(c, st.Kmax);
  return launch_main(c, s, st, in_dtype, ok, split, 0, 0, static_cast<int32_t>(c->tiles1.size()));
}

int32_t fedavg_num_tiles(const fedavg_ctx* c) {
  if (!c) return -1;
  return static_cast<int32_t>(c->tiles1.size());
}

int32_t fedavg_tile_range(const fedavg_ctx* c, int32_t tb, int32_t te, int64_t* acc_begin, int64_t* acc_end) {
  FEDAVG_RET(check_ctx(c));
  const int32_t n = static_cast<int32_t>(c->tiles1.size());
  if (te < 0) te = n;
  if (tb < 0 || tb > te || te > n) return fail(FEDAVG_ERR_INVALID, "bad tile range");
  if (!acc_begin || !acc_end) return fail(FEDAVG_ERR_INVALID, "null out");
  if (tb == te) {
    *acc_begin = *acc_end = (tb < n) ? c->seg_acc_off[c->tiles1[tb].seg] + c->tiles1[tb].start : c->acc_numel;
    return FEDAVG_OK;
  }
  const TileDesc& f = c->tiles1[tb];
  const TileDesc& l = c->tiles1[te - 1];
  *acc_begin = c->seg_acc_off[f.seg] + f.start;
  // include the segment's alignment padding when the range ends a segment
  const int64_t end = c->seg_acc_off[l.seg] + l.start + l.count;
  *acc_end = (l.start + l.count == c->seg_numel[l.seg])
                 ? ((l.seg + 1 < c->T) ? c->seg_acc_off[l.seg + 1] : c->acc_numel)
                 : end;
  return FEDAVG_OK;
}

int32_t fedavg_partial(fedavg_ctx* c, const void* const* client_ptrs, int32_t in_dtype,
                       const double* weights, int32_t K, int32_t zero_init, int32_t tb, int32_t te,
                       void* stream) {
  FEDAVG_RET(check_ctx(c));
  FEDAVG_RET(check_clients(c, client_ptrs, weights, K, in_dtype));
  const int32_t n = static_cast<int32_t>(c->tiles1.size());
  if (te < 0) te = n;
  if (tb < 0 || tb > te || te > n) return fail(FEDAVG_ERR_INVALID, "bad tile range");
  if (!zero_init && K == 0) return FEDAVG_OK;
  FEDAVG_HIP_TRY(hipSetDevice(c->device));
  hipStream_t s = static_cast<hipStream_t>(stream);
  Staged st;
  FEDAVG_RET(stage_tables(c, s, K > 0 ? client_ptrs : nullptr, weights, K, nullptr, nullptr,
                          c->valid.data(), st));
  // tile ranges are defined on the 2048-element tiles: the exact-order kernel
  return launch_main(c, s, st, K > 0 ? in_dtype : FEDAVG_F32, OUT_ACC, 1, zero_init ? 1 : 0, tb, te);
}

int32_t fedavg_set_accumulated(fedavg_ctx* c, const double* total_weights) {
  FEDAVG_RET(check_ctx(c));
  if (!total_weights) return fail(FEDAVG_ERR_INVALID, "null total weights");
  for (int t = 0; t < c->T; ++t) {
    c->wsum[t] = total_weights[t];
    c->valid[t] = 1;
  }
  return FEDAVG_OK;
}

int32_t fedavg_finalize_range(fedavg_ctx* c, void* const* out_ptrs, int32_t out_dtype, int32_t tb,
                              int32_t te, void* stream) {
  FEDAVG_RET(check_ctx(c));
  const int ok = out_kind_of(out_dtype);
  if (ok < 0) return fail(FEDAVG_ERR_INVALID, "out dtype must be FEDAVG_F32 or FEDAVG_F64");
  if (out_ptrs == nullptr) return fail(FEDAVG_ERR_INVALID, "null out table");
  const int32_t n = static_cast<int32_t>(c->tiles1.size());
  if (te < 0) te = n;
  if (tb < 0 || tb > te || te > n) return fail(FEDAVG_ERR_INVALID, "bad tile range");
  for (int t = 0; t < c->T; ++t) {
    if (!c->valid[t]) return fail(FEDAVG_ERR_STATE, "segment " + std::to_string(t) + " not accumulated");
    if (out_ptrs[t] == nullptr) return fail(FEDAVG_ERR_INVALID, "null output pointer");
  }
  FEDAVG_HIP_TRY(hipSetDevice(c->device));
  hipStream_t s = static_cast<hipStream_t>(stream);
  Staged st;
  FEDAVG_RET(stage_tables(c, s, nullptr, nullptr, 0, out_ptrs, c->wsum.data(), c->valid.data(), st));
  return launch_main(c, s, st, FEDAVG_F32, ok, 1, 0, tb, te);
}

int32_t fedavg_check(fedavg_ctx* c, void* stream, uint32_t* flags_out) {
  FEDAVG_RET(check_ctx(c));
  FEDAVG_HIP_TRY(hipSetDevice(c->device));
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (c->dyn.unjoined) {  // a finalized dynamic wave the caller's stream did not wait for
    FEDAVG_HIP_TRY(hipEventSynchronize(c->dyn.done));
    FEDAVG_HIP_TRY(hipEventSynchronize(c->dyn.edge_done));
    c->dyn.unjoined = false;
  }
  FEDAVG_HIP_TRY(hipStreamSynchronize(s));
  const uint32_t f = (__atomic_load_n(&c->h_flag[0], __ATOMIC_ACQUIRE) ? FEDAVG_FLAG_ACC_NAN : 0u) |
                     (__atomic_load_n(&c->h_flag[1], __ATOMIC_ACQUIRE) ? FEDAVG_FLAG_RESULT_NAN : 0u);
  if (flags_out) *flags_out = f;
  if (f & FEDAVG_FLAG_ACC_NAN) return fail(FEDAVG_ERR_NAN_ACCUM, "NaN in the accumulator");
  if (f & FEDAVG_FLAG_RESULT_NAN) return fail(FEDAVG_ERR_NAN_RESULT, "NaN in the aggregated result");
  return FEDAVG_OK;
}

int32_t fedavg_find_nan_clients(fedavg_ctx* c, const void* const* client_ptrs, int32_t in_dtype,
                                int32_t K, int32_t* out_bad, void* stream) {
  FEDAVG_RET(check_ctx(c));
  if (K <= 0 || !client_ptrs || !out_bad) return fail(FEDAVG_ERR_INVALID, "bad arguments");
  if (elem_size(in_dtype) == 0) return fail(FEDAVG_ERR_INVALID, "bad input dtype");
  FEDAVG_HIP_TRY(hipSetDevice(c->device));
  hipStream_t s = static_cast<hipStream_t>(stream);
  // segment-major, uncompacted table (NULL = absent)
  std::vector<const void*> tk(static_cast<size_t>(K) * c->T);
  for (int k = 0; k < K; ++k)
    for (int t = 0; t < c->T; ++t)
      tk[static_cast<size_t>(t) * K + k] = client_ptrs[static_cast<size_t>(k) * c->T + t];
  void* d_tab = nullptr;
  int32_t* d_bad = nullptr;
  FEDAVG_HIP_TRY(hipMalloc(&d_tab, sizeof(void*) * tk.size()));
  FEDAVG_HIP_TRY(hipMalloc(reinterpret_cast<void**>(&d_bad), sizeof(int32_t) * K));
  hipError_t e = hipMemcpyAsync(d_tab, tk.data(), sizeof(void*) * tk.size(), hipMemcpyHostToDevice, s);
  if (e == hipSuccess) e = hipMemsetAsync(d_bad, 0, sizeof(int32_t) * K, s);
  if (e == hipSuccess) {
    dim3 grid(static_cast<unsigned>(c->tiles1.size()), static_cast<unsigned>(K));
    const void* const* tab = static_cast<const void* const*>(d_tab);
    switch (in_dtype) {
      case FEDAVG_QSGD_F32: hipLaunchKernelGGL(qsgd_nan_scan_kernel<float>, grid, dim3(kThreads), 0, s, c->d_tiles1, c->d_segs, tab, K, d_bad); break;
      case FEDAVG_QSGD_F64: hipLaunchKernelGGL(qsgd_nan_scan_kernel<double>, grid, dim3(kThreads), 0, s, c->d_tiles1, c->d_segs, tab, K, d_bad); break;
      case FEDAVG_NNADQ_F32: hipLaunchKernelGGL(nnadq_nan_scan_kernel<float>, grid, dim3(kThreads), 0, s, c->d_tiles1, tab, K, d_bad); break;
      case FEDAVG_NNADQ_F64: hipLaunchKernelGGL(nnadq_nan_scan_kernel<double>, grid, dim3(kThreads), 0, s, c->d_tiles1, tab, K, d_bad); break;
      case FEDAVG_F32: hipLaunchKernelGGL(nan_scan_kernel<float>, grid, dim3(kThreads), 0, s, c->d_tiles1, tab, K, d_bad); break;
      case FEDAVG_F16: hipLaunchKernelGGL(nan_scan_kernel<__half>, grid, dim3(kThreads), 0, s, c->d_tiles1, tab, K, d_bad); break;
      case FEDAVG_BF16: hipLaunchKernelGGL(nan_scan_kernel<bf16_t>, grid, dim3(kThreads), 0, s, c->d_tiles1, tab, K, d_bad); break;
      default: hipLaunchKernelGGL(nan_scan_kernel<double>, grid, dim3(kThreads), 0, s, c->d_tiles1, tab, K, d_bad); break;
    }
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipMemcpyAsync(out_bad, d_bad, sizeof(int32_t) * K, hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  (void)hipFree(d_tab);
  (void)hipFree(d_bad);
  if (e != hipSuccess) return fail(FEDAVG_ERR_HIP, std::string("find_nan_clients: ") + hipGetErrorString(e));
  return FEDAVG_OK;
}

int32_t fedavg_prof_enable(fedavg_ctx* c, int32_t enable) {
  FEDAVG_RET(check_ctx(c));
  c->prof = enable != 0;
  return FEDAVG_OK;
}

int32_t fedavg_prof_collect(fedavg_ctx* c, double* total_ms, int32_t* launches) {
  FEDAVG_RET(check_ctx(c));
  double sum = 0.0;
  for (auto& pr : c->prof_events) {
    FEDAVG_HIP_TRY(hipEventSynchronize(pr.second));
    float ms = 0.f;
    FEDAVG_HIP_TRY(hipEventElapsedTime(&ms, pr.first, pr.second));
    sum += ms;
  }
  if (total_ms) *total_ms = sum;
  if (launches) *launches = static_cast<int32_t>(c->prof_events.size());
  for (auto& pr : c->prof_events) {
    c->event_pool.push_back(pr.first);
    c->event_pool.push_back(pr.second);
  }
  c->prof_events.clear();
  return FEDAVG_OK;
}

int32_t fedavg_plan_create(fedavg_ctx* c, const void* const* client_ptrs, int32_t in_dtype,
                           const double* weights, int32_t K, void* const* out_ptrs, int32_t out_dtype,
                           fedavg_plan** out) {
  FEDAVG_RET(check_ctx(c));
  if (!out) return fail(FEDAVG_ERR_INVALID, "null out");
  *out = nullptr;
  FEDAVG_RET(check_clients(c, client_ptrs, weights, K, in_dtype));
  if (K == 0) return fail(FEDAVG_ERR_STATE, "a plan needs clients");
  const int ok = out_kind_of(out_dtype);
  if (ok < 0) return fail(FEDAVG_ERR_INVALID, "out dtype must be FEDAVG_F32 or FEDAVG_F64");
  if (!out_ptrs) return fail(FEDAVG_ERR_INVALID, "null out table");
  std::vector<double> wtot(c->T, -0.0);
  std::vector<int32_t> has(c->T, 0);
  for (int k = 0; k < K; ++k)
    for (int t = 0; t < c->T; ++t)
      if (client_ptrs[static_cast<int64_t>(k) * c->T + t] != nullptr) {
        wtot[t] += weights[static_cast<int64_t>(k) * c->T + t];  // arrival order
        has[t] = 1;
      }
  for (int t = 0; t < c->T; ++t) {
    if (!has[t]) return fail(FEDAVG_ERR_STATE, "segment " + std::to_string(t) + " has no client data");
    if (!out_ptrs[t]) return fail(FEDAVG_ERR_INVALID, "null output pointer");
  }
  FEDAVG_HIP_TRY(hipSetDevice(c->device));
  auto* p = new fedavg_plan();
  p->ctx = c;
  p->device = c->device;
  p->in_dtype = in_dtype;
  p->out_kind = ok;
  const BlobLayout L(c->T, K);
  std::vector<int32_t> no_acc(c->T, 0);
  std::vector<char> blob;
  build_blob(c, client_ptrs, weights, K, out_ptrs, wtot.data(), no_acc.data(), p->st, blob, L);
  hipError_t e = hipMalloc(reinterpret_cast<void**>(&p->dev), L.bytes);
  if (e == hipSuccess) e = hipMemcpy(p->dev, blob.data(), L.bytes, hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    if (p->dev) (void)hipFree(p->dev);
    delete p;
    return fail(FEDAVG_ERR_HIP, std::string("plan upload: ") + hipGetErrorString(e));
  }
  L.point(p->dev, p->st.tab);
  p->split = choose_split(c, p->st.Kmax);
  *out = p;
  return FEDAVG_OK;
}

namespace {
// Stage a plan's blob once into its own device buffer.
int32_t upload_plan(fedavg_plan* p, std::vector<char>& blob, const BlobLayout& L) {
  hipError_t e = hipMalloc(reinterpret_cast<void**>(&p->dev), L.bytes);
  if (e == hipSuccess) e = hipMemcpy(p->dev, blob.data(), L.bytes, hipMemcpyHostToDevice);
  if (e != hipSuccess) return fail(FEDAVG_ERR_HIP, std::string("plan upload: ") + hipGetErrorString(e));
  L.point(p->dev, p->st.tab);
  return FEDAVG_OK;
}
}  // namespace

int32_t fedavg_plan_create_partial(fedavg_ctx* c, const void* const* client_ptrs, int32_t in_dtype,
                                   const double* weights, int32_t K, int32_t zero_init, fedavg_plan** out) {
  FEDAVG_RET(check_ctx(c));
  if (!out) return fail(FEDAVG_ERR_INVALID, "null out");
  *out = nullptr;
  FEDAVG_RET(check_clients(c, client_ptrs, weights, K, in_dtype));
  FEDAVG_HIP_TRY(hipSetDevice(c->device));
  auto* p = new fedavg_plan();
  p->ctx = c;
  p->device = c->device;
  p->kind = fedavg_plan::PARTIAL;
  p->in_dtype = K > 0 ? in_dtype : FEDAVG_F32;
  p->out_kind = OUT_ACC;
  p->zero_init = zero_init ? 1 : 0;
  const BlobLayout L(c->T, std::max(K, 1));
  std::vector<int32_t> acc_in(c->T, zero_init ? 0 : 1);  // a continuing partial reads every segment
  std::vector<char> blob;
  build_blob(c, K > 0 ? client_ptrs : nullptr, weights, K, nullptr, nullptr, acc_in.data(), p->st, blob, L);
  const int32_t r = upload_plan(p, blob, L);
  if (r != FEDAVG_OK) {
    delete p;
    return r;
  }
  p->split = 1;  // tile ranges are defined on the exact-order tiles
  *out = p;
  return FEDAVG_OK;
}

int32_t fedavg_plan_create_finalize(fedavg_ctx* c, const double* total_weights, void* const* out_ptrs,
                                    int32_t out_dtype, fedavg_plan** out) {
  FEDAVG_RET(check_ctx(c));
  if (!out) return fail(FEDAVG_ERR_INVALID, "null out");
  *out = nullptr;
  const int ok = out_kind_of(out_dtype);
  if (ok < 0) return fail(FEDAVG_ERR_INVALID, "out dtype must be FEDAVG_F32 or FEDAVG_F64");
  if (!out_ptrs || !total_weights) return fail(FEDAVG_ERR_INVALID, "null output table or total weights");
  for (int t = 0; t < c->T; ++t)
    if (!out_ptrs[t]) return fail(FEDAVG_ERR_INVALID, "null output pointer");
  FEDAVG_HIP_TRY(hipSetDevice(c->device));
  auto* p = new fedavg_plan();
  p->ctx = c;
  p->device = c->device;
  p->kind = fedavg_plan::FINALIZE;
  p->in_dtype = FEDAVG_F32;
  p->out_kind = ok;
  const BlobLayout L(c->T, 1);
  std::vector<int32_t> acc_in(c->T, 1);
  std::vector<char> blob;
  build_blob(c, nullptr, nullptr, 0, out_ptrs, total_weights, acc_in.data(), p->st, blob, L);
  const int32_t r = upload_plan(p, blob, L);
  if (r != FEDAVG_OK) {
    delete p;
    return r;
  }
  *out = p;
  return FEDAVG_OK;
}

int32_t fedavg_set_segment_state(fedavg_ctx* c, const double* total_weights, const int32_t* valid) {
  FEDAVG_RET(check_ctx(c));
  if (!valid) return fail(FEDAVG_ERR_INVALID, "null valid flags");
  for (int t = 0; t < c->T; ++t) {
    c->valid[t] = valid[t] ? 1 : 0;
    c->wsum[t] = (total_weights && valid[t]) ? total_weights[t] : -0.0;
  }
  return FEDAVG_OK;
}

int32_t fedavg_segment_state(const fedavg_ctx* c, double* total_weights, int32_t* valid) {
  FEDAVG_RET(check_ctx(c));
  for (int t = 0; t < c->T; ++t) {
    if (total_weights) total_weights[t] = c->wsum[t];
    if (valid) valid[t] = c->valid[t];
  }
  return FEDAVG_OK;
}

int32_t fedavg_accumulate_elementwise(fedavg_ctx* c, const void* const* client_ptrs, int32_t in_dtype,
                                      const void* const* weight_ptrs, const int32_t* weight_dtypes,
                                      const double* scalar_weights, const int32_t* total_fp32, int32_t K,
                                      void* totals, void* stream) {
  FEDAVG_RET(check_ctx(c));
  if (K < 0) return fail(FEDAVG_ERR_INVALID, "num_clients < 0");
  if (K == 0) return FEDAVG_OK;
  if (!client_ptrs || !weight_ptrs || !weight_dtypes || !scalar_weights || !total_fp32 || !totals)
    return fail(FEDAVG_ERR_INVALID, "null argument");
  if (in_dtype != FEDAVG_F32 && in_dtype != FEDAVG_F16 && in_dtype != FEDAVG_BF16 && in_dtype != FEDAVG_F64)
    return fail(FEDAVG_ERR_INVALID, "per-element weights take dense fp32 / fp16 / bf16 / fp64 inputs");
  const int T = c->T;
  for (int64_t i = 0; i < static_cast<int64_t>(K) * T; ++i)
    if (weight_ptrs[i] && weight_dtypes[i] != FEDAVG_F32 && weight_dtypes[i] != FEDAVG_F64)
      return fail(FEDAVG_ERR_INVALID, "per-element weights must be fp32 or fp64");
  FEDAVG_HIP_TRY(hipSetDevice(c->device));
  hipStream_t s = static_cast<hipStream_t>(stream);
  // segment-major compacted tables: x, w, ws, wdt ([T][K]), kseg, flags ([T])
  const size_t TK = static_cast<size_t>(T) * K;
  const size_t o_w = align_up(TK * 8, 16), o_ws = o_w + align_up(TK * 8, 16), o_wdt = o_ws + align_up(TK * 8, 16);
  const size_t o_k = o_wdt + align_up(TK * 4, 16), o_f = o_k + align_up(static_cast<size_t>(T) * 4, 16);
  std::vector<char> blob(o_f + align_up(static_cast<size_t>(T) * 4, 16), 0);
  auto* hx = reinterpret_cast<const void**>(blob.data());
  auto* hw = reinterpret_cast<const void**>(blob.data() + o_w);
  auto* hs = reinterpret_cast<double*>(blob.data() + o_ws);
  auto* hd = reinterpret_cast<int32_t*>(blob.data() + o_wdt);
  auto* hk = reinterpret_cast<int32_t*>(blob.data() + o_k);
  auto* hf = reinterpret_cast<int32_t*>(blob.data() + o_f);
  for (int t = 0; t < T; ++t) {
    int n = 0;
    for (int k = 0; k < K; ++k) {
      const size_t src = static_cast<size_t>(k) * T + t;
      if (!client_ptrs[src]) continue;
      const size_t dst = static_cast<size_t>(t) * K + n++;
      hx[dst] = client_ptrs[src];
      hw[dst] = weight_ptrs[src];
      hs[dst] = scalar_weights[src];
      hd[dst] = weight_dtypes[src];
    }
    hk[t] = n;
    hf[t] = (c->valid[t] ? 1 : 0) | (total_fp32[t] ? 2 : 0);
  }
  char* d = nullptr;
  FEDAVG_RET(aux_upload(c, s, blob, &d));
  EwArgs a;
  a.x = reinterpret_cast<const void* const*>(d);
  a.w = reinterpret_cast<const void* const*>(d + o_w);
  a.ws = reinterpret_cast<const double*>(d + o_ws);
  a.wdt = reinterpret_cast<const int32_t*>(d + o_wdt);
  a.kseg = reinterpret_cast<const int32_t*>(d + o_k);
  a.flags = reinterpret_cast<const int32_t*>(d + o_f);
  a.stride = K;
  a.acc = c->acc;
  a.tot = static_cast<double*>(totals);
  const dim3 grid(static_cast<unsigned>(c->tiles1.size())), block(kThreads);
  switch (in_dtype) {
    case FEDAVG_F32: hipLaunchKernelGGL(ew_fold_kernel<float>, grid, block, 0, s, c->d_tiles1, c->d_segs, a); break;
    case FEDAVG_F16: hipLaunchKernelGGL(ew_fold_kernel<__half>, grid, block, 0, s, c->d_tiles1, c->d_segs, a); break;
    case FEDAVG_BF16: hipLaunchKernelGGL(ew_fold_kernel<bf16_t>, grid, block, 0, s, c->d_tiles1, c->d_segs, a); break;
    default: hipLaunchKernelGGL(ew_fold_kernel<double>, grid, block, 0, s, c->d_tiles1, c->d_segs, a); break;
  }
  FEDAVG_HIP_TRY(hipGetLastError());
  for (int t = 0; t < T; ++t)
    if (hk[t] > 0) c->valid[t] = 1;
  return FEDAVG_OK;
}

int32_t fedavg_finalize_elementwise(fedavg_ctx* c, const void* totals, void* const* out_ptrs, int32_t out_dtype,
                                    void* stream) {
  FEDAVG_RET(check_ctx(c));
  const int ok = out_kind_of(out_dtype);
  if (ok < 0) return fail(FEDAVG_ERR_INVALID, "out dtype must be FEDAVG_F32 or FEDAVG_F64");
  if (!totals || !out_ptrs) return fail(FEDAVG_ERR_INVALID, "null argument");
  for (int t = 0; t < c->T; ++t) {
    if (!c->valid[t])
      return fail(FEDAVG_ERR_STATE, "segment " + std::to_string(t) + " has no accumulated data (fed_avg_algorithm.py:88)");
    if (!out_ptrs[t]) return fail(FEDAVG_ERR_INVALID, "null output pointer");
  }
  FEDAVG_HIP_TRY(hipSetDevice(c->device));
  hipStream_t s = static_cast<hipStream_t>(stream);
  std::vector<char> blob(align_up(sizeof(void*) * c->T, 16));
  std::memcpy(blob.data(), out_ptrs, sizeof(void*) * c->T);
  char* d = nullptr;
  FEDAVG_RET(aux_upload(c, s, blob, &d));
  const dim3 grid(static_cast<unsigned>(c->tiles1.size())), block(kThreads);
  const auto* tot = static_cast<const double*>(totals);
  auto* outs = reinterpret_cast<void* const*>(d);
  if (ok == OUT_F32)
    hipLaunchKernelGGL(ew_finalize_kernel<float>, grid, block, 0, s, c->d_tiles1, c->d_segs, c->acc, tot, outs, c->d_flag);
  else
    hipLaunchKernelGGL(ew_finalize_kernel<double>, grid, block, 0, s, c->d_tiles1, c->d_segs, c->acc, tot, outs, c->d_flag);
  FEDAVG_HIP_TRY(hipGetLastError());
  std::fill(c->wsum.begin(), c->wsum.end(), -0.0);
  std::fill(c->valid.begin(), c->valid.end(), 0);
  return FEDAVG_OK;
}

int64_t fedavg_layout_acc_numel(const int64_t* seg_numel, int32_t num_segments) {
  if (!seg_numel || num_segments <= 0) return -1;
  int64_t off = 0;
  for (int t = 0; t < num_segments; ++t) {
    if (seg_numel[t] <= 0) return -1;
    off += static_cast<int64_t>(align_up(static_cast<size_t>(seg_numel[t]), FEDAVG_ACC_ALIGN));
  }
  return off;
}

int32_t fedavg_plan_finalize_window(fedavg_plan* p, const double* src, int64_t lo, int64_t hi, void* res,
                                    void* stream) {
  if (!p || !p->ctx) return fail(FEDAVG_ERR_INVALID, "null plan");
  if (p->kind != fedavg_plan::FINALIZE) return fail(FEDAVG_ERR_INVALID, "a finalize plan is required");
  fedavg_ctx* c = p->ctx;
  if (lo < 0 || hi < lo || hi > c->acc_numel) return fail(FEDAVG_ERR_INVALID, "bad accumulator window");
  if (hi == lo) return FEDAVG_OK;
  if (!src || !res) return fail(FEDAVG_ERR_INVALID, "null window buffer");
  FEDAVG_HIP_TRY(hipSetDevice(c->device));
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int64_t n = hi - lo;
  const int64_t per_block = static_cast<int64_t>(kThreads) * kWinElems;
  const dim3 grid(static_cast<unsigned>((n + per_block - 1) / per_block)), block(kThreads);
  if (p->out_kind == OUT_F32) {
    hipLaunchKernelGGL(window_finalize_kernel<float>, grid, block, 0, s, src, lo, n, c->d_segs, c->T,
                       p->st.tab.wtot, static_cast<float*>(res), c->d_flag);
  } else {
    hipLaunchKernelGGL(window_finalize_kernel<double>, grid, block, 0, s, src, lo, n, c->d_segs, c->T,
                       p->st.tab.wtot, static_cast<double*>(res), c->d_flag);
  }
  FEDAVG_HIP_TRY(hipGetLastError());
  return FEDAVG_OK;
}

int32_t fedavg_plan_copy_out(fedavg_plan* p, const void* res, void* stream) {
  if (!p || !p->ctx) return fail(FEDAVG_ERR_INVALID, "null plan");
  if (p->kind != fedavg_plan::FINALIZE) return fail(FEDAVG_ERR_INVALID, "a finalize plan is required");
  if (!res) return fail(FEDAVG_ERR_INVALID, "null result buffer");
  fedavg_ctx* c = p->ctx;
  FEDAVG_HIP_TRY(hipSetDevice(c->device));
  hipStream_t s = static_cast<hipStream_t>(stream);
  const dim3 grid(static_cast<unsigned>(c->tiles1.size())), block(kThreads);
  if (p->out_kind == OUT_F32) {
    hipLaunchKernelGGL(copy_out_kernel<float>, grid, block, 0, s, c->d_tiles1, c->d_segs,
                       static_cast<const float*>(res), p->st.tab.outs, c->d_flag);
  } else {
    hipLaunchKernelGGL(copy_out_kernel<double>, grid, block, 0, s, c->d_tiles1, c->d_segs,
                       static_cast<const double*>(res), p->st.tab.outs, c->d_flag);
  }
  FEDAVG_HIP_TRY(hipGetLastError());
  return FEDAVG_OK;
}

int32_t fedavg_plan_out_dtype(const fedavg_plan* p) {
  if (!p) return -1;
  if (p->out_kind == OUT_F32) return FEDAVG_F32;
  if (p->out_kind == OUT_F64) return FEDAVG_F64;
  return -1;
}

// Shared with sharded_comm.cpp: set the profiling flag, return the previous one (the sharded
// round times one chunk launch per round: per-launch markers inside its chunk pipeline would
// perturb what they measure).
__attribute__((visibility("hidden"))) int32_t fedavg_internal_set_prof(fedavg_ctx* c, int32_t on) {
  const int32_t old = c->prof ? 1 : 0;
  c->prof = on != 0;
  return old;
}

// Shared with sharded_comm.cpp: a range launch whose completion also completes *done_ev
// (attached to the kernel's dispatch; the profiling event replaces it when profiling is on).
__attribute__((visibility("hidden"))) int32_t fedavg_internal_plan_run_range(fedavg_plan* p, int32_t tb, int32_t te,
                                                                           void* stream, hipEvent_t* done_ev) {
  if (!p || !p->ctx) return fail(FEDAVG_ERR_INVALID, "null plan");
  if (p->kind == fedavg_plan::AGGREGATE) return fail(FEDAVG_ERR_INVALID, "aggregate plans run whole (fedavg_plan_run)");
  fedavg_ctx* c = p->ctx;
  const int32_t n = static_cast<int32_t>(c->tiles1.size());
  if (te < 0) te = n;
  if (tb < 0 || tb > te || te > n) return fail(FEDAVG_ERR_INVALID, "bad tile range");
  FEDAVG_HIP_TRY(hipSetDevice(c->device));
  return launch_main(c, static_cast<hipStream_t>(stream), p->st, p->in_dtype, p->out_kind, 1, p->zero_init, tb, te,
                     done_ev);
}

// Shared with multi_device.cpp: a zero-initialised partial plan's range launch that writes its fp64
// partial into `acc_out` (accumulator coordinates; a peer device's receive slot) instead of the
// context's accumulator. `done_ev` (optional) completes with the kernel.
__attribute__((visibility("hidden"))) int32_t fedavg_internal_plan_run_range_to(fedavg_plan* p, int32_t tb, int32_t te,
                                                                              void* stream, double* acc_out) {
  if (!p || !p->ctx) return fail(FEDAVG_ERR_INVALID, "null plan");
  if (p->kind != fedavg_plan::PARTIAL || !p->zero_init)
    return fail(FEDAVG_ERR_INVALID, "the multi-device exchange takes zero-initialised partial plans");
  fedavg_ctx* c = p->ctx;
  const int32_t n = static_cast<int32_t>(c->tiles1.size());
  if (tb < 0 || tb > te || te > n) return fail(FEDAVG_ERR_INVALID, "bad tile range");
  FEDAVG_HIP_TRY(hipSetDevice(c->device));
  return launch_main(c, static_cast<hipStream_t>(stream), p->st, p->in_dtype, p->out_kind, 1, 1, tb, te, nullptr,
                     acc_out);
}

// Shared with multi_device.cpp: one launch of a zero-initialised dense partial plan over tiles
// [tb, te) whose tiles store into the window table's destinations (device tables: dst[n] slot
// pointers, edge[n + 1] absolute tile edges). FEDAVG_ERR_INVALID for record plans (the caller then
// launches window by window through fedavg_internal_plan_run_range_to).
__attribute__((visibility("hidden"))) int32_t fedavg_internal_plan_run_windows(fedavg_plan* p, int32_t tb, int32_t te,
                                                                             void* stream, double* const* dst,
                                                                             const int32_t* edge, int32_t n) {
  if (!p || !p->ctx) return fail(FEDAVG_ERR_INVALID, "null plan");
  if (p->kind != fedavg_plan::PARTIAL || !p->zero_init)
    return fail(FEDAVG_ERR_INVALID, "the multi-device exchange takes zero-initialised partial plans");
  if (is_record(p->in_dtype)) return fail(FEDAVG_ERR_INVALID, "windowed launches take dense inputs");
  fedavg_ctx* c = p->ctx;
  const int32_t nt = static_cast<int32_t>(c->tiles1.size());
  if (tb < 0 || tb > te || te > nt || n < 1) return fail(FEDAVG_ERR_INVALID, "bad tile range");
  FEDAVG_HIP_TRY(hipSetDevice(c->device));
  KArgs win{};
  win.win_dst = dst;
  win.win_edge = edge;
  win.win_n = n;
  return launch_main(c, static_cast<hipStream_t>(stream), p->st, p->in_dtype, p->out_kind, 1, 1, tb, te, nullptr,
                     nullptr, &win);
}
// Shared with multi_device.cpp: the own window of the peer exchange. Plan p's clients are folded
// over tiles [tb, te) from -0.0 and, per element, summed in entry order with the other entries'
// partials (comb_src: a device array of comb_n slot pointers, this entry at comb_self), divided
// by totals[seg] and stored into outs[seg] (host tables of T entries; copied into the plan's own
// table blob when they change) — fed_avg_algorithm.py:43-64 then :71-97 for this window.
__attribute__((visibility("hidden"))) int32_t fedavg_internal_plan_run_comb(fedavg_plan* p, int32_t tb, int32_t te,
                                                                          void* stream, const double* const* comb_src,
                                                                          int32_t comb_n, int32_t comb_self,
                                                                          const double* totals, void* const* outs,
                                                                          int32_t out_dtype) {
  if (!p || !p->ctx) return fail(FEDAVG_ERR_INVALID, "null plan");
  if (p->kind != fedavg_plan::PARTIAL || !p->zero_init)
    return fail(FEDAVG_ERR_INVALID, "the multi-device exchange takes zero-initialised partial plans");
  if (is_record(p->in_dtype) || p->st.delta) return fail(FEDAVG_ERR_INVALID, "the own-window combine takes dense folds");
  const int ok = out_kind_of(out_dtype);
  if (ok < 0) return fail(FEDAVG_ERR_INVALID, "out dtype must be FEDAVG_F32 or FEDAVG_F64");
  if (comb_n < 1 || comb_self < 0 || comb_self >= comb_n || !comb_src || !totals || !outs)
    return fail(FEDAVG_ERR_INVALID, "bad combine table");
  fedavg_ctx* c = p->ctx;
  const int32_t nt = static_cast<int32_t>(c->tiles1.size());
  if (tb < 0 || tb > te || te > nt) return fail(FEDAVG_ERR_INVALID, "bad tile range");
  FEDAVG_HIP_TRY(hipSetDevice(c->device));
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int T = c->T;
  // the plan blob's totals / outputs sections (a partial plan leaves them 1.0 / NULL)
  const BlobLayout L(T, std::max(p->st.stride, 1));
  std::vector<char> img(sizeof(double) * T + sizeof(void*) * T);
  std::memcpy(img.data(), totals, sizeof(double) * T);
  std::memcpy(img.data() + sizeof(double) * T, outs, sizeof(void*) * T);
  bool outs16 = true;
  for (int t = 0; t < T; ++t) {
    if (!outs[t]) return fail(FEDAVG_ERR_INVALID, "null output pointer");
    if (reinterpret_cast<uintptr_t>(outs[t]) % 16) outs16 = false;
  }
  if (p->fin_img != img) {
    FEDAVG_HIP_TRY(hipStreamSynchronize(s));  // an earlier combine on this stream may read the old tables
    FEDAVG_HIP_TRY(hipMemcpy(p->dev + L.off_wtot, img.data(), sizeof(double) * T, hipMemcpyHostToDevice));
    FEDAVG_HIP_TRY(hipMemcpy(p->dev + L.off_outs, img.data() + sizeof(double) * T, sizeof(void*) * T,
                             hipMemcpyHostToDevice));
    p->fin_img = img;
  }
  Staged st = p->st;
  st.aligned = st.aligned && outs16;
  KArgs comb{};
  comb.comb_src = comb_src;
  comb.comb_n = comb_n;
  comb.comb_self = comb_self;
  return launch_main(c, s, st, p->in_dtype, ok, 1, 1, tb, te, nullptr, nullptr, nullptr, &comb);
}

__attribute__((visibility("hidden"))) int32_t fedavg_internal_plan_is_record(const fedavg_plan* p) {
  return (p && is_record(p->in_dtype)) ? 1 : 0;
}

// Shared with multi_device.cpp: the device-ordered sum of G fp64 partials over tiles [tb, te) of
// the context's exact-order table, divided by wtot[seg] into outs[seg] (device tables of the
// launching device), NaN flags into the context's words.
__attribute__((visibility("hidden"))) int32_t fedavg_internal_multi_combine(fedavg_ctx* c, int32_t tb, int32_t te,
                                                                          const double* const* slots, int32_t G,
                                                                          const double* wtot, void* const* outs,
                                                                          int32_t out_dtype, int32_t vec, void* stream) {
  if (!c) return fail(FEDAVG_ERR_INVALID, "null context");
  if (G < 1 || G > kMaxDevices) return fail(FEDAVG_ERR_INVALID, "1 to 16 partials per combine");
  const int32_t n = static_cast<int32_t>(c->tiles1.size());
  if (tb < 0 || tb > te || te > n) return fail(FEDAVG_ERR_INVALID, "bad tile range");
  if (tb == te) return FEDAVG_OK;
  SlotPtrs sp{};
  for (int32_t g = 0; g < G; ++g) {
    if (!slots[g] || reinterpret_cast<uintptr_t>(slots[g]) % 16)
      return fail(FEDAVG_ERR_INVALID, "partial buffers must be 16-byte aligned");
    sp.p[g] = slots[g];
  }
  FEDAVG_HIP_TRY(hipSetDevice(c->device));
  hipStream_t s = static_cast<hipStream_t>(stream);
  const dim3 grid(static_cast<unsigned>(te - tb)), block(kThreads);
  if (out_dtype == FEDAVG_F32) {
    if (vec) hipLaunchKernelGGL((multi_combine_kernel<float, true>), grid, block, 0, s, c->d_tiles1, tb, c->d_segs, sp, G, wtot, outs, c->d_flag);
    else hipLaunchKernelGGL((multi_combine_kernel<float, false>), grid, block, 0, s, c->d_tiles1, tb, c->d_segs, sp, G, wtot, outs, c->d_flag);
  } else if (out_dtype == FEDAVG_F64) {
    if (vec) hipLaunchKernelGGL((multi_combine_kernel<double, true>), grid, block, 0, s, c->d_tiles1, tb, c->d_segs, sp, G, wtot, outs, c->d_flag);
    else hipLaunchKernelGGL((multi_combine_kernel<double, false>), grid, block, 0, s, c->d_tiles1, tb, c->d_segs, sp, G, wtot, outs, c->d_flag);
  } else {
    return fail(FEDAVG_ERR_INVALID, "out dtype must be FEDAVG_F32 or FEDAVG_F64");
  }
  FEDAVG_HIP_TRY(hipGetLastError());
  return FEDAVG_OK;
}

// Shared with multi_device.cpp: per-segment "accumulator holds data" flags (out[T]), the tile
// range [*tb, *te) of one segment, and the host state reset of a finished round.
__attribute__((visibility("hidden"))) int32_t fedavg_internal_segment_valid(const fedavg_ctx* c, int32_t* out) {
  if (!c || !out) return fail(FEDAVG_ERR_INVALID, "null argument");
  for (int t = 0; t < c->T; ++t) out[t] = c->valid[t];
  return FEDAVG_OK;
}
__attribute__((visibility("hidden"))) int32_t fedavg_internal_segment_tiles(const fedavg_ctx* c, int32_t seg,
                                                                          int32_t* tb, int32_t* te) {
  if (!c || seg < 0 || seg >= c->T || !tb || !te) return fail(FEDAVG_ERR_INVALID, "bad segment");
  int32_t b = -1, e = -1;
  for (int32_t i = 0; i < static_cast<int32_t>(c->tiles1.size()); ++i)
    if (c->tiles1[i].seg == seg) {
      if (b < 0) b = i;
      e = i + 1;
    }
  *tb = b;
  *te = e;
  return FEDAVG_OK;
}
__attribute__((visibility("hidden"))) void fedavg_internal_clear_state(fedavg_ctx* c) {
  std::fill(c->wsum.begin(), c->wsum.end(), -0.0);
  std::fill(c->valid.begin(), c->valid.end(), 0);
}
__attribute__((visibility("hidden"))) uint32_t fedavg_internal_flags(fedavg_ctx* c, int32_t clear) {
  const uint32_t f = (__atomic_load_n(&c->h_flag[0], __ATOMIC_ACQUIRE) ? FEDAVG_FLAG_ACC_NAN : 0u) |
                     (__atomic_load_n(&c->h_flag[1], __ATOMIC_ACQUIRE) ? FEDAVG_FLAG_RESULT_NAN : 0u);
  if (clear)
    for (int i = 0; i < 4; ++i) __atomic_store_n(&c->h_flag[i], 0u, __ATOMIC_RELEASE);
  return f;
}

int32_t fedavg_plan_run_range(fedavg_plan* p, int32_t tb, int32_t te, void* stream) {
  if (!p || !p->ctx) return fail(FEDAVG_ERR_INVALID, "null plan");
  if (p->kind == fedavg_plan::AGGREGATE) return fail(FEDAVG_ERR_INVALID, "aggregate plans run whole (fedavg_plan_run)");
  fedavg_ctx* c = p->ctx;
  const int32_t n = static_cast<int32_t>(c->tiles1.size());
  if (te < 0) te = n;
  if (tb < 0 || tb > te || te > n) return fail(FEDAVG_ERR_INVALID, "bad tile range");
  FEDAVG_HIP_TRY(hipSetDevice(c->device));
  return launch_main(c, static_cast<hipStream_t>(stream), p->st, p->in_dtype, p->out_kind, 1, p->zero_init, tb, te);
}

int32_t fedavg_plan_run(fedavg_plan* p, void* stream) {
  if (!p || !p->ctx) return fail(FEDAVG_ERR_INVALID, "null plan");
  if (p->kind != fedavg_plan::AGGREGATE) return fedavg_plan_run_range(p, 0, -1, stream);
  fedavg_ctx* c = p->ctx;
  for (int t = 0; t < c->T; ++t)
    if (c->valid[t]) return fail(FEDAVG_ERR_STATE, "plan run on a context holding accumulated data");
  FEDAVG_HIP_TRY(hipSetDevice(c->device));
  return launch_main(c, static_cast<hipStream_t>(stream), p->st, p->in_dtype, p->out_kind, p->split, 0, 0,
                     static_cast<int32_t>(c->tiles1.size()));
}

int32_t fedavg_plan_destroy(fedavg_plan* p) {
  if (!p) return FEDAVG_OK;
  int prev = -1;
  if (hipGetDevice(&prev) != hipSuccess) prev = -1;
  if (p->device >= 0) (void)hipSetDevice(p->device);
  (void)hipDeviceSynchronize();
  if (p->dev) (void)hipFree(p->dev);
  delete p;
  if (prev >= 0) (void)hipSetDevice(prev);
  return FEDAVG_OK;
}

int32_t fedavg_bw_probe(const void* src, int64_t bytes, void* dst, int32_t mode, void* stream) {
  if (!src || !dst || bytes <= 0 || bytes % 16 != 0) return fail(FEDAVG_ERR_INVALID, "bad probe args");
  if (reinterpret_cast<uintptr_t>(src) % 16 || reinterpret_cast<uintptr_t>(dst) % 16)
    return fail(FEDAVG_ERR_INVALID, "probe buffers must be 16-byte aligned");
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int64_t n = bytes / 16;
  const int blocks = 256 * 8;
  if (mode == 0) {
    hipLaunchKernelGGL(bw_copy_kernel, dim3(blocks), dim3(kThreads), 0, s, static_cast<const f32x4*>(src),
                       static_cast<f32x4*>(dst), n);
  } else {
    hipLaunchKernelGGL(bw_read_kernel, dim3(blocks), dim3(kThreads), 0, s, static_cast<const f32x4*>(src),
                       static_cast<uint32_t*>(dst), n);
  }
  FEDAVG_HIP_TRY(hipGetLastError());
  return FEDAVG_OK;
}

}  // extern "C"

// ---- dynamic waves (dyn_wave_kernel) ------------------------------------------------------
namespace {

uint64_t dyn_env_us(const char* name, uint64_t dflt) {
  const char* v = std::getenv(name);
  return (v && *v) ? std::strtoull(v, nullptr, 10) : dflt;
}

// wave epochs, unique in the process: a mirror word left in recycled device memory by another
// context's wave never matches a live one
std::atomic<uint32_t> g_dyn_epoch{0};

// FEDAVG_DYN_TRACE=1: the host time of each step of fedavg_dyn_open / _close on stderr
struct DynTrace {
  bool on;
  const char* what;
  std::chrono::steady_clock::time_point t0, last;
  char buf[256];
  int len = 0;
  explicit DynTrace(const char* w) : on(enabled()), what(w) { t0 = last = std::chrono::steady_clock::now(); }
  static bool enabled() {
    static const bool e = [] { const char* v = std::getenv("FEDAVG_DYN_TRACE"); return v && *v == '1'; }();
    return e;
  }
  void mark(const char* step) {
    if (!on || len > 200) return;
    const auto now = std::chrono::steady_clock::now();
    len += std::snprintf(buf + len, sizeof(buf) - len, " %s=%.1f", step,
                         std::chrono::duration<double, std::micro>(now - last).count());
    last = now;
  }
  ~DynTrace() {
    if (on)
      std::fprintf(stderr, "[dyn %s] total=%.1f us%s\n", what,
                   std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count(), buf);
  }
};

int32_t dyn_wait_ack(fedavg_ctx* c, uint32_t* state, uint32_t* count) {
  auto& d = c->dyn;
  const DynLayout L(c->T, d.cap);
  const DynAck* ack = reinterpret_cast<const DynAck*>(d.host + L.ack);
  // the mirror answers within a poll (~1 µs); a wave whose mirror never runs is ended by its
  // own lifetime limit, so this wait is bounded by that (plus a margin)
  const auto t0 = std::chrono::steady_clock::now();
  const double limit_s = static_cast<double>(d.life_ticks) / 1e8 + 5.0;
  for (;;) {
    const uint64_t aw = __atomic_load_n(&ack->word, __ATOMIC_ACQUIRE);
    const uint32_t st = static_cast<uint32_t>(aw);
    if (st != 0) {
      *state = st;
      *count = static_cast<uint32_t>(aw >> 32);
      return FEDAVG_OK;
    }
    if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > limit_s) {
      // the context recovers: the wave is no longer open, the accumulator holds nothing valid, and
      // the next open waits for the wave's launches (their tiles end themselves after life + 1 s)
      d.active = false;
      d.unjoined = false;
      std::fill(c->valid.begin(), c->valid.end(), 0);
      (void)hipEventRecord(d.done, d.stream);
      if (!d.edge_tiles.empty()) (void)hipEventRecord(d.edge_done, d.edge_stream);
      return fail(FEDAVG_ERR_HIP, "the dynamic wave did not acknowledge its close (the wave is abandoned)");
    }
#if defined(__x86_64__)
    __builtin_ia32_pause();
#endif
  }
}

// The wave's two launches on the private streams: the body tiles, then the edge tiles, each led by
// a mirror candidate workgroup (dyn_elect). `resume`: the accumulators start from the fp64
// accumulator (a wave continuing the round after an earlier one ended itself).
int32_t dyn_launch(fedavg_ctx* c, int32_t resume) {
  auto& d = c->dyn;
  const DynLayout L(c->T, d.cap);
  d.epoch = g_dyn_epoch.fetch_add(1) + 1;
  if (d.epoch == 0) d.epoch = g_dyn_epoch.fetch_add(1) + 1;
  DynArgs a{};
  a.tiles = d.d_tiles;
  a.edge_tiles = d.d_edge_tiles;
  a.segs = c->d_segs;
  a.acc = c->acc;
  a.flag = c->d_flag;
  a.ctl = reinterpret_cast<DynCtl*>(d.dev_alias + L.ctl);
  a.ack = reinterpret_cast<DynAck*>(d.dev_alias + L.ack);
  a.h_wtot = reinterpret_cast<const double*>(d.dev_alias + L.wtot);
  a.h_outs = reinterpret_cast<const uint64_t*>(d.dev_alias + L.outs);
  a.h_wtab = reinterpret_cast<const double*>(d.dev_alias + L.wtab);
  a.h_ptab = reinterpret_cast<const uint64_t*>(d.dev_alias + L.ptab);
  a.wtot = reinterpret_cast<double*>(d.dtab + L.wtot);
  a.outs = reinterpret_cast<uint64_t*>(d.dtab + L.outs);
  a.wtab = reinterpret_cast<double*>(d.dtab + L.wtab);
  a.ptab = reinterpret_cast<uint64_t*>(d.dtab + L.ptab);
  a.mir = reinterpret_cast<DynMirror*>(d.mirror);
  a.elect = reinterpret_cast<uint32_t*>(d.mirror + sizeof(DynMirror) * kDynCopies);
  a.edge_base = static_cast<int32_t>(d.tiles.size());
  a.tend = nullptr;
  if (c->prof) {
    if (!d.tend) FEDAVG_HIP_TRY(hipMalloc(reinterpret_cast<void**>(&d.tend), sizeof(uint64_t) * (d.tiles.size() + d.edge_tiles.size())));
    a.tend = d.tend;
  }
  d.timed = c->prof;
  a.num_tiles = static_cast<int32_t>(d.tiles.size());
  a.num_segs = c->T;
  a.cap = d.cap;
  a.epoch = d.epoch;
  a.idle_ticks = d.idle_ticks;
  a.life_ticks = d.life_ticks;
  a.resume = resume;
  d.prof_start = nullptr;
  if (c->prof) {  // the body launch timed from its enqueue to its end (arrivals included)
    d.prof_start = take_event(c);
    if (!d.prof_start) return fail(FEDAVG_ERR_HIP, "hipEventCreate failed");
    FEDAVG_HIP_TRY(hipEventRecord(d.prof_start, d.stream));
  }
  const dim3 grid(static_cast<unsigned>(a.num_tiles + 1)), block(kDynLanes);
  switch (d.in_dtype) {
    case FEDAVG_F32: hipLaunchKernelGGL((dyn_wave_kernel<float, false>), grid, block, 0, d.stream, a); break;
    case FEDAVG_F16: hipLaunchKernelGGL((dyn_wave_kernel<__half, false>), grid, block, 0, d.stream, a); break;
    case FEDAVG_BF16: hipLaunchKernelGGL((dyn_wave_kernel<bf16_t, false>), grid, block, 0, d.stream, a); break;
    default: hipLaunchKernelGGL((dyn_wave_kernel<double, false>), grid, block, 0, d.stream, a); break;
  }
  FEDAVG_HIP_TRY(hipGetLastError());
  if (!d.edge_tiles.empty()) {
    const dim3 egrid(static_cast<unsigned>(d.edge_tiles.size() + 1));
    switch (d.in_dtype) {
      case FEDAVG_F32: hipLaunchKernelGGL((dyn_wave_kernel<float, true>), egrid, block, 0, d.edge_stream, a); break;
      case FEDAVG_F16: hipLaunchKernelGGL((dyn_wave_kernel<__half, true>), egrid, block, 0, d.edge_stream, a); break;
      case FEDAVG_BF16: hipLaunchKernelGGL((dyn_wave_kernel<bf16_t, true>), egrid, block, 0, d.edge_stream, a); break;
      default: hipLaunchKernelGGL((dyn_wave_kernel<double, true>), egrid, block, 0, d.edge_stream, a); break;
    }
  }
  FEDAVG_HIP_TRY(hipGetLastError());
  ++d.launches;
  return FEDAVG_OK;
}

// The open wave ended itself (FEDAVG_DYN_IDLE_US without a row, or FEDAVG_DYN_LIFE_US): its
// accumulator close stored rows [base, base + folded). A fresh wave continues the round from that
// accumulator — the reference server's poll loop (server.py:133-146) hands updates over in bursts
// with a sleep between them, and a burst after the idle limit is folded while it arrives instead
// of in one launch at aggregate_worker_data. Rows published to the ended wave after it stopped
// reading are moved to the front of the new wave's table.
int32_t dyn_continue(fedavg_ctx* c) {
  auto& d = c->dyn;
  DynTrace tr("reopen");
  const int T = c->T;
  const DynLayout L(T, d.cap);
  DynCtl* ctl = reinterpret_cast<DynCtl*>(d.host + L.ctl);
  DynAck* ack = reinterpret_cast<DynAck*>(d.host + L.ack);
  const uint64_t aw = __atomic_load_n(&ack->word, __ATOMIC_ACQUIRE);
  const int32_t folded = static_cast<int32_t>(aw >> 32);
  FEDAVG_HIP_TRY(hipSetDevice(c->device));
  // the ended wave's launches read the device table and write the accumulator: both finished
  // before the next mirror rewrites the table and the next tiles read the accumulator (the usual
  // case — the burst comes after the idle limit — finds them long done)
  FEDAVG_HIP_TRY(hipEventRecord(d.done, d.stream));
  if (!d.edge_tiles.empty()) FEDAVG_HIP_TRY(hipEventRecord(d.edge_done, d.edge_stream));
  if (hipEventQuery(d.done) != hipSuccess) FEDAVG_HIP_TRY(hipEventSynchronize(d.done));
  if (!d.edge_tiles.empty() && hipEventQuery(d.edge_done) != hipSuccess) FEDAVG_HIP_TRY(hipEventSynchronize(d.edge_done));
  tr.mark("prev");
  if (__atomic_load_n(&ack->error, __ATOMIC_ACQUIRE)) {
    d.active = false;
    std::fill(c->valid.begin(), c->valid.end(), 0);
    return fail(FEDAVG_ERR_HIP, "a dynamic wave's workgroup lost its mirror (the wave's results are invalid)");
  }
  if (d.prof_start) {
    hipEvent_t stop = take_event(c);
    if (!stop) return fail(FEDAVG_ERR_HIP, "hipEventCreate failed");
    FEDAVG_HIP_TRY(hipEventRecord(stop, d.stream));
    d.prof.emplace_back(d.prof_start, stop);
    d.prof_start = nullptr;
  }
  double* wtab = reinterpret_cast<double*>(d.host + L.wtab);
  uint64_t* ptab = reinterpret_cast<uint64_t*>(d.host + L.ptab);
  for (int t = 0; t < T; ++t)
    for (int32_t k = 0; k < folded; ++k) d.wsum_base[t] += wtab[k];  // fed_avg_algorithm.py:59-62, arrival order
  const int32_t left = d.published - d.base - folded;
  if (left > 0 && folded > 0) {
    std::memmove(wtab, wtab + folded, sizeof(double) * left);
    for (int t = 0; t < T; ++t)
      std::memmove(ptab + static_cast<int64_t>(t) * d.cap, ptab + static_cast<int64_t>(t) * d.cap + folded,
                   sizeof(uint64_t) * left);
  }
  d.base += folded;
  __atomic_store_n(&ack->word, uint64_t{0}, __ATOMIC_RELAXED);
  __atomic_store_n(&ack->t_rows, uint64_t{0}, __ATOMIC_RELAXED);
  __atomic_store_n(&ack->error, 0u, __ATOMIC_RELAXED);
  __atomic_store_n(&ctl->word, dyn_word(static_cast<uint32_t>(left), 0u, OUT_ACC, 0u), __ATOMIC_RELEASE);
  ++d.reopens;
  tr.mark("table");
  // nothing folded yet (a wave opened ahead of its first row that idled out): a zero-initialised wave
  return dyn_launch(c, d.base > 0 ? 1 : 0);
}

}  // namespace

extern "C" {

int32_t fedavg_dyn_open(fedavg_ctx* c, int32_t in_dtype, int32_t max_clients, void* stream) {
  FEDAVG_RET(check_ctx(c));
  auto& d = c->dyn;
  if (d.active) return fail(FEDAVG_ERR_STATE, "a dynamic wave is already open");
  if (in_dtype != FEDAVG_F32 && in_dtype != FEDAVG_F16 && in_dtype != FEDAVG_BF16 && in_dtype != FEDAVG_F64)
    return fail(FEDAVG_ERR_INVALID, "dynamic waves take fp32 / fp16 / bf16 / fp64 inputs");
  if (max_clients < 1 || max_clients >= (1 << 24)) return fail(FEDAVG_ERR_INVALID, "max_clients must be in [1, 2^24)");
  for (int t = 0; t < c->T; ++t)
    if (c->valid[t]) return fail(FEDAVG_ERR_STATE, "a dynamic wave opens a round: the accumulator already holds data");
  DynTrace tr("open");
  FEDAVG_HIP_TRY(hipSetDevice(c->device));
  if (!d.stream) {
    FEDAVG_HIP_TRY(hipStreamCreateWithFlags(&d.stream, hipStreamNonBlocking));
    FEDAVG_HIP_TRY(hipStreamCreateWithFlags(&d.edge_stream, hipStreamNonBlocking));
    FEDAVG_HIP_TRY(hipEventCreateWithFlags(&d.edge_done, hipEventDisableTiming));
    FEDAVG_HIP_TRY(hipEventCreateWithFlags(&d.start, hipEventDisableTiming));
    FEDAVG_HIP_TRY(hipEventCreateWithFlags(&d.done, hipEventDisableTiming));
    // kDynCopies mirror words, then the election word (dyn_elect)
    const size_t mbytes = sizeof(DynMirror) * (kDynCopies + 1);
    FEDAVG_HIP_TRY(hipMalloc(reinterpret_cast<void**>(&d.mirror), mbytes));
    // epoch 0 is never a wave's; on the wave's own stream and waited for: a plain hipMemset
    // is not ordered before a launch on a non-blocking stream, and a recycled allocation may
    // hold another context's mirror words (epochs are process-wide besides: g_dyn_epoch)
    FEDAVG_HIP_TRY(hipMemsetAsync(d.mirror, 0, mbytes, d.stream));
    FEDAVG_HIP_TRY(hipStreamSynchronize(d.stream));
    for (int t = 0; t < c->T; ++t) {  // body tiles, then each segment's rest as edge tiles
      const int64_t n = c->seg_numel[t], body = n / kDynTile * kDynTile;
      for (int64_t s0 = 0; s0 < body; s0 += kDynTile) d.tiles.push_back(TileDesc{t, kDynTile, s0});
      for (int64_t s0 = body; s0 < n; s0 += kDynEdgeTile)
        d.edge_tiles.push_back(TileDesc{t, static_cast<int32_t>(std::min<int64_t>(kDynEdgeTile, n - s0)), s0});
    }
    for (auto [host, dev] : {std::pair{&d.tiles, &d.d_tiles}, std::pair{&d.edge_tiles, &d.d_edge_tiles}}) {
      if (host->empty()) continue;
      FEDAVG_HIP_TRY(hipMalloc(reinterpret_cast<void**>(dev), sizeof(TileDesc) * host->size()));
      FEDAVG_HIP_TRY(hipMemcpy(*dev, host->data(), sizeof(TileDesc) * host->size(), hipMemcpyHostToDevice));
    }
    if (!d.idle_ticks) d.idle_ticks = dyn_env_us("FEDAVG_DYN_IDLE_US", 200) * 100;  // s_memrealtime: 100 MHz
    if (!d.life_ticks) d.life_ticks = dyn_env_us("FEDAVG_DYN_LIFE_US", 2000000) * 100;
  }
  if (d.cap < max_clients) {
    FEDAVG_HIP_TRY(hipStreamSynchronize(d.stream));  // the previous wave has left the old block
    FEDAVG_HIP_TRY(hipStreamSynchronize(d.edge_stream));
    if (d.host) FEDAVG_HIP_TRY(hipHostFree(d.host));
    if (d.dtab) FEDAVG_HIP_TRY(hipFree(d.dtab));
    d.host = nullptr;
    d.dtab = nullptr;
    d.cap = 0;
    const int cap = std::max(max_clients, 64);
    const DynLayout L(c->T, cap);
    FEDAVG_HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&d.host), L.bytes, hipHostMallocMapped | hipHostMallocCoherent));
    FEDAVG_HIP_TRY(hipMalloc(reinterpret_cast<void**>(&d.dtab), L.bytes));
    FEDAVG_HIP_TRY(hipHostGetDevicePointer(reinterpret_cast<void**>(&d.dev_alias), d.host, 0));
    d.cap = cap;
    d.bytes = L.bytes;
  }
  // the previous wave read its block to the end (its launches' completion events, recorded at its
  // close; an event never recorded reads as complete)
  tr.mark("setup");
  if (hipEventQuery(d.done) != hipSuccess) FEDAVG_HIP_TRY(hipStreamSynchronize(d.stream));
  if (hipEventQuery(d.edge_done) != hipSuccess) FEDAVG_HIP_TRY(hipStreamSynchronize(d.edge_stream));
  tr.mark("prev");
  const DynLayout L(c->T, d.cap);
  DynCtl* ctl = reinterpret_cast<DynCtl*>(d.host + L.ctl);
  DynAck* ack = reinterpret_cast<DynAck*>(d.host + L.ack);
  __atomic_store_n(&ctl->word, dyn_word(0u, 0u, OUT_ACC, 0u), __ATOMIC_RELAXED);
  __atomic_store_n(&ack->word, uint64_t{0}, __ATOMIC_RELAXED);
  __atomic_store_n(&ack->t_rows, uint64_t{0}, __ATOMIC_RELAXED);
  __atomic_store_n(&ack->error, 0u, __ATOMIC_RELEASE);
  d.wsum.assign(c->T, -0.0);
  d.wsum_base.assign(c->T, -0.0);
  d.published = 0;
  d.base = 0;
  d.in_dtype = in_dtype;
  // the wave starts behind the caller's stream (what it enqueued so far), on the private stream;
  // an idle caller's stream (the usual case: the previous round ended on the host) needs no
  // cross-stream dependency, which costs two queue packets and ~40 us before the launch starts
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (!stream_idle(s)) {
    FEDAVG_HIP_TRY(hipEventRecord(d.start, s));
    FEDAVG_HIP_TRY(hipStreamWaitEvent(d.stream, d.start, 0));
    FEDAVG_HIP_TRY(hipStreamWaitEvent(d.edge_stream, d.start, 0));
    tr.mark("dep");
  } else {
    tr.mark("query");
  }
  FEDAVG_RET(dyn_launch(c, 0));
  tr.mark("launch");
  d.active = true;
  return FEDAVG_OK;
}

int32_t fedavg_dyn_publish(fedavg_ctx* c, const void* const* client_ptrs, const double* weights, int32_t K,
                           void* stream, int32_t* published_out) {
  FEDAVG_RET(check_ctx(c));
  auto& d = c->dyn;
  if (published_out) *published_out = 0;
  if (!d.active) return fail(FEDAVG_ERR_STATE, "no dynamic wave is open");
  if (K < d.published || K - d.base > d.cap) return fail(FEDAVG_ERR_INVALID, "row count outside the wave's table");
  if (K == d.published) return FEDAVG_OK;
  const int T = c->T;
  // rows the wave can take: every tensor present, 16-B aligned, one weight per row; the rows
  // before the first one it cannot take are still published, then FEDAVG_ERR_INVALID
  int good = K;
  for (int k = d.published; k < K && good == K; ++k) {
    const double w = weights[static_cast<int64_t>(k) * T];
    for (int t = 0; t < T; ++t) {
      const void* p = client_ptrs[static_cast<int64_t>(k) * T + t];
      const double wt = weights[static_cast<int64_t>(k) * T + t];
      if (!p || reinterpret_cast<uintptr_t>(p) % 16 != 0 || std::memcmp(&wt, &w, sizeof(double)) != 0) {
        good = k;
        break;
      }
    }
  }
  // the caller's stream must have finished what it enqueued: the arrivals' tensors are then
  // complete (the wave runs on its own stream); otherwise nothing is published now
  if (good > d.published && hipStreamQuery(static_cast<hipStream_t>(stream)) == hipSuccess) {
    const DynLayout L(T, d.cap);
    const DynAck* ack = reinterpret_cast<const DynAck*>(d.host + L.ack);
    if (static_cast<uint32_t>(__atomic_load_n(&ack->word, __ATOMIC_ACQUIRE)) != 0)
      FEDAVG_RET(dyn_continue(c));  // the wave ended itself: a fresh one continues the round
    uint64_t* ptab = reinterpret_cast<uint64_t*>(d.host + L.ptab);
    double* wtab = reinterpret_cast<double*>(d.host + L.wtab);
    for (int k = d.published; k < good; ++k) {
      const double w = weights[static_cast<int64_t>(k) * T];
      const int r = k - d.base;  // the row's place in the current wave's table
      wtab[r] = w;
      for (int t = 0; t < T; ++t) {
        ptab[static_cast<int64_t>(t) * d.cap + r] =
            reinterpret_cast<uint64_t>(client_ptrs[static_cast<int64_t>(k) * T + t]);
        d.wsum[t] += w;  // fed_avg_algorithm.py:59-62, arrival order
      }
    }
    DynCtl* ctl = reinterpret_cast<DynCtl*>(d.host + L.ctl);
    __atomic_store_n(&ctl->word, dyn_word(static_cast<uint32_t>(good - d.base), 0u, OUT_ACC, 0u), __ATOMIC_RELEASE);
    if (published_out) *published_out = good - d.published;
    d.published = good;
  } else if (good == K) {
    return FEDAVG_OK;  // nothing published now (the stream is busy)
  }
  if (good < K)
    return fail(FEDAVG_ERR_INVALID, "a row the dynamic wave cannot take (absent / unaligned tensor, per-tensor weights)");
  return FEDAVG_OK;
}

int32_t fedavg_dyn_close(fedavg_ctx* c, void* const* out_ptrs, int32_t out_dtype, int32_t join, void* stream,
                         int32_t* folded_out, int32_t* finalized_out) {
  FEDAVG_RET(check_ctx(c));
  auto& d = c->dyn;
  if (!d.active) return fail(FEDAVG_ERR_STATE, "no dynamic wave is open");
  DynTrace tr("close");
  const int T = c->T;
  const DynLayout L(T, d.cap);
  DynCtl* ctl = reinterpret_cast<DynCtl*>(d.host + L.ctl);
  uint32_t mode = OUT_ACC;
  if (out_ptrs && d.published > 0) {
    const int ok = out_kind_of(out_dtype);
    if (ok < 0) return fail(FEDAVG_ERR_INVALID, "out dtype must be FEDAVG_F32 or FEDAVG_F64");
    bool aligned = true;
    for (int t = 0; t < T; ++t) aligned = aligned && out_ptrs[t] && reinterpret_cast<uintptr_t>(out_ptrs[t]) % 16 == 0;
    if (aligned) {  // (unaligned outputs: the wave stores the accumulator, the caller divides)
      double* wtot = reinterpret_cast<double*>(d.host + L.wtot);
      uint64_t* outs = reinterpret_cast<uint64_t*>(d.host + L.outs);
      for (int t = 0; t < T; ++t) {
        wtot[t] = d.wsum[t];
        outs[t] = reinterpret_cast<uint64_t>(out_ptrs[t]);
      }
      mode = static_cast<uint32_t>(ok);
    }
  }
  __atomic_store_n(&ctl->word, dyn_word(static_cast<uint32_t>(d.published - d.base), 1u, mode, 0u), __ATOMIC_RELEASE);
  uint32_t state = 0, folded = 0;
  tr.mark("ctl");
  FEDAVG_RET(dyn_wait_ack(c, &state, &folded));
  tr.mark("ack");
  d.active = false;
  FEDAVG_HIP_TRY(hipSetDevice(c->device));
  // an accumulator close always joins `stream` (the ordinary calls continue from the accumulator)
  const bool joined = join || !(state == 1 && mode != OUT_ACC);
  if (d.prof_start) {
    hipEvent_t stop = take_event(c);
    if (!stop) return fail(FEDAVG_ERR_HIP, "hipEventCreate failed");
    FEDAVG_HIP_TRY(hipEventRecord(stop, d.stream));
    d.prof.emplace_back(d.prof_start, stop);
    d.prof_start = nullptr;
  }
  FEDAVG_HIP_TRY(hipEventRecord(d.done, d.stream));
  if (joined) FEDAVG_HIP_TRY(hipStreamWaitEvent(static_cast<hipStream_t>(stream), d.done, 0));
  if (!d.edge_tiles.empty()) {
    FEDAVG_HIP_TRY(hipEventRecord(d.edge_done, d.edge_stream));
    if (joined) FEDAVG_HIP_TRY(hipStreamWaitEvent(static_cast<hipStream_t>(stream), d.edge_done, 0));
  }
  d.unjoined = !joined;
  tr.mark("events");
  if (tr.on) {
    const DynAck* ak = reinterpret_cast<const DynAck*>(d.host + L.ack);
    tr.len += std::snprintf(tr.buf + tr.len, sizeof(tr.buf) - tr.len, " gpu_seen_to_ack=%.1f polls=%u reopens=%d",
                            static_cast<double>(ak->t_done - ak->t_seen) / 100.0, ak->polls, d.reopens);
  }
  const DynAck* ack = reinterpret_cast<const DynAck*>(d.host + L.ack);
  if (__atomic_load_n(&ack->error, __ATOMIC_ACQUIRE)) {
    FEDAVG_HIP_TRY(hipStreamSynchronize(d.stream));
    FEDAVG_HIP_TRY(hipStreamSynchronize(d.edge_stream));
    std::fill(c->valid.begin(), c->valid.end(), 0);
    return fail(FEDAVG_ERR_HIP, "a dynamic wave's workgroup lost its mirror (the wave's results are invalid)");
  }
  const bool finalized = state == 1 && mode != OUT_ACC;
  const int32_t total = d.base + static_cast<int32_t>(folded);  // rows of the round in the accumulator
  if (finalized) {
    fedavg_internal_clear_state(c);  // the round's result is written (fed_avg_algorithm.py:90,98)
  } else if (total > 0) {
    // the accumulator holds rows [0, total): their totals, in arrival order
    const double* wtab = reinterpret_cast<const double*>(d.host + L.wtab);
    for (int t = 0; t < T; ++t) {
      double s = d.wsum_base[t];
      for (uint32_t k = 0; k < folded; ++k) s += wtab[k];
      c->wsum[t] = s;
      c->valid[t] = 1;
    }
  }
  if (folded_out) *folded_out = total;
  if (finalized_out) *finalized_out = finalized ? 1 : 0;
  return FEDAVG_OK;
}

int32_t fedavg_dyn_configure(fedavg_ctx* c, int64_t idle_us, int64_t life_us) {
  FEDAVG_RET(check_ctx(c));
  if (idle_us < 0 || life_us < 0) return fail(FEDAVG_ERR_INVALID, "idle / life limits must be >= 0");
  if (idle_us) c->dyn.idle_ticks = static_cast<uint64_t>(idle_us) * 100;  // s_memrealtime: 100 MHz
  if (life_us) c->dyn.life_ticks = static_cast<uint64_t>(life_us) * 100;
  return FEDAVG_OK;
}

int32_t fedavg_dyn_timing(const fedavg_ctx* c, double* out, int32_t n) {
  FEDAVG_RET(check_ctx(c));
  const auto& d = c->dyn;
  double v[3] = {-1.0, -1.0, -1.0};
  if (d.host && d.timed && d.tend && !d.active) {
    FEDAVG_HIP_TRY(hipSetDevice(c->device));
    FEDAVG_HIP_TRY(hipStreamSynchronize(d.stream));
    FEDAVG_HIP_TRY(hipStreamSynchronize(d.edge_stream));
    std::vector<uint64_t> te(d.tiles.size() + d.edge_tiles.size());
    FEDAVG_HIP_TRY(hipMemcpy(te.data(), d.tend, sizeof(uint64_t) * te.size(), hipMemcpyDeviceToHost));
    const uint64_t t_end = te.empty() ? 0 : *std::max_element(te.begin(), te.end());
    const DynLayout L(c->T, d.cap);
    const DynAck* ack = reinterpret_cast<const DynAck*>(d.host + L.ack);
    const uint64_t t_rows = __atomic_load_n(&ack->t_rows, __ATOMIC_RELAXED);
    const uint64_t t_seen = __atomic_load_n(&ack->t_seen, __ATOMIC_RELAXED);
    if (t_end && t_rows && t_end >= t_rows) v[0] = static_cast<double>(t_end - t_rows) / 100.0;  // 100 MHz
    if (t_end && t_seen && t_end >= t_seen) v[1] = static_cast<double>(t_end - t_seen) / 100.0;
    if (t_seen && t_rows) v[2] = (static_cast<double>(t_seen) - static_cast<double>(t_rows)) / 100.0;
  }
  for (int32_t i = 0; i < n && i < 3; ++i) out[i] = v[i];
  return FEDAVG_OK;
}

int32_t fedavg_dyn_info(const fedavg_ctx* c, int32_t* info, int32_t n) {
  FEDAVG_RET(check_ctx(c));
  const auto& d = c->dyn;
  const int32_t v[5] = {d.active ? 1 : 0, d.published, d.base, d.reopens, d.launches};
  for (int32_t i = 0; i < n && i < 5; ++i) info[i] = v[i];
  return FEDAVG_OK;
}

int32_t fedavg_dyn_prof_collect(fedavg_ctx* c, double* total_ms, int32_t* waves) {
  FEDAVG_RET(check_ctx(c));
  double sum = 0.0;
  for (auto& pr : c->dyn.prof) {
    FEDAVG_HIP_TRY(hipEventSynchronize(pr.second));
    float ms = 0.f;
    FEDAVG_HIP_TRY(hipEventElapsedTime(&ms, pr.first, pr.second));
    sum += ms;
  }
  if (total_ms) *total_ms = sum;
  if (waves) *waves = static_cast<int32_t>(c->dyn.prof.size());
  for (auto& pr : c->dyn.prof) {
    c->event_pool.push_back(pr.first);
    c->event_pool.push_back(pr.second);
  }
  c->dyn.prof.clear();
  return FEDAVG_OK;
}

int32_t fedavg_dyn_state(const fedavg_ctx* c, int32_t* active, int32_t* published) {
  FEDAVG_RET(check_ctx(c));
  if (active) *active = c->dyn.active ? 1 : 0;
  if (published) *published = c->dyn.published;
  return FEDAVG_OK;
}

}  // extern "C"
