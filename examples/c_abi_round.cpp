// c_abi_round.cpp — a FedAvg server round driven through include/fedavg_hip.h alone: no Python,
// no torch. Shows what a C/C++ (or cgo / JNI / N-API) caller of the drop-in boundary does:
//
//   1. fedavg_ctx_create for the model layout (named tensors = segments)
//   2. per arriving client: fedavg_accumulate (streaming, fed_avg_algorithm.py:43-64)
//   3. fedavg_aggregate: ÷ total weight into fp32 / fp64 outputs (:76-99) + fedavg_check
//   4. the multi-GPU exchange on a one-rank RCCL world: fedavg_comm_* + fedavg_sharded_round
//      (reduce to the root) and fedavg_sharded_round_scatter (reduce-scatter + window finalize +
//      gather)
//   5. the round folded while it arrives, in two bursts (fedavg_dyn_*: the wave ends itself in
//      the pause and is continued from the fp64 accumulator by the next publication)
//
// Self-check: the streamed result and the sharded result are compared bit-for-bit with a plain
// fp64 host fold in arrival order (acc = -0.0; acc += double(x) * w; out = acc / W) — the
// reference's arithmetic. Exit code 0 and "PASS" on success. Built by build() next to the
// library (_lib/c_abi_round), run by tests/test_gpu_c_abi.py.
#include <hip/hip_runtime_api.h>

#include <chrono>
#include <cinttypes>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

#include "fedavg_hip.h"

#define CHECK_ST(call)                                                                         \
  do {                                                                                         \
    int32_t st_ = (call);                                                                      \
    if (st_ != FEDAVG_OK) {                                                                    \
      std::fprintf(stderr, "%s -> %d: %s\n", #call, (int)st_, fedavg_last_error());            \
      return 1;                                                                                \
    }                                                                                          \
  } while (0)
#define CHECK_HIP(call)                                                                        \
  do {                                                                                         \
    hipError_t e_ = (call);                                                                    \
    if (e_ != hipSuccess) {                                                                    \
      std::fprintf(stderr, "%s -> %s\n", #call, hipGetErrorString(e_));                        \
      return 1;                                                                                \
    }                                                                                          \
  } while (0)

namespace {

// deterministic client values: a small LCG mapped to [-2, 2) (fp32)
float value(uint64_t client, uint64_t seg, uint64_t i) {
  uint64_t s = (client + 1) * 0x9E3779B97F4A7C15ull ^ (seg + 7) * 0xBF58476D1CE4E5B9ull ^ (i + 3) * 0x94D049BB133111EBull;
  s ^= s >> 31;
  s *= 0xD6E8FEB86659FD93ull;
  s ^= s >> 29;
  return static_cast<float>(static_cast<double>(s >> 40) / static_cast<double>(1ull << 24) * 4.0 - 2.0);
}

bool same_bits(double a, double b) {
  uint64_t x, y;
  std::memcpy(&x, &a, 8);
  std::memcpy(&y, &b, 8);
  return x == y;
}

}  // namespace

int main() {
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1) {
    std::fprintf(stderr, "no GPU\n");
    return 2;
  }
  std::printf("ABI %d\n", (int)fedavg_abi_version());
  const std::vector<int64_t> numel = {3 * 3 * 16 * 8, 16, 1000, 1, 70001};  // segments (named tensors)
  const int32_t T = static_cast<int32_t>(numel.size());
  const int N = 9;
  const double weights[N] = {120, 4999, 333, 1000, 17, 2500, 64, 777, 4096};

  hipStream_t stream;
  CHECK_HIP(hipSetDevice(0));
  CHECK_HIP(hipStreamCreate(&stream));

  // client buckets in HBM (one allocation per client and segment, as a framework would hand over)
  std::vector<void*> dev(static_cast<size_t>(N) * T, nullptr);
  std::vector<std::vector<float>> host(static_cast<size_t>(N) * T);
  for (int k = 0; k < N; ++k)
    for (int t = 0; t < T; ++t) {
      auto& h = host[static_cast<size_t>(k) * T + t];
      h.resize(numel[t]);
      for (int64_t i = 0; i < numel[t]; ++i) h[i] = value(k, t, i);
      CHECK_HIP(hipMalloc(&dev[static_cast<size_t>(k) * T + t], numel[t] * sizeof(float)));
      CHECK_HIP(hipMemcpy(dev[static_cast<size_t>(k) * T + t], h.data(), numel[t] * sizeof(float), hipMemcpyHostToDevice));
    }
  std::vector<void*> out(T, nullptr);
  for (int t = 0; t < T; ++t) CHECK_HIP(hipMalloc(&out[t], numel[t] * sizeof(double)));

  // host fp64 fold in arrival order: the reference's arithmetic
  std::vector<std::vector<double>> want(T);
  double W = -0.0;
  for (int k = 0; k < N; ++k) W += weights[k];
  for (int t = 0; t < T; ++t) {
    want[t].assign(numel[t], -0.0);
    for (int k = 0; k < N; ++k) {
      const auto& h = host[static_cast<size_t>(k) * T + t];
      for (int64_t i = 0; i < numel[t]; ++i) {
        const double p = static_cast<double>(h[i]) * weights[k];
        want[t][i] += p;
      }
    }
    for (int64_t i = 0; i < numel[t]; ++i) want[t][i] /= W;
  }
  auto compare = [&](const char* what) -> int {
    for (int t = 0; t < T; ++t) {
      std::vector<double> got(numel[t]);
      CHECK_HIP(hipMemcpy(got.data(), out[t], numel[t] * sizeof(double), hipMemcpyDeviceToHost));
      for (int64_t i = 0; i < numel[t]; ++i)
        if (!same_bits(got[i], want[t][i])) {
          std::fprintf(stderr, "%s: segment %d element %" PRId64 ": %.17g vs %.17g\n", what, t, i, got[i], want[t][i]);
          return 1;
        }
    }
    std::printf("%s: bit-identical to the host fold\n", what);
    return 0;
  };

  fedavg_ctx* ctx = nullptr;
  CHECK_ST(fedavg_ctx_create(&ctx, 0, numel.data(), T, nullptr));

  // (1) streaming: one call per arriving client, then the finishing call
  for (int k = 0; k < N; ++k) {
    std::vector<double> w(T, weights[k]);
    CHECK_ST(fedavg_accumulate(ctx, &dev[static_cast<size_t>(k) * T], FEDAVG_F32, w.data(), 1, stream));
  }
  CHECK_ST(fedavg_aggregate(ctx, nullptr, FEDAVG_F32, nullptr, 0, out.data(), FEDAVG_F64, stream));
  CHECK_ST(fedavg_check(ctx, stream, nullptr));
  if (compare("streamed round")) return 1;

  // (2) the multi-GPU exchange step on a one-rank RCCL world (4 chunks)
  std::vector<double> wtab(static_cast<size_t>(N) * T);
  for (int k = 0; k < N; ++k)
    for (int t = 0; t < T; ++t) wtab[static_cast<size_t>(k) * T + t] = weights[k];
  std::vector<double> totals(T, W);
  fedavg_plan *partial = nullptr, *finalize = nullptr;
  CHECK_ST(fedavg_plan_create_partial(ctx, dev.data(), FEDAVG_F32, wtab.data(), N, 1, &partial));
  CHECK_ST(fedavg_plan_create_finalize(ctx, totals.data(), out.data(), FEDAVG_F64, &finalize));
  char id[FEDAVG_COMM_ID_BYTES];
  CHECK_ST(fedavg_comm_unique_id(id));
  fedavg_comm* comm = nullptr;
  CHECK_ST(fedavg_comm_create(&comm, id, 1, 0, 0));
  for (int round = 0; round < 2; ++round) {
    for (int t = 0; t < T; ++t) CHECK_HIP(hipMemsetAsync(out[t], 0xFF, numel[t] * sizeof(double), stream));
    CHECK_ST(fedavg_reset(ctx, stream));
    CHECK_ST(fedavg_sharded_round(comm, ctx, partial, finalize, 4, 0, stream));
    CHECK_ST(fedavg_check(ctx, stream, nullptr));
    if (compare(round == 0 ? "sharded round 1" : "sharded round 2")) return 1;
  }
  for (int round = 0; round < 2; ++round) {
    for (int t = 0; t < T; ++t) CHECK_HIP(hipMemsetAsync(out[t], 0xFF, numel[t] * sizeof(double), stream));
    CHECK_ST(fedavg_reset(ctx, stream));
    CHECK_ST(fedavg_sharded_round_scatter(comm, ctx, partial, finalize, 3, 0, stream));
    CHECK_ST(fedavg_check(ctx, stream, nullptr));
    if (compare(round == 0 ? "scatter round 1" : "scatter round 2")) return 1;
  }

  // (3) the round folded while it arrives (fedavg_dyn_*), at the reference server's burst cadence:
  //     4 updates, a pause longer than the wave's idle limit (it ends itself, its rows kept in the
  //     fp64 accumulator), the other 5 — the next publication continues the wave from the
  //     accumulator — then the close divides into the outputs
  CHECK_ST(fedavg_reset(ctx, stream));
  CHECK_HIP(hipStreamSynchronize(stream));
  CHECK_ST(fedavg_dyn_configure(ctx, 300, 0));  // idle limit 300 us
  for (int t = 0; t < T; ++t) CHECK_HIP(hipMemset(out[t], 0xFF, numel[t] * sizeof(double)));
  CHECK_ST(fedavg_dyn_open(ctx, FEDAVG_F32, N, stream));
  int32_t published = 0;
  CHECK_ST(fedavg_dyn_publish(ctx, dev.data(), wtab.data(), 4, stream, &published));
  if (published != 4) {
    std::fprintf(stderr, "dynamic wave: %d of 4 rows published\n", (int)published);
    return 1;
  }
  {
    const auto until = std::chrono::steady_clock::now() + std::chrono::milliseconds(5);
    while (std::chrono::steady_clock::now() < until) {
    }
  }
  CHECK_ST(fedavg_dyn_publish(ctx, dev.data(), wtab.data(), N, stream, &published));
  int32_t info[5] = {0, 0, 0, 0, 0};
  CHECK_ST(fedavg_dyn_info(ctx, info, 5));
  int32_t folded = 0, finalized = 0;
  CHECK_ST(fedavg_dyn_close(ctx, out.data(), FEDAVG_F64, 1, stream, &folded, &finalized));
  CHECK_ST(fedavg_check(ctx, stream, nullptr));
  if (folded != N || !finalized || info[2] != 4 || info[3] < 1) {
    std::fprintf(stderr, "dynamic wave: folded %d finalized %d base %d continued %d\n", (int)folded, (int)finalized,
                 (int)info[2], (int)info[3]);
    return 1;
  }
  if (compare("dynamic wave in two bursts (continued once)")) return 1;

  CHECK_ST(fedavg_comm_destroy(comm));
  CHECK_ST(fedavg_plan_destroy(partial));
  CHECK_ST(fedavg_plan_destroy(finalize));
  CHECK_ST(fedavg_ctx_destroy(ctx));
  for (void* p : dev) CHECK_HIP(hipFree(p));
  for (void* p : out) CHECK_HIP(hipFree(p));
  CHECK_HIP(hipStreamDestroy(stream));
  std::printf("PASS\n");
  return 0;
}
