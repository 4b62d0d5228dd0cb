// threaded_ranks.cpp — TEST INFRASTRUCTURE: the native multi-rank FedAvg round at world 2, 3 and 4,
// every rank a thread of this process on GPU 0, the collectives served by tests/native/fake_rccl.cpp
// (run with FEDAVG_RCCL_LIB=<that library>; see its header for why).
//
// Each world size G runs BASELINE config 3's structure at a small size: N clients sharded in
// contiguous blocks, every rank folds its shard into an fp64 partial (fedavg_plan_create_partial),
// and the round goes through fedavg_sharded_round (reduce to the root) and
// fedavg_sharded_round_scatter (reduce-scatter + per-rank window finalize + gather) at 1, 3 and 4
// chunks and two uneven chunkings (fedavg_sharded_round_edges), fp64 and fp32 outputs, roots 0 and G - 1, two rounds on the same plans. The root's
// outputs are compared bit-for-bit with the host composition the fake's sums define: per-rank
// arrival-order fold (acc = -0.0; acc += double(x) * w), the partials added in rank order, then
// / W (and the fp32 cast). A NaN in the last rank's shard must fail the root's fedavg_check under
// both exchanges. Exit 0 and "PASS" on success.
#include <hip/hip_runtime_api.h>

#include <atomic>
#include <cinttypes>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "fedavg_hip.h"

namespace {

std::mutex g_log_mutex;
std::atomic<int> g_failures{0};

void fail(const std::string& what) {
  std::lock_guard<std::mutex> lk(g_log_mutex);
  std::fprintf(stderr, "FAIL: %s\n", what.c_str());
  ++g_failures;
}

// a failed call ends the process: the other ranks would wait for this one in a collective forever
[[noreturn]] void abort_run(const std::string& what) {
  fail(what);
  std::fflush(stdout);
  std::fflush(stderr);
  std::_Exit(1);
}

#define RK_ST(call)                                                                                  \
  do {                                                                                               \
    int32_t st_ = (call);                                                                            \
    if (st_ != FEDAVG_OK) abort_run(std::string(#call) + " -> " + std::to_string(st_) + ": " + fedavg_last_error()); \
  } while (0)
#define RK_HIP(call)                                                                                 \
  do {                                                                                               \
    hipError_t e_ = (call);                                                                          \
    if (e_ != hipSuccess) abort_run(std::string(#call) + " -> " + hipGetErrorString(e_));            \
  } while (0)

float value(uint64_t client, uint64_t seg, uint64_t i) {
  uint64_t s = (client + 11) * 0x9E3779B97F4A7C15ull ^ (seg + 5) * 0xBF58476D1CE4E5B9ull ^ (i + 1) * 0x94D049BB133111EBull;
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

// segments (named tensors): odd sizes so segment padding, partial last tiles and scatter tails
// (chunk lengths not divisible by 3) all occur; 4096-element tiles -> 12 tiles in all
const std::vector<int64_t> kFixedNumel = {3 * 3 * 16 * 8, 16, 1000, 1, 40001, 7};
constexpr int kClients = 11;
const double kWeights[kClients] = {120, 4999, 333, 1000, 17, 2500, 64, 777, 4096, 3, 250};

struct World {
  int G = 0;
  int root = 0;
  std::vector<int64_t> numel = kFixedNumel;
  bool sweep = false;  // a randomised layout (reported separately)
  char id[FEDAVG_COMM_ID_BYTES];
  std::vector<std::vector<double>> want;  // [segment][element], fp64 result
  double W = 0;
};

// the host composition: per-rank chains, partials summed in rank order, / W
void expected(World& w) {
  const auto& kNumel = w.numel;
  const int T = static_cast<int>(kNumel.size());
  w.W = -0.0;
  for (int k = 0; k < kClients; ++k) w.W += kWeights[k];
  w.want.assign(T, {});
  for (int t = 0; t < T; ++t) {
    std::vector<double> total;
    for (int r = 0; r < w.G; ++r) {
      const int lo = r * kClients / w.G, hi = (r + 1) * kClients / w.G;
      std::vector<double> part(kNumel[t], -0.0);
      for (int k = lo; k < hi; ++k)
        for (int64_t i = 0; i < kNumel[t]; ++i) {
          const double p = static_cast<double>(value(k, t, i)) * kWeights[k];
          part[i] += p;
        }
      if (r == 0) {
        total = part;
      } else {
        for (int64_t i = 0; i < kNumel[t]; ++i) total[i] = total[i] + part[i];
      }
    }
    for (int64_t i = 0; i < kNumel[t]; ++i) total[i] /= w.W;
    w.want[t] = std::move(total);
  }
}

void rank_main(World* w, int rank) {
  const auto& kNumel = w->numel;
  const int T = static_cast<int>(kNumel.size());
  const int G = w->G;
  const int lo = rank * kClients / G, hi = (rank + 1) * kClients / G, n = hi - lo;
  RK_HIP(hipSetDevice(0));
  hipStream_t stream;
  RK_HIP(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));

  std::vector<void*> dev(static_cast<size_t>(n) * T, nullptr);
  for (int k = 0; k < n; ++k)
    for (int t = 0; t < T; ++t) {
      std::vector<float> h(kNumel[t]);
      for (int64_t i = 0; i < kNumel[t]; ++i) h[i] = value(lo + k, t, i);
      void*& d = dev[static_cast<size_t>(k) * T + t];
      RK_HIP(hipMalloc(&d, kNumel[t] * sizeof(float)));
      RK_HIP(hipMemcpy(d, h.data(), kNumel[t] * sizeof(float), hipMemcpyHostToDevice));
    }
  std::vector<void*> out64(T, nullptr), out32(T, nullptr);
  for (int t = 0; t < T; ++t) {
    RK_HIP(hipMalloc(&out64[t], kNumel[t] * sizeof(double)));
    RK_HIP(hipMalloc(&out32[t], kNumel[t] * sizeof(float)));
  }
  std::vector<double> wtab(static_cast<size_t>(n) * T);
  for (int k = 0; k < n; ++k)
    for (int t = 0; t < T; ++t) wtab[static_cast<size_t>(k) * T + t] = kWeights[lo + k];
  std::vector<double> totals(T, w->W);

  fedavg_ctx* ctx = nullptr;
  RK_ST(fedavg_ctx_create(&ctx, 0, kNumel.data(), T, nullptr));
  fedavg_plan *partial = nullptr, *fin64 = nullptr, *fin32 = nullptr;
  RK_ST(fedavg_plan_create_partial(ctx, dev.data(), FEDAVG_F32, wtab.data(), n, 1, &partial));
  RK_ST(fedavg_plan_create_finalize(ctx, totals.data(), out64.data(), FEDAVG_F64, &fin64));
  RK_ST(fedavg_plan_create_finalize(ctx, totals.data(), out32.data(), FEDAVG_F32, &fin32));
  fedavg_comm* comm = nullptr;
  RK_ST(fedavg_comm_create(&comm, w->id, G, rank, 0));

  auto check_root = [&](const std::string& what, bool f32) {
    for (int t = 0; t < T; ++t) {
      std::vector<double> got(kNumel[t]);
      if (f32) {
        std::vector<float> g32(kNumel[t]);
        if (hipMemcpy(g32.data(), out32[t], kNumel[t] * sizeof(float), hipMemcpyDeviceToHost) != hipSuccess)
          return fail(what + ": D2H");
        for (int64_t i = 0; i < kNumel[t]; ++i) got[i] = g32[i];
      } else if (hipMemcpy(got.data(), out64[t], kNumel[t] * sizeof(double), hipMemcpyDeviceToHost) != hipSuccess) {
        return fail(what + ": D2H");
      }
      for (int64_t i = 0; i < kNumel[t]; ++i) {
        const double want = f32 ? static_cast<double>(static_cast<float>(w->want[t][i])) : w->want[t][i];
        if (!same_bits(got[i], want)) {
          char buf[256];
          std::snprintf(buf, sizeof buf, "%s: segment %d element %" PRId64 ": %.17g vs %.17g", what.c_str(), t, i,
                        got[i], want);
          return fail(buf);
        }
      }
    }
  };

  // uneven chunks through fedavg_sharded_round_edges (chunks < 0 below): a short first chunk,
  // then a long one; a short last chunk
  const int32_t ntiles = fedavg_num_tiles(ctx);
  const bool uneven = ntiles >= 4;
  const std::vector<int32_t> edges_a = uneven ? std::vector<int32_t>{0, 1, ntiles / 2, ntiles} : std::vector<int32_t>{};
  const std::vector<int32_t> edges_b = uneven ? std::vector<int32_t>{0, ntiles - 2, ntiles - 1, ntiles}
                                              : std::vector<int32_t>{};
  int checked = 0;
  for (int scatter = 0; scatter < 2; ++scatter)
    for (int chunks : {1, 3, 4, -1, -2})
      if (chunks > 0 || uneven)
      for (int f32 = 0; f32 < 2; ++f32)
        for (int round = 0; round < 2; ++round) {
          fedavg_plan* fin = f32 ? fin32 : fin64;
          const auto& outs = f32 ? out32 : out64;
          for (int t = 0; t < T; ++t)
            RK_HIP(hipMemsetAsync(outs[t], 0xFF, kNumel[t] * (f32 ? 4 : 8), stream));
          RK_ST(fedavg_reset(ctx, stream));
          fedavg_plan* fin_rank = (scatter || rank == w->root) ? fin : nullptr;
          if (chunks < 0) {
            const auto& e = chunks == -1 ? edges_a : edges_b;
            RK_ST(fedavg_sharded_round_edges(comm, ctx, partial, fin_rank, e.data(), static_cast<int32_t>(e.size()),
                                             scatter ? FEDAVG_EXCHANGE_SCATTER : FEDAVG_EXCHANGE_REDUCE, w->root,
                                             stream));
          } else if (scatter) {
            RK_ST(fedavg_sharded_round_scatter(comm, ctx, partial, fin, chunks, w->root, stream));
          } else {
            RK_ST(fedavg_sharded_round(comm, ctx, partial, fin_rank, chunks, w->root, stream));
          }
          RK_ST(fedavg_check(ctx, stream, nullptr));
          if (rank == w->root) {
            check_root(std::string(scatter ? "scatter" : "reduce") + " G=" + std::to_string(G) + " root=" +
                           std::to_string(w->root) + " chunks=" + std::to_string(chunks) + (f32 ? " f32" : " f64") +
                           " round " + std::to_string(round),
                       f32 != 0);
            ++checked;
          }
        }

  // a NaN in the last rank's shard: the root's check must fail under both exchanges
  if (rank == G - 1) {
    const float nan = std::numeric_limits<float>::quiet_NaN();
    int big = 0;
    for (int t = 1; t < T; ++t)
      if (kNumel[t] > kNumel[big]) big = t;
    RK_HIP(hipMemcpy(static_cast<float*>(dev[static_cast<size_t>(n - 1) * T + big]) + kNumel[big] / 2, &nan, 4,
                     hipMemcpyHostToDevice));
  }
  for (int scatter = 0; scatter < 2; ++scatter) {
    RK_ST(fedavg_reset(ctx, stream));
    if (scatter)
      RK_ST(fedavg_sharded_round_scatter(comm, ctx, partial, fin32, 3, w->root, stream));
    else
      RK_ST(fedavg_sharded_round(comm, ctx, partial, rank == w->root ? fin32 : nullptr, 3, w->root, stream));
    const int32_t st = fedavg_check(ctx, stream, nullptr);
    if (rank == w->root && st != FEDAVG_ERR_NAN_ACCUM && st != FEDAVG_ERR_NAN_RESULT)
      fail(std::string(scatter ? "scatter" : "reduce") + " G=" + std::to_string(G) +
           ": the root missed a NaN in another shard (status " + std::to_string(st) + ")");
  }

  RK_ST(fedavg_comm_destroy(comm));
  RK_ST(fedavg_plan_destroy(partial));
  RK_ST(fedavg_plan_destroy(fin64));
  RK_ST(fedavg_plan_destroy(fin32));
  RK_ST(fedavg_ctx_destroy(ctx));
  for (void* p : dev) RK_HIP(hipFree(p));
  for (int t = 0; t < T; ++t) {
    RK_HIP(hipFree(out64[t]));
    RK_HIP(hipFree(out32[t]));
  }
  RK_HIP(hipStreamDestroy(stream));
  if (rank == w->root) {
    std::lock_guard<std::mutex> lk(g_log_mutex);
    if (w->sweep)
      std::printf("sweep G=%d root=%d T=%d: %d root rounds checked\n", G, w->root, T, checked);
    else
      std::printf("G=%d root=%d: %d root rounds checked\n", G, w->root, checked);
  }
}

}  // namespace

int main() {
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1) {
    std::fprintf(stderr, "no GPU\n");
    return 2;
  }
  for (int G : {2, 3, 4})
    for (int root : {0, G - 1}) {
      World w;
      w.G = G;
      w.root = root;
      expected(w);
      if (fedavg_comm_unique_id(w.id) != FEDAVG_OK) {
        std::fprintf(stderr, "fedavg_comm_unique_id: %s\n", fedavg_last_error());
        return 1;
      }
      std::vector<std::thread> ranks;
      for (int r = 0; r < G; ++r) ranks.emplace_back(rank_main, &w, r);
      for (auto& th : ranks) th.join();
      if (g_failures.load()) return 1;
    }
  // randomised layouts: segment sizes from 1 to 3 tiles with odd tails, worlds 2..5 (5 leaves
  // scatter tails), a random root
  uint64_t st = 0x2545F4914F6CDD1Dull;
  auto rnd = [&st](uint64_t m) {
    st ^= st << 13;
    st ^= st >> 7;
    st ^= st << 17;
    return st % m;
  };
  for (int trial = 0; trial < 6; ++trial) {
    World w;
    w.sweep = true;
    w.G = 2 + static_cast<int>(rnd(4));
    w.root = static_cast<int>(rnd(w.G));
    w.numel.clear();
    const int T = 1 + static_cast<int>(rnd(7));
    for (int t = 0; t < T; ++t) {
      const uint64_t kind = rnd(4);
      w.numel.push_back(kind == 0 ? 1 + static_cast<int64_t>(rnd(40))
                        : kind == 1 ? 4096 * (1 + static_cast<int64_t>(rnd(3)))
                                    : 1 + static_cast<int64_t>(rnd(3 * 4096 + 100)));
    }
    expected(w);
    if (fedavg_comm_unique_id(w.id) != FEDAVG_OK) {
      std::fprintf(stderr, "fedavg_comm_unique_id: %s\n", fedavg_last_error());
      return 1;
    }
    std::vector<std::thread> ranks;
    for (int r = 0; r < w.G; ++r) ranks.emplace_back(rank_main, &w, r);
    for (auto& th : ranks) th.join();
    if (g_failures.load()) return 1;
  }
  std::printf("PASS\n");
  return 0;
}
