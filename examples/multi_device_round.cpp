// multi_device_round.cpp — the single-process multi-device FedAvg round driven through
// include/fedavg_hip.h alone (no Python, no torch): what the reference's ONE server process
// (simulation_lib/server/server.py:122-152 -> aggregation_server.py:111-145) does to spread its
// clients over the MI355X of a node.
//
//   1. fedavg_multi_create from a device list (entries may repeat a device: one-GPU tests)
//   2. per entry: its clients' partial plan on fedavg_multi_context(m, g)
//   3. fedavg_multi_round with the peer-window exchange (and, with --exchange reduce|both, the
//      in-process RCCL reduce), then fedavg_multi_check
//   4. the streaming form: per entry fedavg_accumulate waves, then fedavg_multi_combine
//
// Self-check against the host composition of the same arithmetic: each entry's arrival-order
// fp64 chain (acc = -0.0; acc += double(x) * w), the chains summed in entry order, divided by the
// arrival-order total weight — bit-identical for the peer exchange (and for the reduce under the
// in-process RCCL stand-in, which sums in rank order); within 1e-12 relative under real RCCL.
// Usage: multi_device_round [--devices 0,0,0,0] [--exchange peer|reduce|both]. "PASS" + exit 0.
#include <hip/hip_runtime_api.h>

#include <cinttypes>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
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

}  // namespace

int main(int argc, char** argv) {
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1) {
    std::fprintf(stderr, "no GPU\n");
    return 2;
  }
  std::vector<int32_t> devices;
  std::string exchange = "peer";
  for (int i = 1; i + 1 < argc; i += 2) {
    if (!std::strcmp(argv[i], "--devices")) {
      for (char* tok = std::strtok(argv[i + 1], ","); tok; tok = std::strtok(nullptr, ",")) devices.push_back(std::atoi(tok));
    } else if (!std::strcmp(argv[i], "--exchange")) {
      exchange = argv[i + 1];
    }
  }
  if (devices.empty()) {
    if (ndev >= 2)
      for (int d = 0; d < ndev; ++d) devices.push_back(d);
    else
      devices = {0, 0, 0, 0};
  }
  const int32_t G = static_cast<int32_t>(devices.size());
  const bool fake_rccl = std::getenv("FEDAVG_RCCL_LIB") != nullptr;
  const std::vector<int64_t> numel = {3 * 3 * 16 * 8, 16, 1000, 1, 70001, 4096 * 3 + 5};
  const int32_t T = static_cast<int32_t>(numel.size());
  const int N = 11;
  const double weights[N] = {120, 4999, 333, 1000, 17, 2500, 64, 777, 4096, 3, 1234};

  fedavg_multi* m = nullptr;
  CHECK_ST(fedavg_multi_create(&m, devices.data(), G, numel.data(), T, nullptr));
  std::printf("%d entries, peer access %d\n", (int)G, (int)fedavg_multi_peer_access(m));

  // client k lives on the entry that folds it; the round's two assignments: contiguous shards, and
  // the same with entry 1 holding no client (its partial is NULL)
  auto owner = [&](int k, int variant) {
    int g = static_cast<int>(static_cast<int64_t>(k) * G / N);
    if (variant == 1 && G > 1 && g == 1) g = 0;
    return g;
  };
  std::vector<std::vector<float>> host(static_cast<size_t>(N) * T);
  for (int k = 0; k < N; ++k)
    for (int t = 0; t < T; ++t) {
      auto& h = host[static_cast<size_t>(k) * T + t];
      h.resize(numel[t]);
      for (int64_t i = 0; i < numel[t]; ++i) h[i] = value(k, t, i);
    }
  double W = -0.0;
  for (int k = 0; k < N; ++k) W += weights[k];  // arrival order (fed_avg_algorithm.py:59-62)
  std::vector<double> totals(T, W);

  // the host composition of a variant
  auto composition = [&](int variant) {
    std::vector<std::vector<double>> want(T);
    for (int t = 0; t < T; ++t) {
      std::vector<double> sum;
      bool first = true;
      for (int g = 0; g < G; ++g) {
        std::vector<double> part(numel[t], -0.0);
        bool any = false;
        for (int k = 0; k < N; ++k) {
          if (owner(k, variant) != g) continue;
          any = true;
          const auto& h = host[static_cast<size_t>(k) * T + t];
          for (int64_t i = 0; i < numel[t]; ++i) {
            const double p = static_cast<double>(h[i]) * weights[k];
            part[i] += p;
          }
        }
        if (!any) continue;
        if (first) {
          sum = part;
          first = false;
        } else {
          for (int64_t i = 0; i < numel[t]; ++i) sum[i] += part[i];
        }
      }
      want[t].resize(numel[t]);
      for (int64_t i = 0; i < numel[t]; ++i) want[t][i] = sum[i] / W;
    }
    return want;
  };

  const int root = G > 1 ? G - 1 : 0;  // a root other than entry 0
  for (int variant = 0; variant < 2; ++variant) {
    // clients' buckets on their entry's device
    std::vector<void*> dev(static_cast<size_t>(N) * T, nullptr);
    for (int k = 0; k < N; ++k)
      for (int t = 0; t < T; ++t) {
        CHECK_HIP(hipSetDevice(devices[owner(k, variant)]));
        void*& p = dev[static_cast<size_t>(k) * T + t];
        CHECK_HIP(hipMalloc(&p, numel[t] * sizeof(float)));
        CHECK_HIP(hipMemcpy(p, host[static_cast<size_t>(k) * T + t].data(), numel[t] * sizeof(float),
                            hipMemcpyHostToDevice));
      }
    std::vector<fedavg_plan*> partials(G, nullptr);
    for (int g = 0; g < G; ++g) {
      std::vector<const void*> rows;
      std::vector<double> w;
      int K = 0;
      for (int k = 0; k < N; ++k) {
        if (owner(k, variant) != g) continue;
        for (int t = 0; t < T; ++t) {
          rows.push_back(dev[static_cast<size_t>(k) * T + t]);
          w.push_back(weights[k]);
        }
        ++K;
      }
      if (K) CHECK_ST(fedavg_plan_create_partial(fedavg_multi_context(m, g), rows.data(), FEDAVG_F32, w.data(), K, 1,
                                                 &partials[g]));
    }
    const auto want = composition(variant);
    for (int out_f32 = 0; out_f32 < 2; ++out_f32) {
      const size_t eb = out_f32 ? 4 : 8;
      std::vector<void*> out(T, nullptr);
      CHECK_HIP(hipSetDevice(devices[root]));
      for (int t = 0; t < T; ++t) CHECK_HIP(hipMalloc(&out[t], numel[t] * eb));
      auto compare = [&](const char* what, bool exact) -> int {
        for (int t = 0; t < T; ++t) {
          std::vector<char> raw(numel[t] * eb);
          CHECK_HIP(hipSetDevice(devices[root]));
          CHECK_HIP(hipMemcpy(raw.data(), out[t], raw.size(), hipMemcpyDeviceToHost));
          for (int64_t i = 0; i < numel[t]; ++i) {
            double got, ref = want[t][i];
            if (out_f32) {
              float f;
              std::memcpy(&f, raw.data() + 4 * i, 4);
              got = f;
              ref = static_cast<float>(ref);
            } else {
              std::memcpy(&got, raw.data() + 8 * i, 8);
            }
            const bool ok = exact ? same_bits(got, ref) : std::fabs(got - ref) <= 1e-12 * std::fabs(ref) + 1e-300;
            if (!ok) {
              std::fprintf(stderr, "%s: segment %d element %" PRId64 ": %.17g vs %.17g\n", what, t, i, got, ref);
              return 1;
            }
          }
        }
        std::printf("%s: %s the host composition\n", what, exact ? "bit-identical to" : "within 1e-12 of");
        return 0;
      };
      const int32_t n_tiles = fedavg_num_tiles(fedavg_multi_context(m, 0));
      const std::vector<std::vector<int32_t>> shapes = {{0, n_tiles}, {0, n_tiles / 3, (2 * n_tiles) / 3, n_tiles},
                                                        {0, n_tiles - 1, n_tiles}};
      const int32_t odt = out_f32 ? FEDAVG_F32 : FEDAVG_F64;
      for (const char* ex : {"peer", "reduce"}) {
        if (exchange != "both" && exchange != ex) continue;
        const int32_t code = !std::strcmp(ex, "peer") ? FEDAVG_EXCHANGE_PEER : FEDAVG_EXCHANGE_REDUCE;
        for (size_t s = 0; s < shapes.size(); ++s) {
          for (int round = 0; round < 2; ++round) {
            for (int t = 0; t < T; ++t) CHECK_HIP(hipMemset(out[t], 0xFF, numel[t] * eb));
            CHECK_ST(fedavg_multi_round(m, partials.data(), totals.data(), out.data(), odt, root, shapes[s].data(),
                                        static_cast<int32_t>(shapes[s].size()), code, nullptr));
            CHECK_ST(fedavg_multi_check(m, nullptr));
            char what[128];
            std::snprintf(what, sizeof(what), "variant %d %s out %s, %zu chunk(s), round %d", variant, ex,
                          out_f32 ? "fp32" : "fp64", shapes[s].size() - 1, round + 1);
            if (compare(what, code == FEDAVG_EXCHANGE_PEER || fake_rccl)) return 1;
          }
        }
        // the streaming form: each entry folds its clients in waves of 2, then one combine
        for (int t = 0; t < T; ++t) CHECK_HIP(hipMemset(out[t], 0xFF, numel[t] * eb));
        for (int g = 0; g < G; ++g) {
          std::vector<int> mine;
          for (int k = 0; k < N; ++k)
            if (owner(k, variant) == g) mine.push_back(k);
          for (size_t b = 0; b < mine.size(); b += 2) {
            std::vector<const void*> rows;
            std::vector<double> w;
            const size_t e = std::min(mine.size(), b + 2);
            for (size_t q = b; q < e; ++q)
              for (int t = 0; t < T; ++t) {
                rows.push_back(dev[static_cast<size_t>(mine[q]) * T + t]);
                w.push_back(weights[mine[q]]);
              }
            CHECK_ST(fedavg_accumulate(fedavg_multi_context(m, g), rows.data(), FEDAVG_F32, w.data(),
                                       static_cast<int32_t>(e - b), fedavg_multi_stream(m, g)));
          }
        }
        std::vector<void*> streams(G);
        for (int g = 0; g < G; ++g) streams[g] = fedavg_multi_stream(m, g);
        CHECK_ST(fedavg_multi_combine(m, totals.data(), out.data(), odt, root, code, streams.data()));
        CHECK_ST(fedavg_multi_check(m, nullptr));
        char what[128];
        std::snprintf(what, sizeof(what), "variant %d %s out %s, streamed waves + combine", variant, ex,
                      out_f32 ? "fp32" : "fp64");
        if (compare(what, code == FEDAVG_EXCHANGE_PEER || fake_rccl)) return 1;
      }
      for (void* p : out) CHECK_HIP(hipFree(p));
    }
    for (fedavg_plan* p : partials)
      if (p) CHECK_ST(fedavg_plan_destroy(p));
    for (void* p : dev) CHECK_HIP(hipFree(p));
  }
  CHECK_ST(fedavg_multi_destroy(m));
  std::printf("PASS\n");
  return 0;
}
