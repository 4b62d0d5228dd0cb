// host_pack.cpp — native host-side packing of one client update into a pinned staging bucket.
//
// The reference's server receives every update as CPU tensors (aggregation_server.py:129,
// aggregation_worker.py:152). ingest.HostIngest moves a client to HBM with ONE DMA from a
// pinned bucket; this is the host copy that fills the bucket: the client's T named tensors
// (pageable, arbitrary sizes) are copied to their 16-B aligned offsets by a persistent pool of
// threads, the work cut into equal byte ranges across tensors — one C call per client instead
// of T framework copies (which cost ~5 µs of dispatch each, more than a small tensor's copy).
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/fedavg_hip.h"

__attribute__((visibility("hidden"))) int32_t fedavg_internal_fail(int32_t code, const char* msg);

namespace {

struct Piece {
  char* dst;
  const char* src;
  size_t bytes;
};

// A fixed pool of worker threads that run "job" slices. One job at a time (callers are the
// single server thread, like the rest of the ABI); the calling thread takes slice 0.
class PackPool {
 public:
  static PackPool& get() {
    static PackPool pool;
    return pool;
  }

  int threads() const { return static_cast<int>(workers_.size()) + 1; }

  void run(const std::vector<Piece>& pieces, size_t total) {
    const int n = threads();
    if (n == 1 || total < (size_t(4) << 20)) {  // small updates: one thread is faster
      for (const Piece& p : pieces) std::memcpy(p.dst, p.src, p.bytes);
      return;
    }
    {
      std::lock_guard<std::mutex> lk(mu_);
      pieces_ = &pieces;
      total_ = total;
      pending_ = n - 1;
      ++generation_;
    }
    cv_.notify_all();
    work(0, n);
    std::unique_lock<std::mutex> lk(mu_);
    done_cv_.wait(lk, [&] { return pending_ == 0; });
    pieces_ = nullptr;
  }

 private:
  PackPool() {
    int n = 0;
    if (const char* e = std::getenv("FEDAVG_PACK_THREADS")) n = std::atoi(e);
    if (n <= 0) {
      const char* omp = std::getenv("OMP_NUM_THREADS");
      n = omp ? std::atoi(omp) : 0;
      if (n <= 0) n = static_cast<int>(std::thread::hardware_concurrency());
      n = std::min(n, 8);  // host memory bandwidth saturates well before this
    }
    n = std::max(1, std::min(n, 64));
    for (int i = 1; i < n; ++i) workers_.emplace_back([this, i] { loop(i); });
  }

  ~PackPool() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
      ++generation_;
    }
    cv_.notify_all();
    for (auto& t : workers_) t.join();
  }

  void loop(int idx) {
    uint64_t seen = 0;
    for (;;) {
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return stop_ || generation_ != seen; });
        if (stop_) return;
        seen = generation_;
      }
      work(idx, threads());
      {
        std::lock_guard<std::mutex> lk(mu_);
        if (--pending_ == 0) done_cv_.notify_one();
      }
    }
  }

  // slice idx of n: the byte range [total*idx/n, total*(idx+1)/n) of the concatenated pieces
  void work(int idx, int n) {
    const std::vector<Piece>& pieces = *pieces_;
    const size_t lo = total_ * idx / n, hi = total_ * (idx + 1) / n;
    size_t pos = 0;
    for (const Piece& p : pieces) {
      const size_t a = std::max(lo, pos), b = std::min(hi, pos + p.bytes);
      if (a < b) std::memcpy(p.dst + (a - pos), p.src + (a - pos), b - a);
      pos += p.bytes;
      if (pos >= hi) break;
    }
  }

  std::vector<std::thread> workers_;
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  const std::vector<Piece>* pieces_ = nullptr;
  size_t total_ = 0;
  int pending_ = 0;
  uint64_t generation_ = 0;
  bool stop_ = false;
};

}  // namespace

extern "C" {

int32_t fedavg_host_pack(void* dst, const void* const* srcs, const int64_t* nbytes, const int64_t* dst_off,
                         int32_t n) {
  if (n < 0 || (n > 0 && (!dst || !srcs || !nbytes || !dst_off)))
    return fedavg_internal_fail(FEDAVG_ERR_INVALID, "fedavg_host_pack: bad arguments");
  std::vector<Piece> pieces;
  pieces.reserve(n);
  size_t total = 0;
  for (int32_t i = 0; i < n; ++i) {
    if (nbytes[i] < 0 || dst_off[i] < 0) return fedavg_internal_fail(FEDAVG_ERR_INVALID, "fedavg_host_pack: negative size");
    if (nbytes[i] == 0 || srcs[i] == nullptr) continue;
    pieces.push_back(Piece{static_cast<char*>(dst) + dst_off[i], static_cast<const char*>(srcs[i]),
                           static_cast<size_t>(nbytes[i])});
    total += static_cast<size_t>(nbytes[i]);
  }
  PackPool::get().run(pieces, total);
  return FEDAVG_OK;
}

int32_t fedavg_host_pack_threads(void) { return PackPool::get().threads(); }

}  // extern "C"
