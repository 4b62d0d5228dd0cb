// sharded_comm.cpp — the multi-GPU exchange step of the FedAvg reduce, owned by the library.
//
// clients are sharded over one process per GPU; every rank folds its
// shard into an fp64 partial (the partial plan of fedavg_kernels.hip), the partials are summed to
// a root over RCCL (xGMI), and the root divides by the global total weights (the finalize plan).
// The reference has no collective (everything goes to one server process,
// simulation_lib/server/aggregation_server.py:111-145); this is the only exchange of the path.
//
// One round, all enqueued from one host call (no per-chunk framework dispatch):
//
//   compute stream : partial[c0]→ev0  partial[c1]→ev1 ...  partial[cK-1]→evK-1  (wait done) finalize
//   comm stream    :   (wait ev0) reduce[c0]  (wait ev1) reduce[c1] ...  reduce[cK-1] done
//
// The comm stream is a high-priority stream of its own: HIP places it on another hardware queue
// than the compute stream, so its waits do not sit behind later partial kernels (an AQL queue is
// processed in order; DESIGN.md §5 has the kernel traces). RCCL is not linked: the library binds
// the RCCL the process already has (torch's, by SONAME librccl.so.1) or loads it, at
// communicator creation (dlopen/dlsym). rccl.h supplies the types only.
#include <dlfcn.h>
#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/fedavg_hip.h"
#include "rccl_bind.h"

__attribute__((visibility("hidden"))) int32_t fedavg_internal_fail(int32_t code, const char* msg);
extern "C" __attribute__((visibility("hidden"))) int32_t fedavg_internal_plan_run_range(
    fedavg_plan* p, int32_t tb, int32_t te, void* stream, hipEvent_t* done_ev);
extern "C" __attribute__((visibility("hidden"))) int32_t fedavg_internal_set_prof(fedavg_ctx* c, int32_t on);

// The process's RCCL, bound once. FEDAVG_RCCL_LIB (a test stand-in) is loaded as named; otherwise
// RTLD_NOLOAD first: if torch (or the caller) has loaded an RCCL, use that very library, so one
// process never carries two RCCL runtimes.
FedavgRccl& fedavg_rccl() {
  static FedavgRccl r;
  static std::once_flag once;
  std::call_once(once, [] {
    const char* env = std::getenv("FEDAVG_RCCL_LIB");
    if (env && *env) {
      r.handle = dlopen(env, RTLD_NOW | RTLD_LOCAL);
    } else {
      const char* names[] = {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"};
      for (const char* n : names) {
        r.handle = dlopen(n, RTLD_NOW | RTLD_NOLOAD);
        if (r.handle) break;
      }
      for (const char* n : names) {
        if (r.handle) break;
        r.handle = dlopen(n, RTLD_NOW | RTLD_LOCAL);
      }
    }
    if (!r.handle) {
      const char* e = dlerror();
      r.error = std::string("cannot load RCCL: ") + (e ? e : "not found");
      return;
    }
    auto sym = [](const char* name) { return dlsym(r.handle, name); };
    r.get_unique_id = reinterpret_cast<decltype(r.get_unique_id)>(sym("ncclGetUniqueId"));
    r.comm_init_rank = reinterpret_cast<decltype(r.comm_init_rank)>(sym("ncclCommInitRank"));
    r.comm_init_all = reinterpret_cast<decltype(r.comm_init_all)>(sym("ncclCommInitAll"));
    r.comm_destroy = reinterpret_cast<decltype(r.comm_destroy)>(sym("ncclCommDestroy"));
    r.reduce = reinterpret_cast<decltype(r.reduce)>(sym("ncclReduce"));
    r.error_string = reinterpret_cast<decltype(r.error_string)>(sym("ncclGetErrorString"));
    r.reduce_scatter = reinterpret_cast<decltype(r.reduce_scatter)>(sym("ncclReduceScatter"));
    r.group_start = reinterpret_cast<decltype(r.group_start)>(sym("ncclGroupStart"));
    r.group_end = reinterpret_cast<decltype(r.group_end)>(sym("ncclGroupEnd"));
    r.gather = reinterpret_cast<decltype(r.gather)>(sym("ncclGather"));
    r.send = reinterpret_cast<decltype(r.send)>(sym("ncclSend"));
    r.recv = reinterpret_cast<decltype(r.recv)>(sym("ncclRecv"));
    if (!r.get_unique_id || !r.comm_init_rank || !r.comm_destroy || !r.reduce || !r.error_string ||
        !r.reduce_scatter || !r.group_start || !r.group_end || !r.send || !r.recv)
      r.error = "RCCL library lacks a required symbol";
  });
  return r;
}

int32_t fedavg_rccl_ready() {
  FedavgRccl& r = fedavg_rccl();
  if (!r.error.empty()) return fedavg_internal_fail(FEDAVG_ERR_RCCL, r.error.c_str());
  return FEDAVG_OK;
}

int32_t fedavg_rccl_fail(ncclResult_t res, const char* what) {
  std::string m = std::string(what) + ": " + fedavg_rccl().error_string(res);
  return fedavg_internal_fail(FEDAVG_ERR_RCCL, m.c_str());
}

namespace {

using Rccl = FedavgRccl;
Rccl& rccl() { return fedavg_rccl(); }
int32_t rccl_ready() { return fedavg_rccl_ready(); }
int32_t rccl_fail(ncclResult_t res, const char* what) { return fedavg_rccl_fail(res, what); }

#define COMM_HIP_TRY(expr)                                                                          \
  do {                                                                                              \
    hipError_t e_ = (expr);                                                                         \
    if (e_ != hipSuccess)                                                                           \
      return fedavg_internal_fail(FEDAVG_ERR_HIP, (std::string(#expr) + ": " + hipGetErrorString(e_)).c_str()); \
  } while (0)

}  // namespace

struct fedavg_comm {
  ncclComm_t nccl = nullptr;
  int32_t world = 0;
  int32_t rank = 0;
  int32_t device = 0;
  hipStream_t stream = nullptr;  // high-priority comm stream
  // the root's last step (finalize / copy-out) runs on the comm stream right behind the last
  // collective instead of on the compute stream behind a cross-stream wait (FEDAVG_FINISH_ON_COMM)
  bool finish_on_comm = false;
  // the root divides the chunks already reduced while the last chunk is still being reduced
  // (reduce exchange, >= 2 chunks; FEDAVG_OVERLAP_FINALIZE=0 turns it off): only the last chunk's
  // finalize follows the last collective
  bool overlap_finalize = true;
  std::vector<hipEvent_t> chunk_events;
  hipEvent_t done = nullptr;
  hipEvent_t head_done = nullptr;  // every chunk but the last has been reduced
  // scatter exchange scratch: reduce-scattered fp64 windows (+ the root's chunk tails) and the
  // finalized result in accumulator coordinates (output dtype)
  double* slice = nullptr;
  size_t slice_cap = 0;  // elements
  char* res = nullptr;
  size_t res_cap = 0;  // bytes
};

namespace {

int32_t ensure_events(fedavg_comm* c, int32_t chunks) {
  while (static_cast<int32_t>(c->chunk_events.size()) < chunks) {
    hipEvent_t ev = nullptr;
    COMM_HIP_TRY(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    c->chunk_events.push_back(ev);
  }
  return FEDAVG_OK;
}

int32_t ensure_scratch(fedavg_comm* c, hipStream_t s, size_t slice_elems, size_t res_bytes) {
  if (c->slice_cap >= slice_elems && c->res_cap >= res_bytes) return FEDAVG_OK;
  COMM_HIP_TRY(hipStreamSynchronize(c->stream));  // an earlier round may still read the old buffers
  COMM_HIP_TRY(hipStreamSynchronize(s));
  if (c->slice_cap < slice_elems) {
    if (c->slice) COMM_HIP_TRY(hipFree(c->slice));
    c->slice = nullptr;
    c->slice_cap = 0;
    COMM_HIP_TRY(hipMalloc(reinterpret_cast<void**>(&c->slice), std::max<size_t>(slice_elems, 1) * sizeof(double)));
    c->slice_cap = slice_elems;
  }
  if (c->res_cap < res_bytes) {
    if (c->res) COMM_HIP_TRY(hipFree(c->res));
    c->res = nullptr;
    c->res_cap = 0;
    COMM_HIP_TRY(hipMalloc(reinterpret_cast<void**>(&c->res), std::max<size_t>(res_bytes, 16)));
    c->res_cap = res_bytes;
  }
  return FEDAVG_OK;
}

// Root gathers every rank's count-element window: rank i's lands at recv + i * count elements.
ncclResult_t gather_windows(fedavg_comm* c, const char* send, char* recv, size_t count, size_t elem,
                            ncclDataType_t dt, int32_t root) {
  Rccl& r = rccl();
  if (r.gather) return r.gather(send, recv, count, dt, root, c->nccl, c->stream);
  ncclResult_t res = r.group_start();
  if (res != ncclSuccess) return res;
  if (c->rank == root) {
    for (int32_t i = 0; i < c->world && res == ncclSuccess; ++i)
      if (i != root) res = r.recv(recv + static_cast<size_t>(i) * count * elem, count, dt, i, c->nccl, c->stream);
  } else {
    res = r.send(send, count, dt, root, c->nccl, c->stream);
  }
  const ncclResult_t end = r.group_end();
  return res != ncclSuccess ? res : end;
}

// Tile edges of `chunks` equal ranges of n tiles (empty ranges dropped).
std::vector<int32_t> even_edges(int32_t n, int32_t chunks) {
  chunks = std::max(1, std::min(chunks, n));
  std::vector<int32_t> e{0};
  for (int32_t k = 0; k < chunks; ++k) {
    const int32_t te = static_cast<int32_t>((static_cast<int64_t>(n) * (k + 1)) / chunks);
    if (te > e.back()) e.push_back(te);
  }
  return e;
}

// Caller-given edges: 0 = e[0] < e[1] < ... < e[m-1] = n.
int32_t check_edges(const int32_t* e, int32_t m, int32_t n) {
  if (!e || m < 2 || e[0] != 0 || e[m - 1] != n)
    return fedavg_internal_fail(FEDAVG_ERR_INVALID, "tile edges must run from 0 to the context's tile count");
  for (int32_t i = 1; i < m; ++i)
    if (e[i] <= e[i - 1]) return fedavg_internal_fail(FEDAVG_ERR_INVALID, "tile edges must increase");
  return FEDAVG_OK;
}

int32_t round_reduce(fedavg_comm* c, fedavg_ctx* ctx, fedavg_plan* partial, fedavg_plan* finalize,
                     const std::vector<int32_t>& edges, int32_t root, void* stream);
int32_t round_scatter(fedavg_comm* c, fedavg_ctx* ctx, fedavg_plan* partial, fedavg_plan* finalize,
                      const std::vector<int32_t>& edges, int32_t root, void* stream);

}  // namespace

extern "C" {

int32_t fedavg_comm_unique_id(void* id_out) {
  if (!id_out) return fedavg_internal_fail(FEDAVG_ERR_INVALID, "null id buffer");
  if (int32_t st = rccl_ready()) return st;
  ncclUniqueId id;
  ncclResult_t res = rccl().get_unique_id(&id);
  if (res != ncclSuccess) return rccl_fail(res, "ncclGetUniqueId");
  std::memcpy(id_out, id.internal, FEDAVG_COMM_ID_BYTES);
  return FEDAVG_OK;
}

int32_t fedavg_comm_create(fedavg_comm** out, const void* id, int32_t world, int32_t rank, int32_t device) {
  if (!out || !id) return fedavg_internal_fail(FEDAVG_ERR_INVALID, "null argument");
  *out = nullptr;
  if (world < 1 || rank < 0 || rank >= world || device < 0)
    return fedavg_internal_fail(FEDAVG_ERR_INVALID, "bad world / rank / device");
  if (int32_t st = rccl_ready()) return st;
  COMM_HIP_TRY(hipSetDevice(device));
  auto* c = new fedavg_comm();
  c->world = world;
  c->rank = rank;
  c->device = device;
  if (const char* e = std::getenv("FEDAVG_FINISH_ON_COMM")) c->finish_on_comm = std::atoi(e) != 0;
  if (const char* e = std::getenv("FEDAVG_OVERLAP_FINALIZE")) c->overlap_finalize = std::atoi(e) != 0;
  int lo = 0, hi = 0;
  hipError_t e = hipDeviceGetStreamPriorityRange(&lo, &hi);
  if (e == hipSuccess) e = hipStreamCreateWithPriority(&c->stream, hipStreamNonBlocking, hi);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&c->done, hipEventDisableTiming);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&c->head_done, hipEventDisableTiming);
  if (e != hipSuccess) {
    fedavg_comm_destroy(c);
    return fedavg_internal_fail(FEDAVG_ERR_HIP, (std::string("comm stream: ") + hipGetErrorString(e)).c_str());
  }
  ncclUniqueId uid;
  std::memcpy(uid.internal, id, FEDAVG_COMM_ID_BYTES);
  ncclResult_t res = rccl().comm_init_rank(&c->nccl, world, uid, rank);  // collective over the ranks
  if (res != ncclSuccess) {
    c->nccl = nullptr;
    fedavg_comm_destroy(c);
    return rccl_fail(res, "ncclCommInitRank");
  }
  *out = c;
  return FEDAVG_OK;
}

int32_t fedavg_comm_destroy(fedavg_comm* c) {
  if (!c) return FEDAVG_OK;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  if (c->nccl) (void)rccl().comm_destroy(c->nccl);
  for (hipEvent_t ev : c->chunk_events) (void)hipEventDestroy(ev);
  if (c->done) (void)hipEventDestroy(c->done);
  if (c->head_done) (void)hipEventDestroy(c->head_done);
  if (c->slice) (void)hipFree(c->slice);
  if (c->res) (void)hipFree(c->res);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
  return FEDAVG_OK;
}

int32_t fedavg_sharded_round(fedavg_comm* c, fedavg_ctx* ctx, fedavg_plan* partial, fedavg_plan* finalize,
                             int32_t chunks, int32_t root, void* stream) {
  if (!c || !ctx || !partial) return fedavg_internal_fail(FEDAVG_ERR_INVALID, "null argument");
  const int32_t n = fedavg_num_tiles(ctx);
  if (n <= 0) return fedavg_internal_fail(FEDAVG_ERR_INVALID, "context has no tiles");
  return round_reduce(c, ctx, partial, finalize, even_edges(n, chunks), root, stream);
}

int32_t fedavg_sharded_round_edges(fedavg_comm* c, fedavg_ctx* ctx, fedavg_plan* partial, fedavg_plan* finalize,
                                   const int32_t* tile_edges, int32_t num_edges, int32_t exchange, int32_t root,
                                   void* stream) {
  if (!c || !ctx || !partial) return fedavg_internal_fail(FEDAVG_ERR_INVALID, "null argument");
  const int32_t n = fedavg_num_tiles(ctx);
  if (n <= 0) return fedavg_internal_fail(FEDAVG_ERR_INVALID, "context has no tiles");
  if (int32_t st = check_edges(tile_edges, num_edges, n)) return st;
  std::vector<int32_t> edges(tile_edges, tile_edges + num_edges);
  if (exchange == FEDAVG_EXCHANGE_REDUCE) return round_reduce(c, ctx, partial, finalize, edges, root, stream);
  if (exchange == FEDAVG_EXCHANGE_SCATTER) return round_scatter(c, ctx, partial, finalize, edges, root, stream);
  return fedavg_internal_fail(FEDAVG_ERR_INVALID, "exchange must be FEDAVG_EXCHANGE_REDUCE or _SCATTER");
}

int32_t fedavg_sharded_round_scatter(fedavg_comm* c, fedavg_ctx* ctx, fedavg_plan* partial, fedavg_plan* finalize,
                                     int32_t chunks, int32_t root, void* stream) {
  if (!c || !ctx || !partial || !finalize) return fedavg_internal_fail(FEDAVG_ERR_INVALID, "null argument");
  const int32_t n = fedavg_num_tiles(ctx);
  if (n <= 0) return fedavg_internal_fail(FEDAVG_ERR_INVALID, "context has no tiles");
  return round_scatter(c, ctx, partial, finalize, even_edges(n, chunks), root, stream);
}

}  // extern "C"

namespace {

int32_t round_reduce(fedavg_comm* c, fedavg_ctx* ctx, fedavg_plan* partial, fedavg_plan* finalize,
                     const std::vector<int32_t>& edges, int32_t root, void* stream) {
  if (root < 0 || root >= c->world) return fedavg_internal_fail(FEDAVG_ERR_INVALID, "bad root");
  if (c->rank == root && !finalize) return fedavg_internal_fail(FEDAVG_ERR_INVALID, "root needs a finalize plan");
  const int32_t n = edges.back();
  const int32_t chunks = static_cast<int32_t>(edges.size()) - 1;
  COMM_HIP_TRY(hipSetDevice(c->device));
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (int32_t st = ensure_events(c, chunks)) return st;
  double* acc = static_cast<double*>(fedavg_accumulator(ctx));
  // with profiling on (fedavg_prof_enable), only the first chunk's launch is timed
  const int32_t prof = fedavg_internal_set_prof(ctx, 0);
  struct Restore {
    fedavg_ctx* ctx;
    int32_t prof;
    ~Restore() { fedavg_internal_set_prof(ctx, prof); }
  } restore{ctx, prof};
  for (int32_t k = 0; k < chunks; ++k) {
    const int32_t tb = edges[k], te = edges[k + 1];
    fedavg_internal_set_prof(ctx, (k == 0) ? prof : 0);
    // the chunk's event completes with its kernel (no marker packet between chunk kernels)
    hipEvent_t ev = c->chunk_events[k];
    if (int32_t st = fedavg_internal_plan_run_range(partial, tb, te, s, &ev)) return st;
    int64_t a = 0, b = 0;
    if (int32_t st = fedavg_tile_range(ctx, tb, te, &a, &b)) return st;
    COMM_HIP_TRY(hipStreamWaitEvent(c->stream, ev, 0));
    ncclResult_t res = rccl().reduce(acc + a, acc + a, static_cast<size_t>(b - a), ncclFloat64, ncclSum, root,
                                     c->nccl, c->stream);
    if (res != ncclSuccess) return rccl_fail(res, "ncclReduce");
    if (k == chunks - 2) COMM_HIP_TRY(hipEventRecord(c->head_done, c->stream));
  }
  // The compute stream goes on once the reduces have landed (they run in order); the root then
  // divides. With overlap_finalize the tiles of every chunk but the last are divided as soon as
  // their reduces are done — on the compute stream, whose partial kernels have all been issued,
  // while the comm stream still reduces the last chunk — so only the last chunk's division
  // follows the last collective (the exposed tail: DESIGN.md §5 cost model). (Dividing each
  // chunk on the comm stream right behind its reduce was measured slower: 0.595 vs 0.566 ms per
  // one-rank round at 4 chunks — those finalize kernels contend with the next chunk's partial.)
  fedavg_internal_set_prof(ctx, 0);
  if (c->rank == root && c->finish_on_comm)
    if (int32_t st = fedavg_plan_run_range(finalize, 0, n, c->stream)) return st;
  const bool overlap = c->rank == root && !c->finish_on_comm && c->overlap_finalize && chunks >= 2;
  if (overlap) {
    COMM_HIP_TRY(hipStreamWaitEvent(s, c->head_done, 0));
    if (int32_t st = fedavg_plan_run_range(finalize, 0, edges[chunks - 1], s)) return st;
  }
  COMM_HIP_TRY(hipEventRecord(c->done, c->stream));
  COMM_HIP_TRY(hipStreamWaitEvent(s, c->done, 0));
  if (c->rank == root && !c->finish_on_comm)
    return fedavg_plan_run_range(finalize, overlap ? edges[chunks - 1] : 0, n, s);
  return FEDAVG_OK;
}

int32_t round_scatter(fedavg_comm* c, fedavg_ctx* ctx, fedavg_plan* partial, fedavg_plan* finalize,
                      const std::vector<int32_t>& edges, int32_t root, void* stream) {
  if (!finalize) return fedavg_internal_fail(FEDAVG_ERR_INVALID, "every rank needs a finalize plan");
  if (root < 0 || root >= c->world) return fedavg_internal_fail(FEDAVG_ERR_INVALID, "bad root");
  const int32_t odt = fedavg_plan_out_dtype(finalize);
  if (odt != FEDAVG_F32 && odt != FEDAVG_F64)
    return fedavg_internal_fail(FEDAVG_ERR_INVALID, "every rank needs a finalize plan (fp32 / fp64 outputs)");
  const int32_t chunks = static_cast<int32_t>(edges.size()) - 1;
  const int64_t G = c->world;
  const size_t ob = (odt == FEDAVG_F32) ? 4 : 8;
  const ncclDataType_t ndt = (odt == FEDAVG_F32) ? ncclFloat32 : ncclFloat64;
  COMM_HIP_TRY(hipSetDevice(c->device));
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (int32_t st = ensure_events(c, chunks)) return st;

  // geometry: chunk k = tiles [tb, te) = accumulator [A, B); B - A = G*L + R (R = 0 whenever G
  // divides 32: segments start at multiples of FEDAVG_ACC_ALIGN, tiles at multiples of 4096)
  struct Piece {
    int32_t tb, te;
    int64_t A, L, R, off, rem;
  };
  std::vector<Piece> pieces;
  int64_t slice_elems = 0, rem_elems = 0;
  for (int32_t k = 0; k < chunks; ++k) {
    const int32_t tb = edges[k], te = edges[k + 1];
    int64_t a = 0, b = 0;
    if (int32_t st = fedavg_tile_range(ctx, tb, te, &a, &b)) return st;
    Piece p{tb, te, a, (b - a) / G, (b - a) % G, slice_elems, rem_elems};
    slice_elems += p.L;
    rem_elems += p.R;
    pieces.push_back(p);
  }
  const int64_t acc_numel = fedavg_acc_numel(ctx);
  if (int32_t st = ensure_scratch(c, s, static_cast<size_t>(slice_elems + rem_elems), ob * static_cast<size_t>(acc_numel)))
    return st;
  double* acc = static_cast<double*>(fedavg_accumulator(ctx));
  double* rem_base = c->slice + slice_elems;
  const int32_t prof = fedavg_internal_set_prof(ctx, 0);
  struct Restore {
    fedavg_ctx* ctx;
    int32_t prof;
    ~Restore() { fedavg_internal_set_prof(ctx, prof); }
  } restore{ctx, prof};
  Rccl& r = rccl();
  for (size_t k = 0; k < pieces.size(); ++k) {
    const Piece& p = pieces[k];
    fedavg_internal_set_prof(ctx, (k == 0) ? prof : 0);
    hipEvent_t ev = c->chunk_events[k];
    if (int32_t st = fedavg_internal_plan_run_range(partial, p.tb, p.te, s, &ev)) return st;
    COMM_HIP_TRY(hipStreamWaitEvent(c->stream, ev, 0));
    ncclResult_t res = r.group_start();
    if (res == ncclSuccess && p.L > 0)
      res = r.reduce_scatter(acc + p.A, c->slice + p.off, static_cast<size_t>(p.L), ncclFloat64, ncclSum, c->nccl,
                             c->stream);
    if (res == ncclSuccess && p.R > 0)
      res = r.reduce(acc + p.A + G * p.L, rem_base + p.rem, static_cast<size_t>(p.R), ncclFloat64, ncclSum, root,
                     c->nccl, c->stream);
    const ncclResult_t end = r.group_end();
    if (res != ncclSuccess) return rccl_fail(res, "ncclReduceScatter");
    if (end != ncclSuccess) return rccl_fail(end, "ncclGroupEnd");
    // this rank's window (and the root's share of the tail), divided into the result buffer
    const int64_t lo = p.A + c->rank * p.L;
    if (p.L > 0)
      if (int32_t st = fedavg_plan_finalize_window(finalize, c->slice + p.off, lo, lo + p.L, c->res, c->stream))
        return st;
    if (p.R > 0 && c->rank == root)
      if (int32_t st = fedavg_plan_finalize_window(finalize, rem_base + p.rem, p.A + G * p.L, p.A + G * p.L + p.R,
                                                   c->res, c->stream))
        return st;
    if (p.L > 0) {
      res = gather_windows(c, c->res + static_cast<size_t>(lo) * ob, c->res + static_cast<size_t>(p.A) * ob,
                           static_cast<size_t>(p.L), ob, ndt, root);
      if (res != ncclSuccess) return rccl_fail(res, "ncclGather");
    }
  }
  fedavg_internal_set_prof(ctx, 0);
  if (c->rank == root && c->finish_on_comm)
    if (int32_t st = fedavg_plan_copy_out(finalize, c->res, c->stream)) return st;
  COMM_HIP_TRY(hipEventRecord(c->done, c->stream));
  COMM_HIP_TRY(hipStreamWaitEvent(s, c->done, 0));
  if (c->rank == root && !c->finish_on_comm) return fedavg_plan_copy_out(finalize, c->res, s);
  return FEDAVG_OK;
}

}  // namespace
