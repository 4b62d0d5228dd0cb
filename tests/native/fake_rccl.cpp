// fake_rccl.cpp — TEST INFRASTRUCTURE: an in-process stand-in for the handful of RCCL entry
// points sharded_comm.cpp binds (dlsym by name; FEDAVG_RCCL_LIB points the library here).
//
// Why: RCCL refuses two ranks on one GPU ("Duplicate GPU detected"), and the boxes these tests run
// on have one GPU, so the native multi-rank round (fedavg_sharded_round / _scatter at world > 1:
// chunk windows, the scatter tail, the gather placement, a root other than 0) would otherwise first
// run in the driver's 8-GPU bench. Here the ranks are threads of one process on one GPU, and each
// collective runs synchronously on the host at call time: sync the caller's stream (its data is
// then final), meet the other ranks at a barrier, move / sum the bytes with blocking copies, meet
// again (nobody reuses a buffer another rank still reads). Sums run in rank order 0, 1, ..., G-1
// in the element type, so a test can state the expected bits exactly. Semantics follow rccl.h:
// ncclReduce (result on root), ncclReduceScatter (rank r gets window r), ncclGather (rank r's
// buffer at recv + r * count on root; in place when send == that slot), ncclSend / ncclRecv
// (paired through a mailbox, the gather fallback when built with -DFAKE_RCCL_NO_GATHER).
// ncclCommInitAll makes the communicators of ONE host thread driving every rank (the single-process
// multi-device mode, multi_device.cpp): their collectives must sit between ncclGroupStart and
// ncclGroupEnd, are queued there, and run at the outermost ncclGroupEnd — the i-th call of every
// rank forms one collective, summed in rank order like the threaded form.
// Not the product: nothing outside tests/ loads it.
#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

namespace {

struct Group {
  int n = 0;
  int refs = 0;
  std::mutex m;
  std::condition_variable cv;
  int arrived = 0;
  uint64_t generation = 0;
  std::vector<const void*> send;
  std::vector<void*> recv;
  // send / recv mailbox: slot[src * n + dst] = the posted send buffer (count elements)
  std::vector<const void*> box;
  std::vector<size_t> box_count;
};

std::mutex g_registry_mutex;
std::map<std::string, Group*> g_registry;
uint64_t g_next_id = 1;

void barrier(Group* g) {
  std::unique_lock<std::mutex> lk(g->m);
  const uint64_t gen = g->generation;
  if (++g->arrived == g->n) {
    g->arrived = 0;
    ++g->generation;
    g->cv.notify_all();
  } else {
    g->cv.wait(lk, [&] { return g->generation != gen; });
  }
}

size_t elem_size(ncclDataType_t t) {
  switch (t) {
    case ncclInt8:
    case ncclUint8:
      return 1;
    case ncclFloat16:
    case ncclBfloat16:
      return 2;
    case ncclInt32:
    case ncclUint32:
    case ncclFloat32:
      return 4;
    default:
      return 8;
  }
}

// A blocking copy on the caller's stream. (hipMemcpy on the null stream is not enough: a device-to-
// device hipMemcpy may return before the copy is done, and the library's streams are
// non-blocking, so its next kernel would not wait for it.)
bool copy(void* dst, const void* src, size_t bytes, hipStream_t s) {
  return hipMemcpyAsync(dst, src, bytes, hipMemcpyDefault, s) == hipSuccess && hipStreamSynchronize(s) == hipSuccess;
}

// dst = sum over ranks (rank order) of src[r] + off, count elements, on the host
template <typename T>
bool sum_ranks(Group* g, size_t off, size_t count, void* dst, hipStream_t s) {
  std::vector<T> acc(count), tmp(count);
  for (int r = 0; r < g->n; ++r) {
    const char* src = static_cast<const char*>(g->send[r]) + off * sizeof(T);
    if (!copy(r == 0 ? acc.data() : tmp.data(), src, count * sizeof(T), s)) return false;
    if (r > 0)
      for (size_t i = 0; i < count; ++i) acc[i] = acc[i] + tmp[i];
  }
  return copy(dst, acc.data(), count * sizeof(T), s);
}

bool sum_into(Group* g, ncclDataType_t t, size_t off, size_t count, void* dst, hipStream_t s) {
  if (count == 0) return true;
  if (t == ncclFloat64) return sum_ranks<double>(g, off, count, dst, s);
  if (t == ncclFloat32) return sum_ranks<float>(g, off, count, dst, s);
  return false;
}

}  // namespace

struct ncclComm {
  Group* g;
  int rank;
  bool single = false;  // made by ncclCommInitAll: one thread drives every rank
};

namespace {

// grouped calls of single-thread communicators, queued until the outermost ncclGroupEnd
struct Pending {
  ncclComm_t comm;
  const void* send;
  void* recv;
  size_t count;
  ncclDataType_t dt;
  int root;
  hipStream_t stream;
};
thread_local int g_depth = 0;
thread_local std::vector<Pending> g_pending;

ncclResult_t run_pending() {
  std::vector<Pending> ops;
  ops.swap(g_pending);
  // per communicator group: the i-th op of each rank forms collective i
  std::map<Group*, std::vector<std::vector<Pending>>> by_group;
  for (const Pending& p : ops) {
    auto& ranks = by_group[p.comm->g];
    ranks.resize(p.comm->g->n);
    ranks[p.comm->rank].push_back(p);
  }
  for (auto& [g, ranks] : by_group) {
    const size_t n_ops = ranks[0].size();
    for (const auto& r : ranks)
      if (r.size() != n_ops) return ncclInvalidUsage;  // every rank must join every collective
    for (size_t i = 0; i < n_ops; ++i) {
      for (int r = 0; r < g->n; ++r) {
        const Pending& p = ranks[r][i];
        if (hipStreamSynchronize(p.stream) != hipSuccess) return ncclUnhandledCudaError;
        g->send[r] = p.send;
        g->recv[r] = p.recv;
      }
      const Pending& rootp = ranks[ranks[0][i].root][i];
      if (!sum_into(g, rootp.dt, 0, rootp.count, rootp.recv, rootp.stream)) return ncclInvalidArgument;
    }
  }
  return ncclSuccess;
}

}  // namespace

extern "C" {

ncclResult_t ncclGetUniqueId(ncclUniqueId* id) {
  std::memset(id->internal, 0, sizeof(id->internal));
  std::lock_guard<std::mutex> lk(g_registry_mutex);
  std::snprintf(id->internal, sizeof(id->internal), "fake-rccl-%llu", static_cast<unsigned long long>(g_next_id++));
  return ncclSuccess;
}

ncclResult_t ncclCommInitRank(ncclComm_t* comm, int nranks, ncclUniqueId id, int rank) {
  if (!comm || nranks < 1 || rank < 0 || rank >= nranks) return ncclInvalidArgument;
  Group* g = nullptr;
  {
    std::lock_guard<std::mutex> lk(g_registry_mutex);
    const std::string key(id.internal, strnlen(id.internal, sizeof(id.internal)));
    auto it = g_registry.find(key);
    if (it == g_registry.end()) {
      g = new Group();
      g->n = nranks;
      g->send.assign(nranks, nullptr);
      g->recv.assign(nranks, nullptr);
      g->box.assign(static_cast<size_t>(nranks) * nranks, nullptr);
      g->box_count.assign(static_cast<size_t>(nranks) * nranks, 0);
      g_registry[key] = g;
    } else {
      g = it->second;
      if (g->n != nranks) return ncclInvalidUsage;
    }
    ++g->refs;
  }
  *comm = new ncclComm{g, rank};
  barrier(g);  // collective: returns once every rank joined
  return ncclSuccess;
}

ncclResult_t ncclCommDestroy(ncclComm_t comm) {
  if (!comm) return ncclSuccess;
  std::lock_guard<std::mutex> lk(g_registry_mutex);
  if (--comm->g->refs == 0) {
    for (auto it = g_registry.begin(); it != g_registry.end(); ++it)
      if (it->second == comm->g) {
        g_registry.erase(it);
        break;
      }
    delete comm->g;
  }
  delete comm;
  return ncclSuccess;
}

const char* ncclGetErrorString(ncclResult_t) { return "fake rccl: collective failed"; }

ncclResult_t ncclCommInitAll(ncclComm_t* comms, int ndev, const int* devlist) {
  (void)devlist;  // duplicates welcome: every rank may sit on the one test GPU
  if (!comms || ndev < 1) return ncclInvalidArgument;
  Group* g = new Group();
  g->n = ndev;
  g->refs = ndev;
  g->send.assign(ndev, nullptr);
  g->recv.assign(ndev, nullptr);
  g->box.assign(static_cast<size_t>(ndev) * ndev, nullptr);
  g->box_count.assign(static_cast<size_t>(ndev) * ndev, 0);
  {
    std::lock_guard<std::mutex> lk(g_registry_mutex);
    g_registry["fake-rccl-all-" + std::to_string(g_next_id++)] = g;
  }
  for (int r = 0; r < ndev; ++r) comms[r] = new ncclComm{g, r, true};
  return ncclSuccess;
}

ncclResult_t ncclGroupStart() {
  ++g_depth;
  return ncclSuccess;
}
ncclResult_t ncclGroupEnd() {
  if (g_depth <= 0) return ncclInvalidUsage;
  if (--g_depth == 0 && !g_pending.empty()) return run_pending();
  return ncclSuccess;
}

ncclResult_t ncclReduce(const void* sendbuff, void* recvbuff, size_t count, ncclDataType_t datatype, ncclRedOp_t op,
                        int root, ncclComm_t comm, hipStream_t stream) {
  if (op != ncclSum || root < 0 || root >= comm->g->n) return ncclInvalidArgument;
  if (comm->single) {
    if (g_depth == 0) return ncclInvalidUsage;  // one thread, many ranks: grouped calls only
    g_pending.push_back(Pending{comm, sendbuff, recvbuff, count, datatype, root, stream});
    return ncclSuccess;
  }
  if (hipStreamSynchronize(stream) != hipSuccess) return ncclUnhandledCudaError;
  Group* g = comm->g;
  g->send[comm->rank] = sendbuff;
  g->recv[comm->rank] = recvbuff;
  barrier(g);
  bool ok = true;
  if (comm->rank == root) ok = sum_into(g, datatype, 0, count, recvbuff, stream);
  barrier(g);
  return ok ? ncclSuccess : ncclInvalidArgument;
}

ncclResult_t ncclReduceScatter(const void* sendbuff, void* recvbuff, size_t recvcount, ncclDataType_t datatype,
                               ncclRedOp_t op, ncclComm_t comm, hipStream_t stream) {
  if (op != ncclSum) return ncclInvalidArgument;
  if (hipStreamSynchronize(stream) != hipSuccess) return ncclUnhandledCudaError;
  Group* g = comm->g;
  g->send[comm->rank] = sendbuff;
  g->recv[comm->rank] = recvbuff;
  barrier(g);
  const bool ok = sum_into(g, datatype, static_cast<size_t>(comm->rank) * recvcount, recvcount, recvbuff, stream);
  barrier(g);
  return ok ? ncclSuccess : ncclInvalidArgument;
}

#ifndef FAKE_RCCL_NO_GATHER
ncclResult_t ncclGather(const void* sendbuff, void* recvbuff, size_t sendcount, ncclDataType_t datatype, int root,
                        ncclComm_t comm, hipStream_t stream) {
  if (root < 0 || root >= comm->g->n) return ncclInvalidArgument;
  if (hipStreamSynchronize(stream) != hipSuccess) return ncclUnhandledCudaError;
  Group* g = comm->g;
  g->send[comm->rank] = sendbuff;
  g->recv[comm->rank] = recvbuff;
  barrier(g);
  bool ok = true;
  if (comm->rank == root) {
    const size_t bytes = sendcount * elem_size(datatype);
    for (int r = 0; r < g->n && ok; ++r) {
      char* dst = static_cast<char*>(recvbuff) + static_cast<size_t>(r) * bytes;
      if (dst != g->send[r]) ok = copy(dst, g->send[r], bytes, stream);
    }
  }
  barrier(g);
  return ok ? ncclSuccess : ncclInvalidArgument;
}
#endif

ncclResult_t ncclSend(const void* sendbuff, size_t count, ncclDataType_t, int peer, ncclComm_t comm,
                      hipStream_t stream) {
  Group* g = comm->g;
  if (peer < 0 || peer >= g->n) return ncclInvalidArgument;
  if (hipStreamSynchronize(stream) != hipSuccess) return ncclUnhandledCudaError;
  const size_t slot = static_cast<size_t>(comm->rank) * g->n + peer;
  std::unique_lock<std::mutex> lk(g->m);
  g->box[slot] = sendbuff;
  g->box_count[slot] = count;
  g->cv.notify_all();
  g->cv.wait(lk, [&] { return g->box[slot] == nullptr; });  // the receiver copied it
  return ncclSuccess;
}

ncclResult_t ncclRecv(void* recvbuff, size_t count, ncclDataType_t datatype, int peer, ncclComm_t comm,
                      hipStream_t stream) {
  Group* g = comm->g;
  if (peer < 0 || peer >= g->n) return ncclInvalidArgument;
  if (hipStreamSynchronize(stream) != hipSuccess) return ncclUnhandledCudaError;
  const size_t slot = static_cast<size_t>(peer) * g->n + comm->rank;
  std::unique_lock<std::mutex> lk(g->m);
  g->cv.wait(lk, [&] { return g->box[slot] != nullptr; });
  bool ok = g->box_count[slot] == count && copy(recvbuff, g->box[slot], count * elem_size(datatype), stream);
  g->box[slot] = nullptr;
  g->cv.notify_all();
  return ok ? ncclSuccess : ncclInvalidArgument;
}

}  // extern "C"
