// multi_device.cpp — the single-process multi-device mode of the FedAvg reduce (fedavg_multi_*).
//
// the reference aggregates in ONE server process
// (simulation_lib/server/server.py:122-152 -> aggregation_server.py:111-145); this object lets that
// process shard the client sum of fed_avg_algorithm.py:43-64 over the MI355X of a node. It owns one
// context per device entry (the shard's fold: fedavg_kernels.hip), one library stream and one
// high-priority exchange stream per entry, and the peer mappings between the devices.
//
// The PEER exchange (no collective library): chunk k of the tile table is cut into G windows and
// device j owns window j. Per chunk, device g first folds the chunk's OTHER windows (a launch on
// each side of its own): each tile's fp64 partial is stored straight into the window owner's receive
// slot for g over xGMI (the store address is a peer mapping picked per tile from a window table).
// An event after those launches orders every other device's exchange stream behind them. Device j's
// exchange stream then folds its own window of chunk k — its clients from -0.0 — and, per element,
// adds the received partials of the other devices in device order (its own chain taken from
// registers at its place), divides, and stores the result into the root's outputs (a peer store for
// j != root). Per round, HBM carries on each device its clients, the (G-1)/G of the fp64 partial
// arriving from peers, one read of it, and 1/G of the result — no fp64 partial is written and
// re-read whole, no own-window partial at all, and no copy engine or collective kernel sits between
// the fold and the division. Quantised-record plans keep the older form: every
// window (their own included) into the owner's slot, then a separate combine kernel.
//
//   exchange stream j : (wait part[g != j][k]) fold own window of chunk k + combine ... -> done[j]
//   stream g          : partial(chunk k, the other windows: each to its owner's slot) -> part[g][k]
//
// The REDUCE exchange keeps the per-process path's arithmetic: each chunk's partial is reduced to
// the root's accumulator by an in-process RCCL communicator (ncclCommInitAll, grouped calls from
// this one host thread), then the root divides.
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/fedavg_hip.h"
#include "rccl_bind.h"

__attribute__((visibility("hidden"))) int32_t fedavg_internal_fail(int32_t code, const char* msg);
extern "C" {
__attribute__((visibility("hidden"))) int32_t fedavg_internal_plan_run_range(fedavg_plan* p, int32_t tb, int32_t te,
                                                                           void* stream, hipEvent_t* done_ev);
__attribute__((visibility("hidden"))) int32_t fedavg_internal_plan_run_range_to(fedavg_plan* p, int32_t tb, int32_t te,
                                                                              void* stream, double* acc_out);
__attribute__((visibility("hidden"))) int32_t fedavg_internal_plan_run_windows(fedavg_plan* p, int32_t tb, int32_t te,
                                                                             void* stream, double* const* dst,
                                                                             const int32_t* edge, int32_t n);
__attribute__((visibility("hidden"))) int32_t fedavg_internal_plan_is_record(const fedavg_plan* p);
__attribute__((visibility("hidden"))) int32_t fedavg_internal_plan_run_comb(fedavg_plan* p, int32_t tb, int32_t te,
                                                                          void* stream, const double* const* comb_src,
                                                                          int32_t comb_n, int32_t comb_self,
                                                                          const double* totals, void* const* outs,
                                                                          int32_t out_dtype);
__attribute__((visibility("hidden"))) int32_t fedavg_internal_multi_combine(fedavg_ctx* c, int32_t tb, int32_t te,
                                                                          const double* const* slots, int32_t G,
                                                                          const double* wtot, void* const* outs,
                                                                          int32_t out_dtype, int32_t vec, void* stream);
__attribute__((visibility("hidden"))) int32_t fedavg_internal_segment_valid(const fedavg_ctx* c, int32_t* out);
__attribute__((visibility("hidden"))) int32_t fedavg_internal_segment_tiles(const fedavg_ctx* c, int32_t seg,
                                                                          int32_t* tb, int32_t* te);
__attribute__((visibility("hidden"))) void fedavg_internal_clear_state(fedavg_ctx* c);
__attribute__((visibility("hidden"))) uint32_t fedavg_internal_flags(fedavg_ctx* c, int32_t clear);
}

namespace {

#define MULTI_HIP_TRY(expr)                                                                          \
  do {                                                                                               \
    hipError_t e_ = (expr);                                                                          \
    if (e_ != hipSuccess)                                                                            \
      return fedavg_internal_fail(FEDAVG_ERR_HIP, (std::string(#expr) + ": " + hipGetErrorString(e_)).c_str()); \
  } while (0)

int32_t invalid(const char* msg) { return fedavg_internal_fail(FEDAVG_ERR_INVALID, msg); }

}  // namespace

struct fedavg_multi {
  int32_t G = 0;
  int32_t T = 0;
  std::vector<int32_t> devices;
  std::vector<int64_t> seg_numel;
  int64_t acc_numel = 0;
  int32_t num_tiles = 0;
  std::vector<fedavg_ctx*> ctx;
  std::vector<hipStream_t> own;   // the library stream of each entry (streams[g] == NULL)
  std::vector<hipStream_t> xstr;  // the high-priority exchange stream of each entry
  bool peer_ok = true;
  std::string peer_error;
  // slots[j][g]: entry j's receive buffer for entry g's partial of entry j's windows, the windows of
  // a round's chunks packed one after the other (slot_cap[j] elements: 1/G of the accumulator,
  // not all of it); slots[j][j] is entry j's own accumulator. A launch addresses a window through
  // a pointer rebased by the window's accumulator offset (rebased()), so the kernels keep
  // accumulator coordinates.
  std::vector<std::vector<double*>> slots;
  std::vector<std::vector<bool>> slot_owned;
  std::vector<int64_t> slot_cap;
  // this round's windows: [j][chunk] accumulator start of window j of the chunk and its offset in
  // the packed slot (both multiples of FEDAVG_ACC_ALIGN elements)
  std::vector<std::vector<int64_t>> win_acc, win_off;
  // per entry: the combine's device table, T fp64 totals then T output pointers
  std::vector<char*> tab_dev;
  std::vector<std::vector<char>> tab_host;  // what each entry's table holds
  std::vector<hipEvent_t> start_ev;   // the caller's stream g, at round start
  std::vector<hipEvent_t> done_ev;    // entry j's last exchange work of the round
  hipEvent_t end_ev = nullptr;        // entry 0's stream behind every entry's exchange work
  std::vector<std::vector<hipEvent_t>> part_ev;  // [g][chunk]
  // per entry g: its window table for the windowed partial launches — [chunks][G] rebased slot
  // pointers (device j's receive slot for g) then [chunks][G + 1] tile edges — on device g, and its
  // host image
  std::vector<char*> win_dev;
  std::vector<size_t> win_cap;
  std::vector<std::vector<char>> win_host;
  // per entry j: the own-window combine's source tables — [chunks][FEDAVG_MULTI_MAX_DEVICES]
  // rebased slots[j][h] for the round's members h — on device j, and its host image
  std::vector<char*> comb_dev;
  std::vector<std::vector<char>> comb_host;
  bool any_round = false;
  // fedavg_multi_prof_enable: per round, three timing events on entry 0's stream (device 0) — the
  // round's start, the end of entry 0's last chunk fold, the round's end behind every exchange
  bool prof = false;
  std::vector<std::vector<hipEvent_t>> prof_ev;  // rounds x {start, fold end, end}
  std::vector<hipEvent_t> prof_pool;
  // in-process RCCL (REDUCE exchange)
  std::vector<ncclComm_t> nccl;
};

namespace {

size_t tab_bytes(int32_t T) { return static_cast<size_t>(T) * (sizeof(double) + sizeof(void*)); }

int32_t ensure_part_events(fedavg_multi* m, int32_t chunks) {
  for (int32_t g = 0; g < m->G; ++g) {
    MULTI_HIP_TRY(hipSetDevice(m->devices[g]));
    while (static_cast<int32_t>(m->part_ev[g].size()) < chunks) {
      hipEvent_t ev = nullptr;
      // default flags: the marker releases the peer stores at system scope before a peer waits
      MULTI_HIP_TRY(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
      m->part_ev[g].push_back(ev);
    }
  }
  return FEDAVG_OK;
}

// fedavg_multi_prof_enable: a timing event recorded on entry 0's stream (device 0)
int32_t prof_mark(fedavg_multi* m, void* const* streams, int32_t which) {
  if (!m->prof) return FEDAVG_OK;
  MULTI_HIP_TRY(hipSetDevice(m->devices[0]));
  if (which == 0) m->prof_ev.push_back(std::vector<hipEvent_t>(3, nullptr));
  hipEvent_t ev = nullptr;
  if (!m->prof_pool.empty()) {
    ev = m->prof_pool.back();
    m->prof_pool.pop_back();
  } else {
    MULTI_HIP_TRY(hipEventCreate(&ev));
  }
  m->prof_ev.back()[which] = ev;
  MULTI_HIP_TRY(hipEventRecord(ev, (streams && streams[0]) ? static_cast<hipStream_t>(streams[0]) : m->own[0]));
  return FEDAVG_OK;
}

int64_t align_up(int64_t n) { return (n + FEDAVG_ACC_ALIGN - 1) / FEDAVG_ACC_ALIGN * FEDAVG_ACC_ALIGN; }

// The windows of this round's chunks and receive slots big enough for them. Window j of chunk k
// covers tiles [e_k + span*j/G, e_k + span*(j+1)/G) = accumulator elements [a, b); entry j's slots
// pack its windows in chunk order, each rounded up to the accumulator alignment. A slot is
// reallocated (after every device drained: a peer may still write the old one) only when a new
// chunking needs more than it holds.
int32_t ensure_slots(fedavg_multi* m, const std::vector<int32_t>& edges) {
  const int32_t G = m->G, chunks = static_cast<int32_t>(edges.size()) - 1;
  m->win_acc.assign(G, std::vector<int64_t>(chunks, 0));
  m->win_off.assign(G, std::vector<int64_t>(chunks, 0));
  std::vector<int64_t> need(G, 0);
  for (int32_t k = 0; k < chunks; ++k) {
    const int64_t tb = edges[k], span = edges[k + 1] - edges[k];
    for (int32_t j = 0; j < G; ++j) {
      const int32_t wb = static_cast<int32_t>(tb + span * j / G), we = static_cast<int32_t>(tb + span * (j + 1) / G);
      int64_t a = 0, b = 0;
      if (wb < we)
        if (int32_t st = fedavg_tile_range(m->ctx[j], wb, we, &a, &b)) return st;
      m->win_acc[j][k] = a;
      m->win_off[j][k] = need[j];
      need[j] += align_up(b - a);
    }
  }
  bool grow = false;
  for (int32_t j = 0; j < G; ++j) grow = grow || need[j] > m->slot_cap[j];
  if (!grow) return FEDAVG_OK;
  for (int32_t g = 0; g < G; ++g) {
    MULTI_HIP_TRY(hipSetDevice(m->devices[g]));
    MULTI_HIP_TRY(hipDeviceSynchronize());
  }
  for (int32_t j = 0; j < G; ++j) {
    if (need[j] <= m->slot_cap[j]) continue;
    MULTI_HIP_TRY(hipSetDevice(m->devices[j]));
    for (int32_t g = 0; g < G; ++g) {
      if (g == j) continue;
      if (m->slot_owned[j][g] && m->slots[j][g]) MULTI_HIP_TRY(hipFree(m->slots[j][g]));
      m->slots[j][g] = nullptr;
      double* p = nullptr;
      MULTI_HIP_TRY(hipMalloc(reinterpret_cast<void**>(&p), sizeof(double) * static_cast<size_t>(need[j])));
      m->slots[j][g] = p;
      m->slot_owned[j][g] = true;
    }
    m->slot_cap[j] = need[j];
  }
  return FEDAVG_OK;
}

// Where entry g's partial of window (j, chunk k) goes, in accumulator coordinates: entry j's slot
// for g rebased by the window's accumulator start (a kernel adds the tile's accumulator offset);
// entry j's own partial stays in its accumulator.
double* rebased(const fedavg_multi* m, int32_t j, int32_t g, int32_t k) {
  if (g == j) return m->slots[j][j];
  const uintptr_t base = reinterpret_cast<uintptr_t>(m->slots[j][g]);
  return reinterpret_cast<double*>(base + sizeof(double) * static_cast<uintptr_t>(m->win_off[j][k]) -
                                   sizeof(double) * static_cast<uintptr_t>(m->win_acc[j][k]));
}

// Entry j's combine table (totals, outputs); re-uploaded only when it changes (once per plan in a
// server that reuses its output buffers), after the exchange stream stopped reading the old one.
int32_t upload_tables(fedavg_multi* m, const double* totals, void* const* outs) {
  std::vector<char> img(tab_bytes(m->T));
  std::memcpy(img.data(), totals, sizeof(double) * m->T);
  std::memcpy(img.data() + sizeof(double) * m->T, outs, sizeof(void*) * m->T);
  for (int32_t j = 0; j < m->G; ++j) {
    if (m->tab_host[j] == img) continue;
    MULTI_HIP_TRY(hipSetDevice(m->devices[j]));
    MULTI_HIP_TRY(hipStreamSynchronize(m->xstr[j]));
    if (!m->tab_dev[j]) MULTI_HIP_TRY(hipMalloc(reinterpret_cast<void**>(&m->tab_dev[j]), img.size()));
    MULTI_HIP_TRY(hipMemcpy(m->tab_dev[j], img.data(), img.size(), hipMemcpyHostToDevice));
    m->tab_host[j] = img;
  }
  return FEDAVG_OK;
}

// Entry g's window table for this round's chunk edges (re-uploaded only when the edges or the slots
// change, after the device finished the launches that read the old one).
int32_t upload_windows(fedavg_multi* m, const std::vector<int32_t>& edges) {
  const int32_t G = m->G, chunks = static_cast<int32_t>(edges.size()) - 1;
  const size_t ptr_bytes = sizeof(double*) * static_cast<size_t>(chunks) * G;
  for (int32_t g = 0; g < G; ++g) {
    std::vector<char> img(ptr_bytes + sizeof(int32_t) * static_cast<size_t>(chunks) * (G + 1));
    auto* dst = reinterpret_cast<double**>(img.data());
    auto* e = reinterpret_cast<int32_t*>(img.data() + ptr_bytes);
    for (int32_t k = 0; k < chunks; ++k) {
      const int64_t tb = edges[k], span = edges[k + 1] - edges[k];
      for (int32_t j = 0; j < G; ++j) dst[k * G + j] = rebased(m, j, g, k);
      for (int32_t j = 0; j <= G; ++j) e[k * (G + 1) + j] = static_cast<int32_t>(tb + span * j / G);
    }
    if (m->win_host[g] == img) continue;
    MULTI_HIP_TRY(hipSetDevice(m->devices[g]));
    MULTI_HIP_TRY(hipDeviceSynchronize());
    if (m->win_cap[g] < img.size()) {
      if (m->win_dev[g]) MULTI_HIP_TRY(hipFree(m->win_dev[g]));
      m->win_dev[g] = nullptr;
      m->win_cap[g] = 0;
      MULTI_HIP_TRY(hipMalloc(reinterpret_cast<void**>(&m->win_dev[g]), img.size()));
      m->win_cap[g] = img.size();
    }
    MULTI_HIP_TRY(hipMemcpy(m->win_dev[g], img.data(), img.size(), hipMemcpyHostToDevice));
    m->win_host[g] = img;
  }
  return FEDAVG_OK;
}

// Entry j's own-window combine sources for this round's members and chunks (re-uploaded when they
// change, after entry j's exchange stream stopped reading the old table).
int32_t upload_comb(fedavg_multi* m, const std::vector<int32_t>& members, int32_t chunks) {
  const size_t need = sizeof(double*) * FEDAVG_MULTI_MAX_DEVICES * static_cast<size_t>(chunks);
  for (int32_t j = 0; j < m->G; ++j) {
    // the image keeps the allocation's size (a round of fewer chunks leaves the tail as it was)
    std::vector<char> img(std::max(need, m->comb_host[j].size()), 0);
    auto* src = reinterpret_cast<double**>(img.data());
    for (int32_t k = 0; k < chunks; ++k)
      for (size_t i = 0; i < members.size(); ++i) src[k * FEDAVG_MULTI_MAX_DEVICES + i] = rebased(m, j, members[i], k);
    if (m->comb_host[j].size() == img.size() &&
        std::memcmp(m->comb_host[j].data(), img.data(), need) == 0)
      continue;
    MULTI_HIP_TRY(hipSetDevice(m->devices[j]));
    MULTI_HIP_TRY(hipStreamSynchronize(m->xstr[j]));
    if (m->comb_host[j].size() < img.size()) {
      if (m->comb_dev[j]) MULTI_HIP_TRY(hipFree(m->comb_dev[j]));
      m->comb_dev[j] = nullptr;
      MULTI_HIP_TRY(hipMalloc(reinterpret_cast<void**>(&m->comb_dev[j]), img.size()));
    }
    MULTI_HIP_TRY(hipMemcpy(m->comb_dev[j], img.data(), need, hipMemcpyHostToDevice));
    m->comb_host[j] = img;  // only its first `need` bytes are compared
  }
  return FEDAVG_OK;
}

bool outs_aligned(void* const* outs, int32_t T, int32_t out_dtype) {
  const uintptr_t a = (out_dtype == FEDAVG_F32) ? 8 : 16;  // the combine's pair stores
  for (int32_t t = 0; t < T; ++t)
    if (reinterpret_cast<uintptr_t>(outs[t]) % a) return false;
  return true;
}

hipStream_t stream_of(fedavg_multi* m, void* const* streams, int32_t g) {
  return (streams && streams[g]) ? static_cast<hipStream_t>(streams[g]) : m->own[g];
}

int32_t check_common(fedavg_multi* m, const double* totals, void* const* outs, int32_t out_dtype, int32_t root) {
  if (!m) return invalid("null multi-device object");
  if (!totals || !outs) return invalid("null totals or output table");
  if (out_dtype != FEDAVG_F32 && out_dtype != FEDAVG_F64) return invalid("out dtype must be FEDAVG_F32 or FEDAVG_F64");
  if (root < 0 || root >= m->G) return invalid("bad root");
  for (int32_t t = 0; t < m->T; ++t)
    if (!outs[t]) return invalid("null output pointer");
  return FEDAVG_OK;
}

// Every stream the round uses starts after what the caller enqueued on its stream of that entry,
// and after the previous round's exchange work (which read the receive slots this round writes).
int32_t order_round_start(fedavg_multi* m, void* const* streams) {
  for (int32_t g = 0; g < m->G; ++g) {
    MULTI_HIP_TRY(hipSetDevice(m->devices[g]));
    hipStream_t s = stream_of(m, streams, g);
    if (m->any_round)
      for (int32_t j = 0; j < m->G; ++j) MULTI_HIP_TRY(hipStreamWaitEvent(s, m->done_ev[j], 0));
    MULTI_HIP_TRY(hipEventRecord(m->start_ev[g], s));
  }
  // an exchange stream reads every entry's buffers (the combine form reads the accumulators the
  // entries' waves wrote): it starts after all of them
  for (int32_t j = 0; j < m->G; ++j) {
    MULTI_HIP_TRY(hipSetDevice(m->devices[j]));
    for (int32_t g = 0; g < m->G; ++g) MULTI_HIP_TRY(hipStreamWaitEvent(m->xstr[j], m->start_ev[g], 0));
  }
  return FEDAVG_OK;
}

// The caller's root stream (and every caller stream: their next kernels may overwrite client
// buffers the round still reads) continues after the exchange.
int32_t order_round_end(fedavg_multi* m, void* const* streams) {
  for (int32_t j = 0; j < m->G; ++j) {
    MULTI_HIP_TRY(hipSetDevice(m->devices[j]));
    MULTI_HIP_TRY(hipEventRecord(m->done_ev[j], m->xstr[j]));
  }
  for (int32_t g = 0; g < m->G; ++g) {
    MULTI_HIP_TRY(hipSetDevice(m->devices[g]));
    hipStream_t s = stream_of(m, streams, g);
    for (int32_t j = 0; j < m->G; ++j) MULTI_HIP_TRY(hipStreamWaitEvent(s, m->done_ev[j], 0));
  }
  // one event that completes after the whole round (fedavg_multi_round_check waits for it alone)
  MULTI_HIP_TRY(hipSetDevice(m->devices[0]));
  MULTI_HIP_TRY(hipEventRecord(m->end_ev, stream_of(m, streams, 0)));
  m->any_round = true;
  return FEDAVG_OK;
}

int32_t ensure_nccl(fedavg_multi* m) {
  if (!m->nccl.empty()) return FEDAVG_OK;
  if (int32_t st = fedavg_rccl_ready()) return st;
  FedavgRccl& r = fedavg_rccl();
  if (!r.comm_init_all) return fedavg_internal_fail(FEDAVG_ERR_RCCL, "RCCL library lacks ncclCommInitAll");
  std::vector<ncclComm_t> comms(m->G, nullptr);
  std::vector<int> devs(m->devices.begin(), m->devices.end());
  ncclResult_t res = r.comm_init_all(comms.data(), m->G, devs.data());
  if (res != ncclSuccess) return fedavg_rccl_fail(res, "ncclCommInitAll");
  m->nccl = comms;
  return FEDAVG_OK;
}

// One grouped ncclReduce of accumulator range [a, b) of every entry to the root's accumulator, on
// the exchange streams (each already ordered behind its entry's partial).
int32_t grouped_reduce(fedavg_multi* m, int64_t a, int64_t b, int32_t root) {
  FedavgRccl& r = fedavg_rccl();
  ncclResult_t res = r.group_start();
  for (int32_t g = 0; g < m->G && res == ncclSuccess; ++g) {
    double* acc = static_cast<double*>(fedavg_accumulator(m->ctx[g]));
    res = r.reduce(acc + a, acc + a, static_cast<size_t>(b - a), ncclFloat64, ncclSum, root, m->nccl[g], m->xstr[g]);
  }
  const ncclResult_t end = r.group_end();
  if (res != ncclSuccess) return fedavg_rccl_fail(res, "ncclReduce");
  if (end != ncclSuccess) return fedavg_rccl_fail(end, "ncclGroupEnd");
  return FEDAVG_OK;
}

int32_t root_finalize(fedavg_multi* m, const double* totals, void* const* outs, int32_t out_dtype, int32_t root) {
  fedavg_ctx* rc = m->ctx[root];
  MULTI_HIP_TRY(hipSetDevice(m->devices[root]));
  if (int32_t st = fedavg_set_accumulated(rc, totals)) return st;
  const int32_t st = fedavg_finalize_range(rc, outs, out_dtype, 0, m->num_tiles, m->xstr[root]);
  fedavg_internal_clear_state(rc);  // the round is finished (fed_avg_algorithm.py:90,98)
  return st;
}

}  // namespace

extern "C" {

// Every entry point switches devices (hipSetDevice per entry) and hands the caller's current
// device back on return: the caller (torch's current device, a C program's hipSetDevice) must not
// find its device changed by a call that only enqueued work.
struct DeviceRestore {
  int prev = -1;
  DeviceRestore() {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
  }
  ~DeviceRestore() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

int32_t fedavg_multi_create(fedavg_multi** out, const int32_t* devices, int32_t num_devices, const int64_t* seg_numel,
                            int32_t num_segments, void* const* accumulators) {
  DeviceRestore restore_device;
  if (!out) return invalid("null out");
  *out = nullptr;
  if (!devices || num_devices < 1 || num_devices > FEDAVG_MULTI_MAX_DEVICES)
    return invalid("1 to FEDAVG_MULTI_MAX_DEVICES device entries are required");
  int count = 0;
  MULTI_HIP_TRY(hipGetDeviceCount(&count));
  for (int32_t g = 0; g < num_devices; ++g)
    if (devices[g] < 0 || devices[g] >= count) return invalid("device index out of range");
  auto* m = new fedavg_multi();
  m->G = num_devices;
  m->T = num_segments;
  m->devices.assign(devices, devices + num_devices);
  m->ctx.assign(m->G, nullptr);
  m->own.assign(m->G, nullptr);
  m->xstr.assign(m->G, nullptr);
  m->slots.assign(m->G, std::vector<double*>(m->G, nullptr));
  m->slot_owned.assign(m->G, std::vector<bool>(m->G, false));
  m->slot_cap.assign(m->G, 0);
  m->tab_dev.assign(m->G, nullptr);
  m->tab_host.assign(m->G, {});
  m->start_ev.assign(m->G, nullptr);
  m->done_ev.assign(m->G, nullptr);
  m->part_ev.assign(m->G, {});
  m->win_dev.assign(m->G, nullptr);
  m->win_cap.assign(m->G, 0);
  m->win_host.assign(m->G, {});
  m->comb_dev.assign(m->G, nullptr);
  m->comb_host.assign(m->G, {});
  auto bail = [&](int32_t st) {
    fedavg_multi_destroy(m);
    return st;
  };
  for (int32_t g = 0; g < m->G; ++g) {
    if (int32_t st = fedavg_ctx_create(&m->ctx[g], devices[g], seg_numel, num_segments,
                                       accumulators ? accumulators[g] : nullptr))
      return bail(st);
    hipError_t e = hipSetDevice(devices[g]);
    int lo = 0, hi = 0;
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&m->own[g], hipStreamNonBlocking);
    if (e == hipSuccess) e = hipDeviceGetStreamPriorityRange(&lo, &hi);
    if (e == hipSuccess) e = hipStreamCreateWithPriority(&m->xstr[g], hipStreamNonBlocking, hi);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&m->start_ev[g], hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&m->done_ev[g], hipEventDisableTiming);
    if (e == hipSuccess && g == 0) e = hipEventCreateWithFlags(&m->end_ev, hipEventDisableTiming);
    if (e != hipSuccess)
      return bail(fedavg_internal_fail(FEDAVG_ERR_HIP, (std::string("multi-device streams: ") + hipGetErrorString(e)).c_str()));
    m->slots[g][g] = static_cast<double*>(fedavg_accumulator(m->ctx[g]));
  }
  m->seg_numel.assign(seg_numel, seg_numel + num_segments);
  m->acc_numel = fedavg_acc_numel(m->ctx[0]);
  m->num_tiles = fedavg_num_tiles(m->ctx[0]);
  // peer mappings between distinct devices (xGMI on an MI355X node); entries on one device need none
  for (int32_t a = 0; a < m->G && m->peer_ok; ++a)
    for (int32_t b = 0; b < m->G; ++b) {
      const int da = devices[a], db = devices[b];
      if (da == db) continue;
      int can = 0;
      if (hipDeviceCanAccessPeer(&can, da, db) != hipSuccess || !can) {
        m->peer_ok = false;
        m->peer_error = "device " + std::to_string(da) + " cannot access device " + std::to_string(db);
        break;
      }
      if (hipSetDevice(da) != hipSuccess) return bail(fedavg_internal_fail(FEDAVG_ERR_HIP, "hipSetDevice"));
      const hipError_t e = hipDeviceEnablePeerAccess(db, 0);
      if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) {
        m->peer_ok = false;
        m->peer_error = std::string("hipDeviceEnablePeerAccess: ") + hipGetErrorString(e);
        break;
      }
      (void)hipGetLastError();  // clear an "already enabled"
    }
  *out = m;
  return FEDAVG_OK;
}

int32_t fedavg_multi_destroy(fedavg_multi* m) {
  DeviceRestore restore_device;
  if (!m) return FEDAVG_OK;
  for (int32_t g = 0; g < m->G; ++g) {
    (void)hipSetDevice(m->devices[g]);
    if (m->own[g]) (void)hipStreamSynchronize(m->own[g]);
    if (m->xstr[g]) (void)hipStreamSynchronize(m->xstr[g]);
  }
  if (!m->nccl.empty()) {
    FedavgRccl& r = fedavg_rccl();
    for (ncclComm_t c : m->nccl)
      if (c) (void)r.comm_destroy(c);
  }
  for (int32_t j = 0; j < m->G; ++j) {
    (void)hipSetDevice(m->devices[j]);
    for (int32_t g = 0; g < m->G; ++g)
      if (m->slot_owned[j][g] && m->slots[j][g]) (void)hipFree(m->slots[j][g]);
    if (m->tab_dev[j]) (void)hipFree(m->tab_dev[j]);
    if (m->win_dev[j]) (void)hipFree(m->win_dev[j]);
    if (m->comb_dev[j]) (void)hipFree(m->comb_dev[j]);
    for (hipEvent_t ev : m->part_ev[j]) (void)hipEventDestroy(ev);
    if (m->start_ev[j]) (void)hipEventDestroy(m->start_ev[j]);
    if (m->done_ev[j]) (void)hipEventDestroy(m->done_ev[j]);
    if (j == 0 && m->end_ev) (void)hipEventDestroy(m->end_ev);
    if (j == 0) {
      for (auto& r : m->prof_ev)
        for (hipEvent_t ev : r)
          if (ev) (void)hipEventDestroy(ev);
      for (hipEvent_t ev : m->prof_pool) (void)hipEventDestroy(ev);
    }
    if (m->own[j]) (void)hipStreamDestroy(m->own[j]);
    if (m->xstr[j]) (void)hipStreamDestroy(m->xstr[j]);
    if (m->ctx[j]) (void)fedavg_ctx_destroy(m->ctx[j]);
  }
  delete m;
  return FEDAVG_OK;
}

int32_t fedavg_multi_num_devices(const fedavg_multi* m) { return m ? m->G : -1; }

int32_t fedavg_multi_device(const fedavg_multi* m, int32_t index) {
  return (m && index >= 0 && index < m->G) ? m->devices[index] : -1;
}

fedavg_ctx* fedavg_multi_context(fedavg_multi* m, int32_t index) {
  return (m && index >= 0 && index < m->G) ? m->ctx[index] : nullptr;
}

void* fedavg_multi_stream(fedavg_multi* m, int32_t index) {
  return (m && index >= 0 && index < m->G) ? static_cast<void*>(m->own[index]) : nullptr;
}

int32_t fedavg_multi_peer_access(const fedavg_multi* m) { return (m && m->peer_ok) ? 1 : 0; }

int32_t fedavg_multi_round(fedavg_multi* m, fedavg_plan* const* partials, const double* total_weights,
                           void* const* out_ptrs, int32_t out_dtype, int32_t root, const int32_t* tile_edges,
                           int32_t num_edges, int32_t exchange, void* const* streams) {
  DeviceRestore restore_device;
  if (int32_t st = check_common(m, total_weights, out_ptrs, out_dtype, root)) return st;
  if (!partials) return invalid("null partial plan table");
  const int32_t n = m->num_tiles;
  std::vector<int32_t> edges;
  if (tile_edges) {
    if (num_edges < 2 || tile_edges[0] != 0 || tile_edges[num_edges - 1] != n)
      return invalid("tile edges must run from 0 to the context's tile count");
    for (int32_t i = 1; i < num_edges; ++i)
      if (tile_edges[i] <= tile_edges[i - 1]) return invalid("tile edges must increase");
    edges.assign(tile_edges, tile_edges + num_edges);
  } else {
    edges = {0, n};
  }
  const int32_t chunks = static_cast<int32_t>(edges.size()) - 1;
  std::vector<int32_t> members;  // entries holding clients: their partials take part
  for (int32_t g = 0; g < m->G; ++g)
    if (partials[g]) members.push_back(g);
  if (members.empty()) return fedavg_internal_fail(FEDAVG_ERR_STATE, "no device holds a client");
  if (exchange == FEDAVG_EXCHANGE_PEER) {
    if (!m->peer_ok) return invalid(("the peer exchange needs peer access: " + m->peer_error).c_str());
    if (static_cast<int32_t>(members.size()) > FEDAVG_MULTI_MAX_DEVICES) return invalid("too many devices");
    if (int32_t st = ensure_slots(m, edges)) return st;
    if (int32_t st = ensure_part_events(m, chunks)) return st;
    if (int32_t st = upload_tables(m, total_weights, out_ptrs)) return st;
    if (int32_t st = upload_windows(m, edges)) return st;
    if (int32_t st = upload_comb(m, members, chunks)) return st;
    if (int32_t st = order_round_start(m, streams)) return st;
    if (int32_t st = prof_mark(m, streams, 0)) return st;
    if (partials[0] == nullptr)
      if (int32_t st = prof_mark(m, streams, 1)) return st;  // entry 0 folds nothing
    const int32_t vec = outs_aligned(out_ptrs, m->T, out_dtype) ? 1 : 0;
    // a member with a dense plan folds its own window last, with the other members' partials of
    // it added in entry order in the same kernel (no own-window slot store and re-read)
    std::vector<int32_t> fused(m->G, 0), rank_of(m->G, -1);
    for (size_t i = 0; i < members.size(); ++i) {
      rank_of[members[i]] = static_cast<int32_t>(i);
      fused[members[i]] = fedavg_internal_plan_is_record(partials[members[i]]) ? 0 : 1;
    }
    for (int32_t k = 0; k < chunks; ++k) {
      const int64_t tb = edges[k], span = edges[k + 1] - edges[k];
      auto window = [&](int32_t j, int32_t& wb, int32_t& we) {
        wb = static_cast<int32_t>(tb + span * j / m->G);
        we = static_cast<int32_t>(tb + span * (j + 1) / m->G);
      };
      for (int32_t g : members) {
        MULTI_HIP_TRY(hipSetDevice(m->devices[g]));
        hipStream_t s = stream_of(m, streams, g);
        if (fused[g]) {
          // the chunk's other windows: each tile stores into its window owner's slot (one launch
          // on each side of the own window)
          const char* wt = m->win_dev[g];
          int32_t ob = 0, oe = 0;
          window(g, ob, oe);
          const int32_t ranges[2][2] = {{edges[k], ob}, {oe, edges[k + 1]}};
          for (const auto& r : ranges) {
            if (r[0] >= r[1]) continue;
            if (int32_t st = fedavg_internal_plan_run_windows(
                    partials[g], r[0], r[1], s, reinterpret_cast<double* const*>(wt) + static_cast<size_t>(k) * m->G,
                    reinterpret_cast<const int32_t*>(wt + sizeof(double*) * static_cast<size_t>(chunks) * m->G) +
                        k * (m->G + 1),
                    m->G))
              return st;
          }
        } else {
          for (int32_t r = 1; r <= m->G; ++r) {
            const int32_t j = (g + r) % m->G;  // quantised records: one launch per window, own last
            int32_t wb = 0, we = 0;
            window(j, wb, we);
            if (wb == we) continue;
            if (int32_t st = fedavg_internal_plan_run_range_to(partials[g], wb, we, s, rebased(m, j, g, k))) return st;
          }
        }
        MULTI_HIP_TRY(hipSetDevice(m->devices[g]));
        MULTI_HIP_TRY(hipEventRecord(m->part_ev[g][k], s));
        if (g == 0 && k == chunks - 1)
          if (int32_t st = prof_mark(m, streams, 1)) return st;
      }
      for (int32_t j = 0; j < m->G; ++j) {
        int32_t wb = 0, we = 0;
        window(j, wb, we);
        if (wb == we) continue;
        MULTI_HIP_TRY(hipSetDevice(m->devices[j]));
        if (fused[j]) {
          for (int32_t g : members)
            if (g != j) MULTI_HIP_TRY(hipStreamWaitEvent(m->xstr[j], m->part_ev[g][k], 0));
          if (int32_t st = fedavg_internal_plan_run_comb(
                  partials[j], wb, we, m->xstr[j],
                  reinterpret_cast<const double* const*>(m->comb_dev[j]) + static_cast<size_t>(k) * FEDAVG_MULTI_MAX_DEVICES,
                  static_cast<int32_t>(members.size()), rank_of[j], total_weights, out_ptrs, out_dtype))
            return st;
          continue;
        }
        for (int32_t g : members) MULTI_HIP_TRY(hipStreamWaitEvent(m->xstr[j], m->part_ev[g][k], 0));
        std::vector<const double*> src;
        for (int32_t g : members) src.push_back(rebased(m, j, g, k));
        const char* tab = m->tab_dev[j];
        if (int32_t st = fedavg_internal_multi_combine(
                m->ctx[j], wb, we, src.data(), static_cast<int32_t>(src.size()), reinterpret_cast<const double*>(tab),
                reinterpret_cast<void* const*>(tab + sizeof(double) * m->T), out_dtype, vec, m->xstr[j]))
          return st;
      }
    }
    if (int32_t st = order_round_end(m, streams)) return st;
    return prof_mark(m, streams, 2);
  }
  if (exchange == FEDAVG_EXCHANGE_REDUCE) {
    if (int32_t st = ensure_nccl(m)) return st;
    if (int32_t st = ensure_part_events(m, chunks)) return st;
    if (int32_t st = order_round_start(m, streams)) return st;
    if (int32_t st = prof_mark(m, streams, 0)) return st;
    for (int32_t k = 0; k < chunks; ++k) {
      for (int32_t g = 0; g < m->G; ++g) {
        MULTI_HIP_TRY(hipSetDevice(m->devices[g]));
        hipStream_t s = stream_of(m, streams, g);
        if (partials[g]) {
          if (int32_t st = fedavg_plan_run_range(partials[g], edges[k], edges[k + 1], s)) return st;
        } else {
          // a device without clients joins the collective with identities (-0.0)
          if (int32_t st = fedavg_partial(m->ctx[g], nullptr, FEDAVG_F32, nullptr, 0, 1, edges[k], edges[k + 1], s))
            return st;
        }
        MULTI_HIP_TRY(hipSetDevice(m->devices[g]));
        MULTI_HIP_TRY(hipEventRecord(m->part_ev[g][k], s));
        MULTI_HIP_TRY(hipStreamWaitEvent(m->xstr[g], m->part_ev[g][k], 0));
        if (g == 0 && k == chunks - 1)
          if (int32_t st = prof_mark(m, streams, 1)) return st;
      }
      int64_t a = 0, b = 0;
      if (int32_t st = fedavg_tile_range(m->ctx[0], edges[k], edges[k + 1], &a, &b)) return st;
      if (int32_t st = grouped_reduce(m, a, b, root)) return st;
    }
    if (int32_t st = root_finalize(m, total_weights, out_ptrs, out_dtype, root)) return st;
    if (int32_t st = order_round_end(m, streams)) return st;
    return prof_mark(m, streams, 2);
  }
  return invalid("exchange must be FEDAVG_EXCHANGE_PEER or FEDAVG_EXCHANGE_REDUCE");
}

int32_t fedavg_multi_combine(fedavg_multi* m, const double* total_weights, void* const* out_ptrs, int32_t out_dtype,
                             int32_t root, int32_t exchange, void* const* streams) {
  DeviceRestore restore_device;
  if (int32_t st = check_common(m, total_weights, out_ptrs, out_dtype, root)) return st;
  // which entries folded which segments (fed_avg_algorithm.py:55-62: a name the shard never saw)
  std::vector<std::vector<int32_t>> valid(m->G, std::vector<int32_t>(m->T, 0));
  for (int32_t g = 0; g < m->G; ++g) fedavg_internal_segment_valid(m->ctx[g], valid[g].data());
  std::vector<int32_t> members;
  for (int32_t g = 0; g < m->G; ++g)
    if (std::any_of(valid[g].begin(), valid[g].end(), [](int32_t v) { return v != 0; })) members.push_back(g);
  for (int32_t t = 0; t < m->T; ++t) {
    bool any = false;
    for (int32_t g : members) any = any || valid[g][t];
    if (!any)
      return fedavg_internal_fail(FEDAVG_ERR_STATE,
                                  ("segment " + std::to_string(t) + " has no accumulated data (fed_avg_algorithm.py:88)").c_str());
  }
  if (exchange == FEDAVG_EXCHANGE_PEER && !m->peer_ok)
    return invalid(("the peer exchange needs peer access: " + m->peer_error).c_str());
  if (exchange != FEDAVG_EXCHANGE_PEER && exchange != FEDAVG_EXCHANGE_REDUCE)
    return invalid("exchange must be FEDAVG_EXCHANGE_PEER or FEDAVG_EXCHANGE_REDUCE");
  if (exchange == FEDAVG_EXCHANGE_REDUCE)
    if (int32_t st = ensure_nccl(m)) return st;
  if (exchange == FEDAVG_EXCHANGE_PEER)
    if (int32_t st = upload_tables(m, total_weights, out_ptrs)) return st;
  // a segment an entry never folded holds stale data: the identity -0.0 (a zero-client partial),
  // on the entry's stream before the exchange reads it; under REDUCE every entry takes part
  const std::vector<int32_t> parts = (exchange == FEDAVG_EXCHANGE_REDUCE) ? [&] {
    std::vector<int32_t> all(m->G);
    for (int32_t g = 0; g < m->G; ++g) all[g] = g;
    return all;
  }() : members;
  for (int32_t g : parts)
    for (int32_t t = 0; t < m->T; ++t) {
      if (valid[g][t]) continue;
      int32_t tb = 0, te = 0;
      if (int32_t st = fedavg_internal_segment_tiles(m->ctx[g], t, &tb, &te)) return st;
      if (int32_t st = fedavg_partial(m->ctx[g], nullptr, FEDAVG_F32, nullptr, 0, 1, tb, te, stream_of(m, streams, g)))
        return st;
    }
  if (int32_t st = order_round_start(m, streams)) return st;
  if (exchange == FEDAVG_EXCHANGE_REDUCE) {
    if (int32_t st = grouped_reduce(m, 0, m->acc_numel, root)) return st;
    if (int32_t st = root_finalize(m, total_weights, out_ptrs, out_dtype, root)) return st;
  } else {
    // every entry's accumulator is read in place by the window's owner (peer loads)
    std::vector<const double*> src;
    for (int32_t g : members) src.push_back(static_cast<const double*>(fedavg_accumulator(m->ctx[g])));
    const int32_t vec = outs_aligned(out_ptrs, m->T, out_dtype) ? 1 : 0;
    for (int32_t j = 0; j < m->G; ++j) {
      const int32_t wb = static_cast<int32_t>(static_cast<int64_t>(m->num_tiles) * j / m->G);
      const int32_t we = static_cast<int32_t>(static_cast<int64_t>(m->num_tiles) * (j + 1) / m->G);
      if (wb == we) continue;
      MULTI_HIP_TRY(hipSetDevice(m->devices[j]));
      const char* tab = m->tab_dev[j];
      if (int32_t st = fedavg_internal_multi_combine(
              m->ctx[j], wb, we, src.data(), static_cast<int32_t>(src.size()), reinterpret_cast<const double*>(tab),
              reinterpret_cast<void* const*>(tab + sizeof(double) * m->T), out_dtype, vec, m->xstr[j]))
        return st;
    }
  }
  for (int32_t g = 0; g < m->G; ++g) fedavg_internal_clear_state(m->ctx[g]);
  return order_round_end(m, streams);
}

int32_t fedavg_multi_check(fedavg_multi* m, uint32_t* flags_out) {
  DeviceRestore restore_device;
  if (!m) return invalid("null multi-device object");
  uint32_t f = 0;
  for (int32_t g = 0; g < m->G; ++g) {
    MULTI_HIP_TRY(hipSetDevice(m->devices[g]));
    MULTI_HIP_TRY(hipStreamSynchronize(m->own[g]));
    MULTI_HIP_TRY(hipStreamSynchronize(m->xstr[g]));
    if (m->any_round) MULTI_HIP_TRY(hipEventSynchronize(m->done_ev[g]));
  }
  for (int32_t g = 0; g < m->G; ++g) f |= fedavg_internal_flags(m->ctx[g], 0);
  if (flags_out) *flags_out = f;
  if (f & FEDAVG_FLAG_ACC_NAN) return fedavg_internal_fail(FEDAVG_ERR_NAN_ACCUM, "NaN in the accumulator");
  if (f & FEDAVG_FLAG_RESULT_NAN) return fedavg_internal_fail(FEDAVG_ERR_NAN_RESULT, "NaN in the aggregated result");
  return FEDAVG_OK;
}

int32_t fedavg_multi_round_check(fedavg_multi* m, uint32_t* flags_out) {
  DeviceRestore restore_device;
  if (!m) return invalid("null multi-device object");
  if (!m->any_round) return fedavg_multi_check(m, flags_out);
  // the NaN words are host-coherent pinned memory the kernels store into at system scope: once
  // the round's end event completed, every store of the round is visible here
  MULTI_HIP_TRY(hipSetDevice(m->devices[0]));
  MULTI_HIP_TRY(hipEventSynchronize(m->end_ev));
  uint32_t f = 0;
  for (int32_t g = 0; g < m->G; ++g) f |= fedavg_internal_flags(m->ctx[g], 0);
  if (flags_out) *flags_out = f;
  if (f & FEDAVG_FLAG_ACC_NAN) return fedavg_internal_fail(FEDAVG_ERR_NAN_ACCUM, "NaN in the accumulator");
  if (f & FEDAVG_FLAG_RESULT_NAN) return fedavg_internal_fail(FEDAVG_ERR_NAN_RESULT, "NaN in the aggregated result");
  return FEDAVG_OK;
}

int32_t fedavg_multi_prof_enable(fedavg_multi* m, int32_t on) {
  if (!m) return invalid("null multi-device object");
  m->prof = on != 0;
  return FEDAVG_OK;
}

int32_t fedavg_multi_prof_collect(fedavg_multi* m, double* fold_ms, double* tail_ms, int32_t* rounds) {
  DeviceRestore restore_device;
  if (!m) return invalid("null multi-device object");
  double fold = 0.0, tail = 0.0;
  int32_t n = 0;
  MULTI_HIP_TRY(hipSetDevice(m->devices[0]));
  for (auto& r : m->prof_ev) {
    if (!r[0] || !r[1] || !r[2]) continue;  // a round that failed while enqueuing
    MULTI_HIP_TRY(hipEventSynchronize(r[2]));
    float a = 0.f, b = 0.f;
    MULTI_HIP_TRY(hipEventElapsedTime(&a, r[0], r[1]));
    MULTI_HIP_TRY(hipEventElapsedTime(&b, r[1], r[2]));
    fold += a;
    tail += b;
    ++n;
  }
  for (auto& r : m->prof_ev)
    for (hipEvent_t ev : r)
      if (ev) m->prof_pool.push_back(ev);
  m->prof_ev.clear();
  if (fold_ms) *fold_ms = fold;
  if (tail_ms) *tail_ms = tail;
  if (rounds) *rounds = n;
  return FEDAVG_OK;
}

int32_t fedavg_multi_reset(fedavg_multi* m) {
  DeviceRestore restore_device;
  if (!m) return invalid("null multi-device object");
  for (int32_t g = 0; g < m->G; ++g) {
    MULTI_HIP_TRY(hipSetDevice(m->devices[g]));
    MULTI_HIP_TRY(hipStreamSynchronize(m->own[g]));
    MULTI_HIP_TRY(hipStreamSynchronize(m->xstr[g]));
    fedavg_internal_clear_state(m->ctx[g]);
    (void)fedavg_internal_flags(m->ctx[g], 1);
  }
  return FEDAVG_OK;
}

}  // extern "C"
