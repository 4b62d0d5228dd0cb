// rccl_bind.h — the RCCL entry points the library uses, bound at run time (sharded_comm.cpp).
//
// RCCL is not linked: the library binds the RCCL the process already has (torch's, by SONAME
// librccl.so.1) or loads it, the first time a communicator is made. FEDAVG_RCCL_LIB names a
// library to load instead (test stand-ins: tests/native/fake_rccl.cpp). rccl.h supplies the types.
#pragma once

#include <rccl/rccl.h>

#include <string>

struct FedavgRccl {
  void* handle = nullptr;
  decltype(&ncclGetUniqueId) get_unique_id = nullptr;
  decltype(&ncclCommInitRank) comm_init_rank = nullptr;
  decltype(&ncclCommInitAll) comm_init_all = nullptr;  // single-process communicators (multi_device.cpp)
  decltype(&ncclCommDestroy) comm_destroy = nullptr;
  decltype(&ncclReduce) reduce = nullptr;
  decltype(&ncclReduceScatter) reduce_scatter = nullptr;
  decltype(&ncclGroupStart) group_start = nullptr;
  decltype(&ncclGroupEnd) group_end = nullptr;
  decltype(&ncclGather) gather = nullptr;  // RCCL extension; grouped send / recv when absent
  decltype(&ncclSend) send = nullptr;
  decltype(&ncclRecv) recv = nullptr;
  decltype(&ncclGetErrorString) error_string = nullptr;
  std::string error;  // non-empty: RCCL is unusable (why)
};

// The process-wide binding (bound once, thread-safe).
__attribute__((visibility("hidden"))) FedavgRccl& fedavg_rccl();
// FEDAVG_OK, or FEDAVG_ERR_RCCL with the binding's error as the last error.
__attribute__((visibility("hidden"))) int32_t fedavg_rccl_ready();
// FEDAVG_ERR_RCCL with "<what>: <RCCL's error string>" as the last error.
__attribute__((visibility("hidden"))) int32_t fedavg_rccl_fail(ncclResult_t res, const char* what);
