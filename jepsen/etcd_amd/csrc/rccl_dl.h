// rccl_dl.h — the RCCL entry points the frontier exchange uses, resolved at
// run time (dlopen of librccl), so liblincheck.so still loads — and every
// single-GPU path runs — on a host without RCCL.  Only the types come from
// <rccl/rccl.h>; nothing links against librccl.
#pragma once

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <string>

struct RcclApi {
  decltype(&ncclGetUniqueId) GetUniqueId = nullptr;
  decltype(&ncclCommInitAll) CommInitAll = nullptr;
  decltype(&ncclCommInitRank) CommInitRank = nullptr;
  decltype(&ncclCommDestroy) CommDestroy = nullptr;
  decltype(&ncclCommAbort) CommAbort = nullptr;
  decltype(&ncclGroupStart) GroupStart = nullptr;
  decltype(&ncclGroupEnd) GroupEnd = nullptr;
  decltype(&ncclSend) Send = nullptr;
  decltype(&ncclRecv) Recv = nullptr;
  decltype(&ncclAllReduce) AllReduce = nullptr;
  decltype(&ncclAllToAll) AllToAll = nullptr;
  decltype(&ncclGetErrorString) GetErrorString = nullptr;
  bool ok = false;
  std::string err;  // why it is not usable (ok == false)
};

// Loaded once per process (thread-safe); check .ok before use.
const RcclApi &rccl_api();
