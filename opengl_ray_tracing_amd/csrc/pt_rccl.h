// pt_rccl.h -- RCCL entry points the in-process multi-GPU gather uses
// (pt_runtime.cpp, pt_config.n_devices > 1), resolved at run time so libpt.so
// has no link-time RCCL dependency and, inside a PyTorch process, shares the
// RCCL PyTorch already loaded (one RCCL, one HIP runtime per process).
#pragma once
#include <rccl/rccl.h>

#include <string>

namespace pt {

struct Rccl {
  decltype(&ncclCommInitAll) commInitAll = nullptr;
  decltype(&ncclCommDestroy) commDestroy = nullptr;
  decltype(&ncclGroupStart) groupStart = nullptr;
  decltype(&ncclGroupEnd) groupEnd = nullptr;
  decltype(&ncclSend) send = nullptr;
  decltype(&ncclRecv) recv = nullptr;
  decltype(&ncclGetErrorString) errorString = nullptr;
  bool ok = false;
  std::string err;   // why it could not be loaded
  std::string path;  // which library serves it
};

// The process's RCCL (loaded on first use; ok == false if it cannot be found).
const Rccl& rccl();

}  // namespace pt
