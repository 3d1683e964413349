// pt_rccl.cpp -- run-time binding of RCCL (see pt_rccl.h).
#include "pt_rccl.h"

#include <dlfcn.h>

namespace pt {

namespace {

Rccl load() {
  Rccl r;
  void* h = nullptr;
  // an RCCL already in the process (PyTorch-ROCm's) first, so the gather runs on
  // the same RCCL and HIP runtime as the rest of the process; then the system one
  const char* names[] = {"librccl.so.1", "librccl.so"};
  for (const char* n : names)
    if (!h && (h = dlopen(n, RTLD_NOW | RTLD_NOLOAD))) r.path = std::string(n) + " (already loaded)";
  const char* paths[] = {"librccl.so.1", "/opt/rocm/lib/librccl.so.1"};
  for (const char* p : paths)
    if (!h && (h = dlopen(p, RTLD_NOW | RTLD_LOCAL))) r.path = p;
  if (!h) {
    const char* e = dlerror();
    r.err = std::string("RCCL not found: ") + (e ? e : "dlopen failed");
    return r;
  }
  auto sym = [&](const char* name) { return dlsym(h, name); };
  r.commInitAll = reinterpret_cast<decltype(r.commInitAll)>(sym("ncclCommInitAll"));
  r.commDestroy = reinterpret_cast<decltype(r.commDestroy)>(sym("ncclCommDestroy"));
  r.groupStart = reinterpret_cast<decltype(r.groupStart)>(sym("ncclGroupStart"));
  r.groupEnd = reinterpret_cast<decltype(r.groupEnd)>(sym("ncclGroupEnd"));
  r.send = reinterpret_cast<decltype(r.send)>(sym("ncclSend"));
  r.recv = reinterpret_cast<decltype(r.recv)>(sym("ncclRecv"));
  r.errorString = reinterpret_cast<decltype(r.errorString)>(sym("ncclGetErrorString"));
  r.ok = r.commInitAll && r.commDestroy && r.groupStart && r.groupEnd && r.send && r.recv && r.errorString;
  if (!r.ok) r.err = "RCCL at " + r.path + " lacks an entry point";
  return r;
}

}  // namespace

const Rccl& rccl() {
  static const Rccl r = load();
  return r;
}

}  // namespace pt
