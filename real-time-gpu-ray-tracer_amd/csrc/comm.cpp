// comm.cpp — run-time resolution of the RCCL entry points (see comm.hpp).
#include "comm.hpp"

#include <dlfcn.h>

#include <cstdlib>

namespace rtamd {
namespace {

Rccl load() {
    Rccl r;
    void *h = nullptr;
    // RTAMD_RCCL_LIB: an explicit RCCL build (tests/fake_rccl: an N-rank world inside one process, so the world > 1
    // gather runs on a one-GPU box); it must load, no fallback
    if (const char *path = std::getenv("RTAMD_RCCL_LIB")) {
        if (*path) {
            h = dlopen(path, RTLD_NOW | RTLD_LOCAL);
            if (!h) {
                const char *e = dlerror();
                r.error = std::string("cannot load RTAMD_RCCL_LIB=") + path + ": " + (e ? e : "not found");
                return r;
            }
        }
    }
    // an RCCL the process already holds (e.g. PyTorch's), else ROCm's
    for (const char *name : {"librccl.so.1", "librccl.so"}) {
        if (h) break;
        h = dlopen(name, RTLD_NOW | RTLD_NOLOAD);
        if (h) break;
    }
    for (const char *name : {"librccl.so.1", "/opt/rocm/lib/librccl.so.1", "librccl.so"}) {
        if (h) break;
        h = dlopen(name, RTLD_NOW | RTLD_LOCAL);
    }
    if (!h) {
        const char *e = dlerror();
        r.error = std::string("cannot load librccl.so.1: ") + (e ? e : "not found");
        return r;
    }
    bool ok = true;
    auto sym = [&](auto &fn, const char *name) {
        fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(h, name));
        if (!fn) {
            ok = false;
            r.error += std::string(r.error.empty() ? "" : ", ") + "missing " + name;
        }
    };
    sym(r.GetUniqueId, "ncclGetUniqueId");
    sym(r.CommInitRank, "ncclCommInitRank");
    sym(r.CommSplit, "ncclCommSplit");
    sym(r.CommDestroy, "ncclCommDestroy");
    sym(r.CommAbort, "ncclCommAbort");
    sym(r.CommGetAsyncError, "ncclCommGetAsyncError");
    sym(r.GroupStart, "ncclGroupStart");
    sym(r.GroupEnd, "ncclGroupEnd");
    sym(r.Send, "ncclSend");
    sym(r.Recv, "ncclRecv");
    sym(r.GetErrorString, "ncclGetErrorString");
    r.ok = ok;
    return r;
}

}  // namespace

const Rccl &rccl() {
    static const Rccl r = load();
    return r;
}

}  // namespace rtamd
