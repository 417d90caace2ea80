// comm.hpp — RCCL (= NCCL API on ROCm) entry points the multi-GPU frame uses, resolved at run time.
//
// The reference is single-GPU (no NCCL/MPI anywhere); the screen-tile gather over xGMI is new
// (SURVEY §5, §8e).  librtamd.so does not link librccl: a single-GPU caller never needs it, and a
// process that already holds an RCCL (PyTorch ships one) must not load a second copy.  The first
// rt_comm_* / rt_scene_attach_comm call resolves the symbols from the RCCL already loaded in the process
// (RTLD_NOLOAD), else loads librccl.so.1 (ROCm's, /opt/rocm/lib).
#pragma once
#include <rccl/rccl.h>

#include <string>

namespace rtamd {

struct Rccl {
    bool ok = false;
    std::string error;                   // why loading failed
    decltype(&ncclGetUniqueId) GetUniqueId = nullptr;
    decltype(&ncclCommInitRank) CommInitRank = nullptr;
    decltype(&ncclCommSplit) CommSplit = nullptr;
    decltype(&ncclCommDestroy) CommDestroy = nullptr;
    decltype(&ncclCommAbort) CommAbort = nullptr;
    decltype(&ncclCommGetAsyncError) CommGetAsyncError = nullptr;
    decltype(&ncclGroupStart) GroupStart = nullptr;
    decltype(&ncclGroupEnd) GroupEnd = nullptr;
    decltype(&ncclSend) Send = nullptr;
    decltype(&ncclRecv) Recv = nullptr;
    decltype(&ncclGetErrorString) GetErrorString = nullptr;
};

// The process-wide table (loaded once, thread-safe).
const Rccl &rccl();

}  // namespace rtamd
