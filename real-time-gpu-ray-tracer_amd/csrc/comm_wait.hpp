// comm_wait.hpp — bounded waits for multi-GPU frames (rt_comm_set_timeout).
//
// A frame that gathers over RCCL can block forever when a peer dies: the reference has no multi-GPU code
// and exits on any error (src/Global/Global.cu:34-41); SURVEY §5 asks for RCCL errors as status codes.
// Every wait the library does on such a frame polls instead of blocking: the frame's completion, the
// communicators' asynchronous error state (ncclCommGetAsyncError: ncclInProgress / ncclSuccess mean "no
// error yet"), and an optional deadline.  Header-only and free of HIP / RCCL types so that the policy is
// unit-tested on the CPU with fake completion and error sources (tests/test_comm_wait.py).
#pragma once
#include <chrono>
#include <cstdint>
#include <thread>

namespace rtamd {

enum class WaitResult { done, failed, async_error, timeout };

// done():  1 = complete, 0 = still running, -1 = the wait itself failed (device error)
// async(): 0 = no asynchronous communicator error, else the error code (reported in *code)
template <class Done, class Async>
WaitResult poll_wait(Done &&done, Async &&async, uint32_t timeout_ms, int *code = nullptr) {
    using clock = std::chrono::steady_clock;
    const auto t0 = clock::now();
    auto next_async = t0;                           // the communicators' state: first poll, then every 100 us
    for (;;) {
        const int d = done();
        if (d > 0) return WaitResult::done;
        if (d < 0) return WaitResult::failed;
        const auto now = clock::now();
        if (now >= next_async) {
            const int e = async();
            if (e != 0) {
                if (code) *code = e;
                return WaitResult::async_error;
            }
            next_async = now + std::chrono::microseconds(100);
        }
        if (timeout_ms && now - t0 >= std::chrono::milliseconds(timeout_ms)) return WaitResult::timeout;
        // most waits end within a frame (0.05-20 ms) and a pipelined host waits often: spin on the completion
        // for the first 2 ms (a 50 us sleep from the first spins made the world-1 comm path 0.17 -> 0.28 ms per
        // frame), then yield the core in 20 us steps
        if (now - t0 >= std::chrono::milliseconds(2)) std::this_thread::sleep_for(std::chrono::microseconds(20));
        else std::this_thread::yield();
    }
}

// The communicators' asynchronous state (ncclCommGetAsyncError): ncclSuccess (0) and ncclInProgress (7,
// non-blocking communicators while an operation runs) are "no error"; anything else is the first error.
// get(q, &state) returns the call's own status (0 = the state is valid).
constexpr int NCCL_SUCCESS = 0, NCCL_IN_PROGRESS = 7;
template <class Get>
int first_async_error(int ncomm, Get &&get) {
    for (int q = 0; q < ncomm; q++) {
        int st = NCCL_SUCCESS;
        if (get(q, &st) == NCCL_SUCCESS && st != NCCL_SUCCESS && st != NCCL_IN_PROGRESS) return st;
    }
    return 0;
}

}  // namespace rtamd
