"""Bounded waits of multi-GPU frames (rt_comm_set_timeout, csrc/comm_wait.hpp): the polling policy the
library runs instead of blocking in hipStreamSynchronize on a frame whose RCCL gather may never complete
(SURVEY §5 failure row: RCCL errors surface as status codes; the reference exit()s, Global.cu:34-41).
The policy header is compiled with g++ against fake completion / RCCL state sources: a communicator stuck
in ncclInProgress, an asynchronous error, a device error, a frame that completes.  CPU only."""
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "real-time-gpu-ray-tracer_amd", "csrc")

DRIVER = r'''
#include "comm_wait.hpp"
#include <chrono>
#include <cstdio>
using namespace rtamd;
static const char *name(WaitResult w) {
    return w == WaitResult::done ? "done" : w == WaitResult::failed ? "failed" : w == WaitResult::async_error ? "async" : "timeout";
}
int main() {
    // fake RCCL table: per communicator the state ncclCommGetAsyncError reports, and the call's own status
    int state[3] = {NCCL_IN_PROGRESS, NCCL_SUCCESS, NCCL_IN_PROGRESS};
    int call[3] = {0, 0, 0};
    auto get = [&](int q, int *st) { *st = state[q]; return call[q]; };
    auto async = [&] { return first_async_error(3, get); };
    int polls = 0, code = 0;
    // 1. a frame that completes after 5 polls, communicators in progress: done
    WaitResult w = poll_wait([&] { return ++polls >= 5 ? 1 : 0; }, async, 1000, &code);
    std::printf("complete %s %d\n", name(w), polls);
    // 2. never completes, every communicator stays ncclInProgress: the 40 ms deadline
    auto t0 = std::chrono::steady_clock::now();
    w = poll_wait([] { return 0; }, async, 40, &code);
    long ms = (long)std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now() - t0).count();
    std::printf("stuck %s %ld\n", name(w), ms);
    // 3. communicator 2 reports ncclRemoteError (6): async error, no deadline needed
    state[2] = 6;
    w = poll_wait([] { return 0; }, async, 0, &code);
    std::printf("peer %s %d\n", name(w), code);
    // 4. the state query itself fails on communicator 2: not an error report
    call[2] = 3;
    std::printf("query_failed %d\n", first_async_error(3, get));
    // 5. the device wait fails: failed
    state[2] = NCCL_IN_PROGRESS; call[2] = 0;
    w = poll_wait([] { return -1; }, async, 0, &code);
    std::printf("device %s\n", name(w));
    return 0;
}
'''


@pytest.fixture(scope="module")
def results(tmp_path_factory):
    d = tmp_path_factory.mktemp("commwait")
    src = d / "drv.cpp"
    src.write_text(DRIVER)
    exe = d / "drv"
    subprocess.run(["g++", "-std=c++17", "-O1", "-pthread", "-I", CSRC, "-o", str(exe), str(src)], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True, timeout=30).stdout
    return {line.split()[0]: line.split()[1:] for line in out.strip().splitlines()}


def test_completion_is_done(results):
    assert results["complete"] == ["done", "5"]


def test_in_progress_forever_times_out(results):
    kind, ms = results["stuck"]
    assert kind == "timeout" and 40 <= int(ms) < 1000


def test_async_error_aborts_without_deadline(results):
    assert results["peer"] == ["async", "6"]


def test_failed_state_query_is_not_an_error(results):
    assert results["query_failed"] == ["0"]


def test_device_failure(results):
    assert results["device"] == ["failed"]
