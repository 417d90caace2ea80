"""Test configuration: paths, the `gpu` marker, and build fixtures.

`-m "not gpu"` tests run on CPU (oracle, host logic, ABI exports, gloo multi-process).
`-m gpu` tests run the HIP path through the C ABI and compare it with the oracle.
"""
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "real-time-gpu-ray-tracer_amd")
for p in (REPO, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path through librtamd.so)")


@pytest.fixture(scope="session")
def oracle_lib():
    from oracle import oracle
    oracle.build()
    return oracle


def pytest_report_header(config):
    """Which library this run tests: its hash, the hash of the sources it was built from, the git HEAD
    that built it (rtamd/provenance.py; the GPU box's copy of the tree has no .git)."""
    from rtamd import provenance
    ok, msg = provenance.check()
    return [("tested " if ok else "PROVENANCE MISMATCH (rebuilt by the rtlib_path fixture): ") + msg]


@pytest.fixture(scope="session")
def rtlib_path():
    """Path of librtamd.so, built from the sources in this tree: (re)built when missing or when its build
    stamp does not match the library or the sources (hipcc cross-compiles without a GPU)."""
    from rtamd import abi, provenance
    if not os.path.exists(abi.LIB_PATH) or not provenance.check()[0]:
        subprocess.run(["make", "-s", "-j4", "-C", os.path.join(PKG, "csrc")], check=True)
    ok, msg = provenance.check()
    assert ok, msg
    print(f"\n[provenance] {msg}", flush=True)
    return abi.LIB_PATH


@pytest.fixture(scope="session")
def gpu_lib(rtlib_path):
    """librtamd.so on a GPU box; fails loudly (never skips to a fallback) if no device is visible."""
    import torch  # noqa: F401  (load torch's HIP runtime first so both share one runtime)
    from rtamd import abi
    lib = abi.load_library()
    n = lib.rt_device_count()
    assert n > 0, "gpu test collected but no HIP device is visible"
    return lib
