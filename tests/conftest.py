import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

HARNESS_SRC = os.path.join(ROOT, "tests", "harness", "host_harness.hip")
HARNESS_LIB = os.path.join(ROOT, "tests", "harness", "build", "libhost_harness.so")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) device")


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle_py
    oracle_py.lib()
    return oracle_py


def build_harness(asan=False):
    """The SerialPolicy host harness (tests/harness/host_harness.hip); asan: host code built with
    AddressSanitizer + UndefinedBehaviorSanitizer (clang runtime, preloaded by the caller)."""
    lib_path = HARNESS_LIB.replace(".so", "_asan.so") if asan else HARNESS_LIB
    deps = [HARNESS_SRC] + [os.path.join(ROOT, "orbslam3lib_amd", "csrc", f)
                            for f in os.listdir(os.path.join(ROOT, "orbslam3lib_amd", "csrc"))]
    if not os.path.exists(lib_path) or any(os.path.getmtime(d) > os.path.getmtime(lib_path)
                                           for d in deps):
        os.makedirs(os.path.dirname(lib_path), exist_ok=True)
        san = ["-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined",
               "-fno-omit-frame-pointer", "-g"] if asan else []
        subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O2", "-std=c++17",
                               "-fPIC", "-ffp-contract=off"] + san + ["-shared", "-o", lib_path,
                                                                      HARNESS_SRC])
    return lib_path


@pytest.fixture(scope="session")
def harness():
    import ctypes as C
    lib = C.CDLL(build_harness(asan=os.environ.get("ORBGPU_HARNESS_ASAN") == "1"))
    lib.harness_fast_atan2.restype = C.c_float
    lib.harness_fast_atan2.argtypes = [C.c_float, C.c_float]
    return lib
