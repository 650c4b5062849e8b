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


@pytest.fixture(scope="session")
def harness():
    import ctypes as C
    deps = [HARNESS_SRC] + [os.path.join(ROOT, "orbslam3lib_amd", "csrc", f)
                            for f in os.listdir(os.path.join(ROOT, "orbslam3lib_amd", "csrc"))]
    if not os.path.exists(HARNESS_LIB) or any(os.path.getmtime(d) > os.path.getmtime(HARNESS_LIB)
                                              for d in deps):
        os.makedirs(os.path.dirname(HARNESS_LIB), exist_ok=True)
        subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O2", "-std=c++17",
                               "-fPIC", "-ffp-contract=off", "-shared", "-o", HARNESS_LIB,
                               HARNESS_SRC])
    lib = C.CDLL(HARNESS_LIB)
    lib.harness_fast_atan2.restype = C.c_float
    lib.harness_fast_atan2.argtypes = [C.c_float, C.c_float]
    return lib
