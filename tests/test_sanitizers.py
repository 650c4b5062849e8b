"""The oracle under AddressSanitizer + UndefinedBehaviorSanitizer (host code only; GPU sanitizers
are not available on this pool).  `make -C oracle asan` builds liborb_oracle_asan.so; a child
Python process preloads the ASan runtime, loads that build in place of the default one and runs
the oracle entry points the tests use (extraction with both lapping-area forms, per-level
keypoints, pyramid and blur, kNN2 with ties and empty train sets, the stereo matcher, the fisheye
triangulation, the thread pool).  Any sanitizer report makes the child exit non-zero."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import sys, numpy as np
sys.path.insert(0, ROOT)
from oracle import oracle_py as o
from orbslam3lib_amd import synth
o._load(ROOT + "/oracle/build/liborb_oracle_asan.so")
L, R = synth.stereo_pair(240, 320, 3)
for lap in ((0, 0), (40, 200)):
    k, d, m = o.extract(L, nfeatures=500, lap=lap)
    assert len(k) > 0
lv = o.extract_levels(L, nfeatures=500)
pyr = o.pyramid(L)
o.blur(pyr[0])
kl, dl, ml = o.extract(L, nfeatures=500, lap=(0, 320))
kr, dr, mr = o.extract(R, nfeatures=500, lap=(0, 320))
i1, d1, i2, d2 = o.knn2(dl, dr)
o.knn2(dl, dr[:0]); o.knn2(dl[:0], dr); o.knn2(np.concatenate([dl, dl]), dl[:1])
o.stereo_matches(kl, dl, kr, dr, o.pyramid(L), o.pyramid(R), 47.9, 0.11)
rig = dict(cam_left=[190.0, 190.0, 160.0, 120.0, 0.0035, 0.0007, -0.002, 0.0002],
           cam_right=[190.0, 190.0, 160.0, 120.0, 0.0035, 0.0007, -0.002, 0.0002],
           R12=np.eye(3, dtype=np.float32), t12=[0.1, 0.0, 0.0])
s2 = (1.2 ** (2 * np.arange(8))).astype(np.float32)
o.fisheye_stereo(kl, ml, kr, mr, i1, d1, rig, s2)
o.extract_many(np.stack([L, R, L]), 3, nfeatures=300)
print("asan-ok")
"""


def _asan_runtime():
    try:
        p = subprocess.check_output(["gcc", "-print-file-name=libasan.so"], text=True).strip()
    except (OSError, subprocess.CalledProcessError):
        return None
    return p if os.path.isabs(p) and os.path.exists(p) else None


def test_oracle_under_asan_ubsan():
    rt = _asan_runtime()
    if rt is None:
        pytest.skip("no libasan runtime")
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "asan"])
    env = dict(os.environ)
    env["LD_PRELOAD"] = rt
    env["ASAN_OPTIONS"] = "detect_leaks=0:halt_on_error=1:abort_on_error=1"
    env["UBSAN_OPTIONS"] = "halt_on_error=1:print_stacktrace=1"
    r = subprocess.run([sys.executable, "-c", CHILD.replace("ROOT", repr(ROOT))], env=env,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0 and "asan-ok" in r.stdout, (r.stdout[-2000:], r.stderr[-4000:])


def _clang_asan_runtime():
    import glob
    c = sorted(glob.glob("/opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so"))
    return c[-1] if c else None


def test_host_harness_under_asan_ubsan():
    """The device algorithms' SerialPolicy instantiations (octree, FAST cell, introsorts,
    fastAtan2, sincosf) built with host ASan + UBSan (hipcc: -Xarch_host -fsanitize=...) and run
    through tests/test_host_harness.py in a child pytest with the clang ASan runtime preloaded."""
    rt = _clang_asan_runtime()
    if rt is None:
        pytest.skip("no clang ASan runtime")
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from conftest import build_harness
    build_harness(asan=True)
    env = dict(os.environ)
    env["LD_PRELOAD"] = rt
    env["ORBGPU_HARNESS_ASAN"] = "1"
    env["ASAN_OPTIONS"] = "detect_leaks=0:halt_on_error=1:abort_on_error=1"
    env["UBSAN_OPTIONS"] = "halt_on_error=1:print_stacktrace=1"
    r = subprocess.run([sys.executable, "-m", "pytest", "-x", "-q", "-p", "no:cacheprovider",
                        os.path.join(ROOT, "tests", "test_host_harness.py")], env=env, cwd=ROOT,
                       capture_output=True, text=True, timeout=1200)
    assert r.returncode == 0 and " passed" in r.stdout, (r.stdout[-3000:], r.stderr[-3000:])
