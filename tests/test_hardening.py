"""CPU: the product library's guards (no device compute).

* Measurement knobs (ORBGPU_STREAMS, ORBGPU_OCT_SPLIT, ...) change launch shapes and kernel
  variants; liborbgpu.so honours them only under ORBGPU_DIAGNOSTICS=1, so a stray variable in a
  deployment never changes the kernel path (orbgpu_diagnostic_knobs reports what is in effect).
* Two HIP runtimes in one process (liborbgpu.so mapped /opt/rocm's libamdhip64 first, torch then
  loaded its bundled copy by path): orbgpu_create and the batch entry points refuse with
  ORBGPU_ERR_RUNTIME instead of letting torch run device-less.
Each case runs in a child process: the environment and the mapped libraries are process state.
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_KNOBS = """
import json, orbslam3lib_amd as og
print(json.dumps(og.diagnostic_knobs()))
"""

_RUNTIMES = """
import ctypes as C, json, sys
torch_first = sys.argv[1] == "torch_first"
if torch_first:
    import torch
import orbslam3lib_amd as og
lib = og.load_library()
if not torch_first:
    import torch  # loads torch/lib/libamdhip64.so by path beside /opt/rocm's copy
maps = sorted({l.split()[-1] for l in open("/proc/self/maps") if "libamdhip64" in l})
p = og._Params(1000, 1.2, 8, 20, 7)
h = C.c_void_p()
r = lib.orbgpu_create(C.byref(p), 0, 640, 480, 2, C.byref(h))
err = lib.orbgpu_last_error().decode()
if r == 0:
    lib.orbgpu_destroy(h)
print(json.dumps({"maps": maps, "create": r, "error": err}))
"""


def _child(code, env_extra=None, args=()):
    env = {k: v for k, v in os.environ.items() if not k.startswith("ORBGPU_")}
    env.update(env_extra or {})
    env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
    out = subprocess.run([sys.executable, "-c", code] + list(args), cwd=ROOT, env=env, capture_output=True,
                         text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    return json.loads(out.stdout.strip().splitlines()[-1])


def test_knobs_ignored_without_the_diagnostics_gate():
    knobs = {"ORBGPU_STREAMS": "1", "ORBGPU_OCT_SPLIT": "3", "ORBGPU_FAST_PITCH": "80", "ORBGPU_GRAPH": "0",
             "ORBGPU_KNN_NOSPLIT": "1", "ORBGPU_OD_ITERS": "4"}
    assert _child(_KNOBS, knobs) == {}
    assert _child(_KNOBS, dict(knobs, ORBGPU_DIAGNOSTICS="0")) == {}
    assert _child(_KNOBS, dict(knobs, ORBGPU_DIAGNOSTICS="1")) == knobs
    assert _child(_KNOBS, {"ORBGPU_DIAGNOSTICS": "1"}) == {}


def test_second_hip_runtime_fails_loudly():
    r = _child(_RUNTIMES, args=("lib_first",))
    assert len(r["maps"]) == 2, r  # the hazard is real in this image
    assert r["create"] == -7, r  # ORBGPU_ERR_RUNTIME (include/orbgpu.h)
    assert "two HIP runtimes" in r["error"] and "import torch before" in r["error"]


def test_one_runtime_when_torch_comes_first():
    r = _child(_RUNTIMES, args=("torch_first",))
    assert len(r["maps"]) == 1, r
    assert r["create"] != -7, r  # ORBGPU_ERR_NO_DEVICE here, a context on the GPU box
