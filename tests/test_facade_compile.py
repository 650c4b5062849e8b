"""The C++ drop-in compiles where the reference's callers compile (CPU, compile-only).

* -DORBGPU_WITH_OPENCV against tests/cpp/opencv_api: a declaration-only restatement of OpenCV 4.2's
  API shape (CV_8U / CV_8UC1 as macros, InputArray = const _InputArray&, OutputArray =
  const _OutputArray&, Mat::step a MatStep), i.e. the mode INTEGRATION.md §2 prescribes;
* tests/cpp/reference_tu.cpp in that mode: Frame.cc's shape -- ORBextractor.h together with the
  reference's own ORBmatcher class (Frame.cc:24,26), the CPU and side-by-side stereo extractor
  calls, BFMatchORB(mnIdMatchingData, ...) (Frame.cc:1164) and mvImagePyramid;
* the facade against the library's own shim (the tests/cpp GPU program's mode).
The GPU behaviour of the same sources is tests/cpp/facade_test.cpp (test_gpu_parity.py)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FACADE = ["orbslam3lib_amd/facade/ORBextractor.cc", "orbslam3lib_amd/facade/LynxHardwareAccelerator.cc"]


def _compile(src, opencv):
    cmd = ["g++", "-std=c++17", "-Wall", "-Wextra", "-Werror", "-fsyntax-only", "-Iinclude/orbslam3"]
    if opencv:
        cmd += ["-DORBGPU_WITH_OPENCV", "-Itests/cpp/opencv_api"]
    r = subprocess.run(cmd + [src], cwd=ROOT, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-3000:]


@pytest.mark.parametrize("src", FACADE + ["tests/cpp/reference_tu.cpp"])
def test_facade_compiles_against_opencv_api(src):
    _compile(src, opencv=True)


@pytest.mark.parametrize("src", FACADE)
def test_facade_compiles_against_shim(src):
    _compile(src, opencv=False)


def test_opencv_api_stub_rejects_the_round1_mistakes(tmp_path):
    """The stub is strict where round 1's facade was wrong: cv::CV_8U and taking an OutputArray's
    address as a Mat* do not compile against OpenCV's shape."""
    bad = tmp_path / "bad.cpp"
    bad.write_text('#include <opencv2/core/core.hpp>\n'
                   'int f(cv::OutputArray o) { cv::Mat* m = &o; return m->type() == cv::CV_8U; }\n')
    r = subprocess.run(["g++", "-std=c++17", "-fsyntax-only", "-Itests/cpp/opencv_api", str(bad)], cwd=ROOT,
                       capture_output=True, text=True, timeout=60)
    assert r.returncode != 0
