"""CPU: liborbgpu.so loads and exports every entry point include/orbgpu.h declares (no device
compute here); host-only entry points behave."""
import ctypes as C
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    txt = open(os.path.join(ROOT, "include", "orbgpu.h")).read()
    return sorted(set(re.findall(r"\b(orbgpu_[a-z0-9_]+)\s*\(", txt)))


def test_all_declared_symbols_exported():
    import orbslam3lib_amd as og
    lib = og.load_library()
    names = _declared()
    assert len(names) >= 20
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    assert set(names) == set(og.EXPORTED)


def test_library_has_gfx950_code_object():
    data = open(os.path.join(ROOT, "orbslam3lib_amd", "liborbgpu.so"), "rb").read()
    assert b"gfx950" in data
    for k in (b"k_fast_cells", b"k_octree", b"k_orient_desc", b"k_knn2_mfma_pairs", b"k_blur_resize", b"k_blur",
              b"k_pyr_tail", b"k_level_linear"):
        assert k in data, k
    # the measured-slower alternates of rounds 1-4 are not in the product library
    for k in (b"k_fast_wave", b"k_pyramid", b"k_knn2_pairs", b"k_resize", b"k_fast_bands", b"k_fast_sb"):
        assert k not in data, k


def test_host_entry_points():
    import orbslam3lib_amd as og
    lib = og.load_library()
    assert lib.orbgpu_abi_version() == 2  # 2: packed export, ORBGPU_DEVICE_CURRENT
    names = [lib.orbgpu_stage_name(i) for i in range(lib.orbgpu_num_stages())]
    assert names == [b"k_blur_resize", b"k_blur", b"k_fast_cells<48>", b"k_fast_cells<64>", b"k_fast_cells<80>", b"k_octree",
                     b"k_orient_desc", b"k_finalize", b"k_knn2", b"k_stereo", b"k_undistort_grid", b"k_sbs_split", b"k_pack_soa", b"k_sbp", b"k_fisheye_stereo",
                     b"k_pyr_tail"]
    a = np.arange(32, dtype=np.uint8)
    b = np.full(32, 255, np.uint8)
    assert og.ORBmatcher.DescriptorDistance(a, b) == int(np.unpackbits(a ^ b).sum())
    # null arguments are rejected with a status code, never a crash
    assert lib.orbgpu_create(None, 0, 640, 480, 1, None) == -3
    assert lib.orbgpu_destroy(None) == 0


@pytest.mark.parametrize("scale", [1.0, 0.8])
def test_create_rejects_unsupported_scale_factor(scale):
    """orbgpu_create validates the parameters before it looks for a device: a scale factor that
    is not above 1 (ORBextractor's only requirement) is ORBGPU_ERR_INVALID, with or without a
    GPU.  Steps above 2 are accepted since round 5 (k_level_linear)."""
    import orbslam3lib_amd as og
    with pytest.raises(og.OrbGpuError) as e:
        og.ORBextractor(1000, scale, 8, 20, 7, max_width=640, max_height=480)
    assert e.value.code == -3  # ORBGPU_ERR_INVALID (include/orbgpu.h)
