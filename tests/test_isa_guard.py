"""CPU: an ISA guard for the fault class k_pyr_tail hit in round 4.

The kernels that keep their working set in LDS must address it with ds_* instructions.  An LDS
buffer reached through a generic pointer compiles to flat_* instructions instead; k_pyr_tail's
first GPU run faulted on exactly that (a 4-byte-aligned 12-byte LDS row read emitted as
flat_load_dwordx3).  This test disassembles the gfx950 code object of the product library and
fails if any of those kernels contains a flat_* instruction, so the regression is caught on the
CPU before a GPU run."""
import collections
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "orbslam3lib_amd", "liborbgpu.so")
OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"

# mangled-name fragments of the LDS-resident kernels (every instantiation of each)
LDS_KERNELS = ("k_pyr_tail", "k_blur_resize", "6k_blurE", "k_fast_cells", "k_orient_desc",
               "k_knn2_mfma_pairs", "k_knn2_mfma_plain", "k_finalize")


def _flat_per_kernel(tmp_path):
    shutil.copy(LIB, tmp_path / "liborbgpu.so")
    subprocess.check_call([OBJDUMP, "--offloading", "liborbgpu.so"], cwd=tmp_path, stdout=subprocess.DEVNULL)
    objs = sorted(p for p in os.listdir(tmp_path) if p.endswith("gfx950"))
    assert objs, "no gfx950 code object in liborbgpu.so"
    flat = collections.Counter()
    seen = set()
    for o in objs:
        dis = subprocess.run([OBJDUMP, "-d", o], cwd=tmp_path, check=True, capture_output=True, text=True).stdout
        name = None
        for line in dis.splitlines():
            m = re.match(r"^[0-9a-f]+ <(\S+)>:", line)
            if m:
                name = m.group(1)
                seen.add(name)
            elif name and re.match(r"^\s+flat_", line):
                flat[name] += 1
    return flat, seen


@pytest.mark.skipif(not (os.path.exists(LIB) and os.path.exists(OBJDUMP)), reason="library or llvm-objdump missing")
def test_lds_resident_kernels_have_no_flat_instructions(tmp_path):
    flat, seen = _flat_per_kernel(tmp_path)
    for frag in LDS_KERNELS:
        assert any(frag in s for s in seen), "kernel %s not found in the code object" % frag
    bad = {k: v for k, v in flat.items() if any(f in k for f in LDS_KERNELS)}
    assert not bad, "flat_* instructions in LDS-resident kernels: %s" % bad
