"""Repeatability probe of the small-list FAST path and its overflow queue (orb_kernels.hip
k_fast_cells<CP, true> / k_fast_cells_ovf) on a batch shaped like the bench's chunks: 24
synthetic 640x480 stereo pairs and 8 pairs of uniform noise (whose cells overflow the capped
lists), 64 images on the default chunk streams.  Each setting runs R batches on one context:
the default (cells queued only when they overflow) and ORBGPU_FAST_OVF_ALL=1 (every small-list
cell through the queue).  Every run's keypoints and descriptors must equal the first default
run's, and four images are checked against the oracle.
Usage: python tools/fast_ovf_probe.py [R]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from orbslam3lib_amd import synth  # noqa: E402


def main():
    R = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    os.environ["ORBGPU_DIAGNOSTICS"] = "1"
    import orbslam3lib_amd as og
    from oracle import oracle_py as oracle
    rng = np.random.default_rng(5)
    imgs = [x for i in range(24) for x in synth.stereo_pair(480, 640, 500 + i)]
    imgs += [rng.integers(0, 256, (480, 640), dtype=np.uint8) for _ in range(16)]
    imgs = np.stack(imgs)

    def runs(env):
        for k, v in env.items():
            os.environ[k] = v
        be = og.BatchExtractor(2000, 1.2, 8, 20, 7, width=640, height=480, max_images=len(imgs))
        be.upload(imgs)
        out = []
        for _ in range(R):
            be.run()
            be.synchronize()
            out.append([be.result(i) for i in range(len(imgs))])
        for k in env:
            del os.environ[k]
        return out

    base = runs({})
    bad = 0
    for name, env in (("default", {}), ("ovf_all", {"ORBGPU_FAST_OVF_ALL": "1"})):
        got = base if name == "default" else runs(env)
        for r in range(R):
            for i in range(len(imgs)):
                k, d, m = got[r][i]
                fk, fd, fm = base[0][i]
                if m != fm or not np.array_equal(k.view(np.uint8), fk.view(np.uint8)) or not np.array_equal(d, fd):
                    bad += 1
                    print("%s run %d image %d differs (%d vs %d keypoints)" % (name, r, i, m, fm))
        print("%s: %d runs x %d images compared" % (name, R, len(imgs)))
    for i in (0, 1, len(imgs) - 2, len(imgs) - 1):
        k, d, m = base[0][i]
        rk, rd, rm = oracle.extract(imgs[i], nfeatures=2000)
        ok = m == rm and np.array_equal(d, rd.reshape(-1, 32))
        bad += 0 if ok else 1
        print("image %d vs oracle: %s (%d keypoints)" % (i, "equal" if ok else "DIFFERS", m))
    print("RESULT", "ok" if bad == 0 else "%d mismatches" % bad)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
