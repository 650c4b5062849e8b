"""C4 step time (one pair per step, extraction + kNN2): run_match vs run + match_stereo, 200 steps
each after warmup.  ORBGPU_DIAGNOSTICS=1 ORBGPU_GRAPH=0 in the environment disables the graph capture."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import orbslam3lib_amd as og
from orbslam3lib_amd import synth
L, R = synth.stereo_pair(480, 640, 0)
be = og.BatchExtractor(2000, 1.2, 8, 20, 7, width=640, height=480, max_images=2)
be.upload(np.stack([L, R]))
for mode in ("run_match", "split", "run_match", "split"):
    step = be.run_match if mode == "run_match" else (lambda: (be.run(), be.match_stereo(False)))
    for _ in range(20):
        step()
    be.synchronize()
    t = time.perf_counter()
    for _ in range(200):
        step()
    be.synchronize()
    print("graph=%s %-9s %.1f us/step" % (os.environ.get("ORBGPU_GRAPH", "1"), mode, (time.perf_counter() - t) / 200 * 1e6))
