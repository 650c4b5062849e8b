"""Runs a few bench-shaped steps (256 stereo pairs, extract + kNN2) for rocprofv3 passes."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import orbslam3lib_amd as og
from orbslam3lib_amd import synth
P = int(os.environ.get("PAIRS", "256"))  # bench.py --pairs default
steps = int(os.environ.get("STEPS", "3"))
U = 8
uniq = [synth.stereo_pair(480, 640, i) for i in range(U)]
imgs = np.stack([uniq[(i // 2) % U][i % 2] for i in range(2 * P)])
be = og.BatchExtractor(2000, 1.2, 8, 20, 7, width=640, height=480, max_images=2 * P)
be.upload(imgs)
for _ in range(steps):
    be.run()
    be.match_stereo()
be.synchronize()
print("done")
