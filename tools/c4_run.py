"""C4 latency shape for tracing: one stereo pair per step, extraction + kNN2 as one submission
(BatchExtractor.run_match), 30 steps.  MODE=split runs run() then match_stereo() instead."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import orbslam3lib_amd as og
from orbslam3lib_amd import synth
L, R = synth.stereo_pair(480, 640, 0)
be = og.BatchExtractor(2000, 1.2, 8, 20, 7, width=640, height=480, max_images=2)
be.upload(np.stack([L, R]))
split = os.environ.get("MODE") == "split"
for _ in range(int(os.environ.get("STEPS", "30"))):
    if split:
        be.run()
        be.match_stereo(False)
    else:
        be.run_match()
be.synchronize()
