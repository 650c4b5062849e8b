"""Diagnostic: run one 64-pair batch with ORBGPU_OCT_STAMPS=1 to print octree phase times."""
import os, sys
os.environ["ORBGPU_OCT_STAMPS"] = "1"
os.environ["ORBGPU_DIAGNOSTICS"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import orbslam3lib_amd as og
from orbslam3lib_amd import synth
P = int(sys.argv[1]) if len(sys.argv) > 1 else 64
U = 8
uniq = [synth.stereo_pair(480, 640, i) for i in range(U)]
imgs = np.stack([uniq[(i // 2) % U][i % 2] for i in range(2 * P)])
be = og.BatchExtractor(2000, 1.2, 8, 20, 7, width=640, height=480, max_images=2 * P)
be.upload(imgs)
be.run()
be.synchronize()
