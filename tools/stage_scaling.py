"""Per-stage kernel time vs batch size (serialized profiling pass): which stages scale with the
work and which sit on a per-launch latency floor."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import orbslam3lib_amd as og
from orbslam3lib_amd import synth

uniq = [synth.stereo_pair(480, 640, i) for i in range(4)]
for P in [int(x) for x in os.environ.get("PAIRS_LIST", "1,4,16,64,128").split(",")]:
    imgs = np.stack([uniq[(i // 2) % 4][i % 2] for i in range(2 * P)])
    be = og.BatchExtractor(2000, 1.2, 8, 20, 7, width=640, height=480, max_images=2 * P)
    be.upload(imgs)
    for _ in range(2):
        be.run(); be.match_stereo()
    be.synchronize()
    be.set_profiling(True, serialize=True)
    be.reset_stage_times()
    for _ in range(3):
        be.run(); be.match_stereo()
    be.synchronize()
    st = be.stage_times()
    print("pairs %4d  " % P + "  ".join("%s %.1f" % (k, v[0] / v[1] * 1e3) for k, v in st.items() if v[1]))
    del be
