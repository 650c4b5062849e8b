#!/usr/bin/env python3
"""Diagnostics: the pipelined ingest loop of bench.py (async upload of step k+1 beside step k),
timed per variant; host-side time of each call printed so blocking calls show."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import orbslam3lib_amd as og  # noqa: E402
from orbslam3lib_amd import synth  # noqa: E402

P = int(os.environ.get("PAIRS", "128"))
uniq = [synth.stereo_pair(480, 640, i) for i in range(8)]
imgs = np.stack([uniq[(i // 2) % 8][i % 2] for i in range(2 * P)])
be = og.BatchExtractor(2000, 1.2, 8, 20, 7, width=640, height=480, max_images=2 * P)
be.upload(imgs)
pin = be.pinned(imgs.shape)
pin[:] = imgs
for _ in range(3):
    be.run(); be.match_stereo(False)
be.synchronize()
t0 = time.perf_counter()
for _ in range(10):
    be.run(); be.match_stereo(False)
be.synchronize()
comp = (time.perf_counter() - t0) / 10
t0 = time.perf_counter()
for _ in range(10):
    be.upload_async(pin); be.run()
be.synchronize()
print("compute %.3f ms/step" % (comp * 1e3))
for rep in range(2):
    be.synchronize()
    t0 = time.perf_counter()
    tu = tr = 0.0
    be.upload_async(pin)
    for k in range(10):
        a = time.perf_counter(); be.run(); be.match_stereo(False); b = time.perf_counter()
        if k < 9:
            be.upload_async(pin)
        c = time.perf_counter()
        tr += b - a; tu += c - b
    be.synchronize()
    el = (time.perf_counter() - t0) / 10
    print("pipelined %.3f ms/step (host: run %.3f ms, upload call %.3f ms)" % (el * 1e3, tr / 10 * 1e3, tu / 10 * 1e3))
be.free_pinned()
