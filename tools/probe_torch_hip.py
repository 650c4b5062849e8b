"""Probe: can torch's HIP runtime and liborbgpu's share a process, in either init order?"""
import sys

order = sys.argv[1]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import orbslam3lib_amd as og  # noqa: E402

if order == "torch_first":
    x = torch.ones(4, device="cuda:0")
    print("torch ok", x.sum().item(), flush=True)
    be = og.BatchExtractor(100, 1.2, 8, 20, 7, width=640, height=480, max_images=2)
    be.upload(np.zeros((2, 480, 640), np.uint8))
    be.run()
    be.synchronize()
    print("orbgpu ok", flush=True)
else:
    be = og.BatchExtractor(100, 1.2, 8, 20, 7, width=640, height=480, max_images=2)
    be.upload(np.zeros((2, 480, 640), np.uint8))
    be.run()
    be.synchronize()
    print("orbgpu ok", flush=True)
    print("count", torch.cuda.device_count(), flush=True)
    x = torch.ones(4, device="cuda:0")
    print("torch ok", x.sum().item(), flush=True)
