"""FPS timing (the SA1 shape: N = 30000, 512 samples) on a lidar-like and a Gaussian cloud, B = 1
and B = 32, HIP events over 20 calls."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pointcloud_style_transfer_amd import _hip  # noqa: E402
from pointcloud_style_transfer_amd.synthetic import lidar_like_cloud  # noqa: E402

mode = os.path.basename(_hip.LIB_PATH)
for name in ("lidar", "gauss"):
    for B in (1, 32):
        if name == "lidar":
            xyz = np.stack([lidar_like_cloud(100 + b, 30000) for b in range(B)]).astype(np.float32)
        else:
            xyz = np.random.default_rng(B).standard_normal((B, 30000, 3)).astype(np.float32)
        x = torch.from_numpy(xyz).cuda()
        st = torch.zeros(B, dtype=torch.long, device="cuda")
        for _ in range(3):
            _hip.fps(x, 512, st)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            _hip.fps(x, 512, st)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 20
        print(f"cull={mode} {name:5s} B={B:2d}: {ms:.3f} ms  {ms * 1e3 / 512:.3f} us/round", flush=True)
