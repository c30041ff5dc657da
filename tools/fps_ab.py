"""FPS A/B (experiment runs): PCST_LIB=<lib> python tools/fps_ab.py -> per cloud kind and batch,
ms per call, us per round and a hash of the sampled indices (equal hashes across libraries:
the same samples).  Shapes: the SA1 shape (N = 30000, 512 samples), B = 1 and 32, lidar-like,
Gaussian and a lattice (ties)."""
import hashlib
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))
import knobs  # noqa: E402

knobs.apply()
from pointcloud_style_transfer_amd import _hip  # noqa: E402
from pointcloud_style_transfer_amd.synthetic import lidar_like_cloud  # noqa: E402

mode = os.path.basename(_hip.LIB_PATH)
for name in ("lidar", "gauss", "lattice"):
    for B in (1, 32):
        if name == "lidar":
            xyz = np.stack([lidar_like_cloud(100 + b, 30000) for b in range(B)]).astype(np.float32)
        elif name == "gauss":
            xyz = np.random.default_rng(B).standard_normal((B, 30000, 3)).astype(np.float32)
        else:
            g = np.stack(np.meshgrid(np.arange(40), np.arange(30), np.arange(25), indexing="ij"), -1)
            xyz = np.broadcast_to(g.reshape(1, -1, 3).astype(np.float32) * 0.1, (B, 30000, 3)).copy()
        x = torch.from_numpy(xyz).cuda()
        st = torch.zeros(B, dtype=torch.long, device="cuda")
        for _ in range(3):
            idx = _hip.fps(x, 512, st)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            _hip.fps(x, 512, st)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 20
        h = hashlib.sha256(idx.cpu().numpy().tobytes()).hexdigest()[:16]
        print(f"{mode} {name:7s} B={B:2d}: {ms:.3f} ms  {ms * 1e3 / 512:.3f} us/round  idx {h}",
              flush=True)
