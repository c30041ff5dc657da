"""Chamfer forward timing on the configs[2] loss shape (8 clouds x 30000 coarse points, both
directions): python tools/bench_chamfer.py [--reps R]"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pointcloud_style_transfer_amd import _hip  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=10)
ap.add_argument("--B", type=int, default=8)
ap.add_argument("--N", type=int, default=30000)
ap.add_argument("--kind", default="gauss", choices=["gauss", "lidar"])
ap.add_argument("--noise", type=float, default=0.05)
ap.add_argument("--mode", type=int, default=0, help="0 auto, 1 exhaustive, 2 grid")
a = ap.parse_args()
ap2 = a
rng = np.random.default_rng(0)
if a.kind == "gauss":
    p = (rng.standard_normal((a.B, a.N, 3)) * [1, 1, 0.2]).astype(np.float32)
    q = (rng.standard_normal((a.B, a.N, 3)) * [1, 1, 0.2]).astype(np.float32)
else:  # the trainer's pair: a predicted x0 (noisy, spread) against the lidar-like coarse cloud
    from pointcloud_style_transfer_amd.synthetic import lidar_like_cloud
    q = np.stack([lidar_like_cloud(100 + i, a.N) for i in range(a.B)]).astype(np.float32)
    p = (q + rng.standard_normal(q.shape) * a.noise).astype(np.float32)
p, q = torch.from_numpy(p).cuda(), torch.from_numpy(q).cuda()
_hip.chamfer_fwd(p, q, a.mode)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(a.reps):
    out, _, _ = _hip.chamfer_fwd(p, q, a.mode)
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / a.reps
pairs = 2 * a.B * a.N * a.N
print(json.dumps({"kind": a.kind, "noise": a.noise, "mode": a.mode, "ms_per_fwd": round(ms, 4), "pairs": pairs, "Gpairs_per_s": round(pairs / ms / 1e6, 1),
                  "out0": float(out[0])}))
