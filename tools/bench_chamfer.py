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
a = ap.parse_args()
rng = np.random.default_rng(0)
p = torch.from_numpy((rng.standard_normal((a.B, a.N, 3)) * [1, 1, 0.2]).astype(np.float32)).cuda()
q = torch.from_numpy((rng.standard_normal((a.B, a.N, 3)) * [1, 1, 0.2]).astype(np.float32)).cuda()
_hip.chamfer_fwd(p, q)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(a.reps):
    out, _, _ = _hip.chamfer_fwd(p, q)
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / a.reps
pairs = 2 * a.B * a.N * a.N
print(json.dumps({"ms_per_fwd": round(ms, 4), "pairs": pairs, "Gpairs_per_s": round(pairs / ms / 1e6, 1),
                  "out0": float(out[0])}))
