"""kNN result hashes for A/B runs of experiment libraries (PCST_LIB=<lib> python
tools/knn_check.py): the compact and rows layouts' kNN-3 upsampling on the step's inputs (the
bench's x_T and a LiDAR-like cloud, the voxel downsample's indices for 2 CFG rows, and 64 rows of
32 clouds), hashed: equal hashes across libraries = the same bits as the product library, whose
results the GPU suite checks against the oracle."""
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
from pointcloud_style_transfer_amd.synthetic import lidar_like_cloud, standard_normal  # noqa: E402


def h(t):
    return hashlib.sha256(t.detach().cpu().numpy().tobytes()).hexdigest()[:16]


dev = torch.device("cuda", 0)
N, T = 120000, 30000
for name, C, mk in (("x_T", 1, lambda c: standard_normal(3000 + c, (N, 3))),
                    ("lidar", 1, lambda c: lidar_like_cloud(1000 + c, N)),
                    ("lidar32", 32, lambda c: lidar_like_cloud(1000 + c, N))):
    x = torch.from_numpy(np.ascontiguousarray(np.stack([mk(c) for c in range(C)]), np.float32)).to(dev)
    _, idx = _hip.voxel_downsample(x, T, seed=77, copies=2)
    idx = idx.contiguous()
    x_cat = torch.cat([x, x]).contiguous()
    coarse = torch.randn(2 * C, T, 3, device=dev, generator=torch.Generator(device=dev).manual_seed(9))
    hc = _hip.knn3_build(x_cat, idx)
    a = _hip.knn3_query(coarse, hc)
    r = _hip.knn3_rows_build(x, T, 2)
    _hip.knn3_rows_refs(r, idx)
    b = _hip.knn3_rows_query(coarse, r)
    torch.cuda.synchronize()
    print(f"{os.path.basename(_hip.LIB_PATH)} {name}: compact {h(a)} rows {h(b)} same {torch.equal(a, b)}",
          flush=True)
