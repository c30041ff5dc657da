"""kNN outlier counts along the bench trajectory (the bench's cloud, x_T and schedule):
python tools/knn_outliers.py [--steps-list 0,1,5,10,20,100,500,900]"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pointcloud_style_transfer_amd import _hip  # noqa: E402
from pointcloud_style_transfer_amd.config.config import Config  # noqa: E402
from pointcloud_style_transfer_amd.models.diffusion_model import (DiffusionProcess,  # noqa: E402
                                                                   PointCloudDiffusionModel)
from pointcloud_style_transfer_amd.synthetic import lidar_like_cloud  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--steps-list", default="0,1,2,5,10,20,50,100,200,500,800,999")
a = ap.parse_args()
want = sorted(int(s) for s in a.steps_list.split(","))
cfg = Config(make_dirs=False, precision="bf16")
torch.manual_seed(0)
model = PointCloudDiffusionModel(cfg).cuda().eval()
dp = DiffusionProcess(cfg, "cuda")
src = torch.from_numpy(lidar_like_cloud(1000, 120000)).cuda()[None]
cond = torch.from_numpy(lidar_like_cloud(2000, 120000)).cuda()[None]
x = torch.randn(1, 120000, 3, device="cuda")
hp = model.hierarchical_processor
npred = model.noise_predictor
with torch.no_grad():
    style = model.style_encoder(hp.downsample(cond)[0])
    style_in = torch.cat([style, torch.zeros_like(style)])
    ts = dp._timesteps(1000)
    x_cat = torch.cat([x, x]).contiguous()
    for i, t in enumerate(ts):
        t_prev = ts[i + 1] if t > 0 else -1
        xc, xi = hp.downsample_copies(x, 2)
        nc = npred(xc, torch.full((2,), t, device="cuda", dtype=torch.long), style_in)
        st = [] if i in want else None
        eps = _hip.knn3_interp(nc, x_cat, xi, stats=st)
        if st:
            print(f"step {i} t={t}: chunks {st[0]['chunks']} outliers {st[0]['outliers']}", flush=True)
        x = _hip.cfg_ddim_step(x, eps[:1], eps[1:], src, 7.5, dp._coeffs(t, t_prev), x_cat=x_cat)
        if i >= want[-1]:
            break
