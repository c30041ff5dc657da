"""Diagnostics: save x at a few steps of the bench trajectory (random-init weights)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pointcloud_style_transfer_amd import _hip  # noqa: E402
from pointcloud_style_transfer_amd.config.config import Config  # noqa: E402
from pointcloud_style_transfer_amd.models.diffusion_model import (DiffusionProcess,  # noqa: E402
                                                                    PointCloudDiffusionModel)
from pointcloud_style_transfer_amd.synthetic import lidar_like_cloud, standard_normal  # noqa: E402

cfg = Config(precision="bf16", make_dirs=False)
torch.manual_seed(0)
m = PointCloudDiffusionModel(cfg).cuda().eval()
dp = DiffusionProcess(cfg, "cuda")
src = torch.from_numpy(lidar_like_cloud(1000, 120000)[None]).cuda()
cond = torch.from_numpy(lidar_like_cloud(2000, 120000)[None]).cuda()
x = torch.from_numpy(standard_normal(3000, (1, 120000, 3))).cuda()
hp, npred = m.hierarchical_processor, m.noise_predictor
keep = {0, 1, 10, 100, 300, 500, 700, 900, 990, 999}
out = {}
with torch.no_grad():
    style = m.style_encoder(hp.downsample(cond)[0])
    style_in = torch.cat([style, torch.zeros_like(style)])
    ts = torch.linspace(999, 0, 1000).long().tolist()
    x_cat = torch.cat([x, x]).contiguous()
    for i, t in enumerate(ts):
        if i in keep:
            out[f"x{i}"] = x.cpu().numpy()[0]
        tp = ts[i + 1] if t > 0 else -1
        xc, xi = hp.downsample(x_cat)
        if i in keep:
            out[f"idx{i}"] = xi.cpu().numpy()
        eps = hp.upsample_knn(npred(xc, torch.full((2,), t, device="cuda"), style_in), x_cat, xi)
        x = _hip.cfg_ddim_step(x, eps[:1], eps[1:], src, 7.5, dp._coeffs(t, tp), x_cat=x_cat)
os.makedirs("gpurun_out", exist_ok=True)
np.savez_compressed("gpurun_out/traj.npz", **out)
print("saved", list(out))
