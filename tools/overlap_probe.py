"""Experiment: the kNN build on a side stream during the noise MLP (bench trajectory).
python tools/overlap_probe.py --mode seq|side|side_lo [--steps 20]  (PCST_KNN_BUILD_LDS_PAD
sets the build workgroups' dynamic LDS, keeping them off CUs that hold an MLP workgroup)"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pointcloud_style_transfer_amd import _hip  # noqa: E402
from pointcloud_style_transfer_amd.config.config import Config  # noqa: E402
from pointcloud_style_transfer_amd.models.diffusion_model import (DiffusionProcess,  # noqa: E402
                                                                   PointCloudDiffusionModel)
from pointcloud_style_transfer_amd.synthetic import lidar_like_cloud, standard_normal  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--mode", default="seq")
ap.add_argument("--steps", type=int, default=20)
ap.add_argument("--warmup", type=int, default=5)
a = ap.parse_args()
cfg = Config(make_dirs=False, precision="bf16")
torch.manual_seed(0)
model = PointCloudDiffusionModel(cfg).cuda().eval()
dp = DiffusionProcess(cfg, "cuda")
src = torch.from_numpy(lidar_like_cloud(1000, 120000)[None]).cuda()
cond = torch.from_numpy(lidar_like_cloud(2000, 120000)[None]).cuda()
xT = torch.from_numpy(standard_normal(3000, (1, 120000, 3))).cuda()
hp, npred = model.hierarchical_processor, model.noise_predictor
side = None
if a.mode == "side":
    side = torch.cuda.Stream()
elif a.mode == "side_lo":  # main stream at high priority, the build on a default-priority one
    side = torch.cuda.Stream(priority=0)
    torch.cuda.set_stream(torch.cuda.Stream(priority=-1))
main = torch.cuda.current_stream()
with torch.no_grad():
    style = model.style_encoder(hp.downsample(cond)[0])
    style_in = torch.cat([style, torch.zeros_like(style)])
    ts = dp._timesteps(1000)
    keep = []

    def run(nsteps):
        x = xT.clone()
        x_cat = torch.cat([x, x]).contiguous()
        for i in range(nsteps):
            t = ts[i]
            t_prev = ts[i + 1] if t > 0 else -1
            xc, xi = hp.downsample_copies(x, 2)
            if side is None:
                h = _hip.knn3_build(x_cat, xi)
            else:
                ev = torch.cuda.Event()
                ev.record(main)
                side.wait_event(ev)
                with torch.cuda.stream(side):
                    h = _hip.knn3_build(x_cat, xi)
                    done = torch.cuda.Event()
                    done.record(side)
            keep.append(h)
            nc = npred(xc, torch.full((2,), t, device="cuda", dtype=torch.long), style_in)
            if side is not None:
                main.wait_event(done)
            eps = _hip.knn3_query(nc, h)
            x = _hip.cfg_ddim_step(x, eps[:1], eps[1:], src, 7.5, dp._coeffs(t, t_prev), x_cat=x_cat)
        return x

    run(a.warmup)
    torch.cuda.synchronize()
    keep.clear()
    t0 = time.perf_counter()
    out = run(a.steps)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    keep.clear()
print(json.dumps({"mode": a.mode, "pad": os.environ.get("PCST_KNN_BUILD_LDS_PAD", "0"),
                  "steps": a.steps, "ms_per_step": round(el / a.steps * 1e3, 4),
                  "checksum": float(out.double().abs().sum())}))
