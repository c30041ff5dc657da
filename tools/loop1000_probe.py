"""Distance of the HIP guided loop from the committed 1000-step oracle output (BASELINE
configs[1]'s full schedule), fp32 and bf16 noise MLP, same x_T and counter-keyed draws as
tests/golden/gen_oracle_loop.py.  Prints one JSON line per precision (metrics.py:20-44 Chamfer,
p99.9 / max / mean |hip - oracle|).  GPU; a measurement tool for the gate in
tests/test_gpu_configs.py (tools/ only).

    python tools/loop1000_probe.py [--steps 1000]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests", "golden"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=1000)
    args = ap.parse_args()
    from detweights import load_into
    from pointcloud_style_transfer_amd import rng
    from pointcloud_style_transfer_amd.config.config import Config
    from pointcloud_style_transfer_amd.evaluation.metrics import PointCloudMetrics
    from pointcloud_style_transfer_amd.models.diffusion_model import (DiffusionProcess,
                                                                        PointCloudDiffusionModel)
    from pointcloud_style_transfer_amd.synthetic import lidar_like_cloud, standard_normal

    S = args.steps
    name = "oracle_loop120k.npz" if S == 50 else f"oracle_loop120k_{S}.npz"
    ref = torch.from_numpy(np.load(os.path.join(REPO, "tests", "golden", name))[f"x_{S}"]).cuda()
    src = torch.from_numpy(lidar_like_cloud(1000, 120000)[None]).cuda()
    cond = torch.from_numpy(lidar_like_cloud(2000, 120000)[None]).cuda()
    xT = torch.from_numpy(standard_normal(3000, (1, 120000, 3))).cuda()
    for prec in ("fp32", "bf16"):
        cfg = Config(make_dirs=False, precision=prec)
        model = PointCloudDiffusionModel(cfg)
        load_into(model)
        model = model.cuda().eval()
        dp = DiffusionProcess(cfg, device="cuda")
        t0 = time.perf_counter()
        with torch.no_grad(), rng.replay(rng.CounterRNG(6000)):
            out = dp.guided_sample_loop(model, src, cond, S, 7.5, x_T=xT)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        ch = float(PointCloudMetrics().chamfer_distance(out, ref)[0])
        d = (out - ref).abs().flatten().double()
        print(json.dumps({"steps": S, "precision": prec, "chamfer_vs_oracle": ch,
                          "p999_abs": float(torch.quantile(d, 0.999)), "max_abs": float(d.max()),
                          "mean_abs": float(d.mean()),
                          "frac_within_1e-3_abs": float((d <= 1e-3).double().mean()),
                          "seconds": round(el, 1)}), flush=True)


if __name__ == "__main__":
    main()
