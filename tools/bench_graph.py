"""Eager vs hipGraph-captured guided sampling (BASELINE configs[4]: a captured denoise step),
whole-loop wall time per step at 1 and 32 clouds per GPU; the one-time style encode and graph
capture are included in the loop time (reported as measured).

    python tools/bench_graph.py [--steps 200]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from pointcloud_style_transfer_amd.config.config import Config  # noqa: E402
from pointcloud_style_transfer_amd.models.diffusion_model import (DiffusionProcess,  # noqa: E402
                                                                    PointCloudDiffusionModel)
from pointcloud_style_transfer_amd.synthetic import lidar_like_cloud  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    args = ap.parse_args()
    cfg = Config(make_dirs=False, precision="bf16")
    torch.manual_seed(0)
    model = PointCloudDiffusionModel(cfg).cuda().eval()
    dp = DiffusionProcess(cfg, device="cuda")
    for C in (1, 32):
        src = torch.from_numpy(np.stack([lidar_like_cloud(1000 + i) for i in range(C)])).cuda()
        cond = torch.from_numpy(np.stack([lidar_like_cloud(2000 + i) for i in range(C)])).cuda()
        res = {}
        for graph in (False, True, False, True):
            torch.manual_seed(1)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            dp.guided_sample_loop(model, src, cond, num_inference_steps=args.steps, graph=graph)
            torch.cuda.synchronize()
            res["graph" if graph else "eager"] = (time.perf_counter() - t0) / args.steps * 1e3
        print(json.dumps({"clouds_per_gpu": C, "steps": args.steps,
                          "ms_per_step_eager": round(res["eager"], 4),
                          "ms_per_step_graph": round(res["graph"], 4),
                          "cloud_steps_per_s_graph": round(C / res["graph"] * 1e3, 1)}), flush=True)


if __name__ == "__main__":
    main()
