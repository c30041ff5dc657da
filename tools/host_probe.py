"""Is the eager sampling loop host-bound?  Runs the bench's step (product loop layout: step on the
high-priority stream, kNN build on the side stream) for 20 steps from t = 999 and reports the
host enqueue time per step next to the GPU time per step (enqueue + the final synchronize)."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pointcloud_style_transfer_amd import _hip  # noqa: E402
from pointcloud_style_transfer_amd.config.config import Config  # noqa: E402
from pointcloud_style_transfer_amd.models import diffusion_model as dmod  # noqa: E402
from pointcloud_style_transfer_amd.synthetic import lidar_like_cloud, standard_normal  # noqa: E402

cfg = Config(make_dirs=False, precision="bf16")
torch.manual_seed(0)
m = dmod.PointCloudDiffusionModel(cfg).cuda().eval()
dp = dmod.DiffusionProcess(cfg, "cuda")
hp, npred = m.hierarchical_processor, m.noise_predictor
src = torch.from_numpy(lidar_like_cloud(1000, 120000)[None]).cuda()
cond = torch.from_numpy(lidar_like_cloud(2000, 120000)[None]).cuda()
x = torch.from_numpy(standard_normal(3000, (1, 120000, 3))).cuda()
with torch.no_grad():
    style = m.style_encoder(hp.downsample(cond)[0])
    style_in = torch.cat([style, torch.zeros_like(style)])
    ts = dp._timesteps(1000)
    S = len(ts)
    t_rows = torch.tensor(ts).repeat_interleave(2).view(S, 2).cuda()
    conds = npred.cond(t_rows.reshape(-1), style_in.repeat(S, 1)).view(S, 2, -1)
    x_cat = torch.cat([x, x]).contiguous()
    state = dmod.StepState("cuda")
    loop, side = state.loop, state.side
    loop.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(loop):
        ws = _hip.knn_workspace(2, 120000, cfg.global_points, device="cuda")

    def step(i):
        global x
        t = ts[i]
        tp = ts[i + 1] if t > 0 else -1
        xc, xi = hp.downsample_copies(x, 2)
        c = conds[i]
        eps = dmod.hierarchical_eps(hp, lambda a: npred.forward_cond(a, c), xc, xi, x_cat, ws, state)
        x = _hip.cfg_ddim_step(x, eps[:1], eps[1:], src, 7.5, dp._coeffs(t, tp), x_cat=x_cat)

    with torch.cuda.stream(loop):
        for i in range(5):
            step(i)
    torch.cuda.synchronize()
    for rep in range(3):
        host = []
        t0 = time.perf_counter()
        with torch.cuda.stream(loop):
            for i in range(20):
                h0 = time.perf_counter()
                step(i)
                host.append(time.perf_counter() - h0)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"host enqueue {1e6 * np.mean(host):.0f} us/step (max {1e6 * np.max(host):.0f}); "
              f"wall {1e6 * (t2 - t0) / 20:.0f} us/step; waited at sync {1e6 * (t2 - t1):.0f} us", flush=True)
