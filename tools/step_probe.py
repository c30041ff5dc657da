"""Experiment: what the sampling step's stream layout and the bench's MLP timing events cost.

    python tools/step_probe.py [--steps 20] [--reps 3] [--modes bench,noev,seq,seq_ev]

Runs the bench's loop (120k cloud, CFG x2, 30k coarse, bf16, the first `steps` steps from t = 999,
as the driver's invocation) in several layouts, interleaved over `reps` rounds, and prints the
median ms/step of each:
  bench   the product layout (loop stream + side-stream kNN build, device-scope events, the loop ->
          side flag written by the MLP launch) with the bench's two timing events around every MLP
  msig    noev with the loop -> side flag written by the MLP launch (pcst_noise_mlp_ex)
  noev    the same without the timing events, the loop -> side flag by a signal launch
  seq     one stream: the kNN build inline before the MLP, no events at all
  seq_ev  seq with the timing events around the MLP
  evready noev with the loop -> side dependency as an event instead of the kernel-side signal
  nocap   noev with the side-stream build at its natural grids (no max_wg cap)
  capK    noev with the side-stream build capped at K work-groups per launch
  srch    the product step (diffusion_model.hierarchical_step): build + neighbour search on the
          side stream, the fused finish + CFG/DDIM after the MLP
  nosrch  hierarchical_step with SEARCH_BESIDE_MLP off (build-only overlap, query after the MLP)
  bev     noev with the side -> loop dependency as an event instead of the kernel-side flag
  mw      noev with the MLP's last work-group waiting for the build's flag (mlp_waits: the product)
A development tool (tools/ only)."""
import argparse
import os
import statistics
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from pointcloud_style_transfer_amd import _hip  # noqa: E402
from pointcloud_style_transfer_amd.models import diffusion_model as dmod  # noqa: E402
from pointcloud_style_transfer_amd.synthetic import lidar_like_cloud, standard_normal  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--modes", default="bench,noev,seq,seq_ev")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    cfg, model, dp = bench.build_model("bf16", dev)
    hp, npred = model.hierarchical_processor, model.noise_predictor
    src = torch.from_numpy(lidar_like_cloud(1000, 120000)[None]).to(dev)
    cond = torch.from_numpy(lidar_like_cloud(2000, 120000)[None]).to(dev)
    xT = torch.from_numpy(standard_normal(3000, (1, 120000, 3))).to(dev)
    state = dmod.StepState(dev)
    loop = state.loop
    state.begin(torch.cuda.current_stream())
    res = {m: [] for m in a.modes.split(",")}
    with torch.no_grad(), torch.cuda.stream(loop):
        style = model.style_encoder(hp.downsample(cond)[0])
        style_in = torch.cat([style, torch.zeros_like(style)])
        ts = torch.linspace(999, 0, 1000).long().tolist()
        t_rows = torch.tensor(ts, dtype=torch.long).repeat_interleave(2).view(1000, 2).to(dev)
        conds = npred.cond(t_rows.reshape(-1), style_in.repeat(1000, 1)).view(1000, 2, -1)
        blob, bias = npred.packed()[:2]
        ws = _hip.knn_workspace(2, 120000, cfg.global_points, device=dev)
        cap0 = dmod.KNN_BUILD_MAX_WG

        def run(mode, n):
            dmod.KERNEL_SIGNAL = mode != "evready"  # evready: the loop -> side dependency as an event
            dmod.BUILT_SIGNAL = mode != "bev"  # bev: the side -> loop dependency as an event
            # nocap: natural build grids; capK: at most K build work-groups per launch
            dmod.KNN_BUILD_MAX_WG = (0 if mode == "nocap" else
                                     int(mode[3:]) if mode.startswith("cap") else cap0)
            x = xT.clone()
            x_cat = torch.cat([x, x]).contiguous()
            timed = mode.endswith("ev") or mode == "bench"
            for i in range(n):
                t, tp = ts[i], ts[i + 1]
                xc, xi = hp.downsample_copies(x, 2)

                def mlp(c, wait=None, start=None):
                    if timed:
                        e0, e1 = _hip.DeviceEvent(timing=True), _hip.DeviceEvent(timing=True)
                        e0.record()
                    out = _hip.noise_mlp(c.reshape(-1, 3), cfg.global_points, conds[i], blob, bias,
                                         npred.precision_code, wait=wait, signal=start).view(2, -1, 3)
                    if timed:
                        e1.record()
                    return out

                if mode in ("srch", "nosrch"):
                    dmod.SEARCH_BESIDE_MLP = mode == "srch"
                    x = dmod.hierarchical_step(hp, mlp, xc, xi, x_cat, x, src, 7.5, dp._coeffs(t, tp),
                                               ws, state)
                    continue
                if mode.startswith("seq"):
                    h = _hip.knn3_build(x_cat, xi, ws, 0)
                    eps = _hip.knn3_query(mlp(xc), h)
                else:
                    eps = dmod.hierarchical_eps(hp, mlp, xc, xi, x_cat, ws, state, mlp_waits=mode == "mw",
                                                mlp_signals=mode in ("msig", "bench"))
                x = _hip.cfg_ddim_step(x, eps[:1], eps[1:], src, 7.5, dp._coeffs(t, tp), x_cat=x_cat)
            return x

        for m in res:
            run(m, 3)
        torch.cuda.synchronize()
        for _ in range(a.reps):
            for m in res:
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                run(m, a.steps)
                torch.cuda.synchronize()
                res[m].append((time.perf_counter() - t0) / a.steps * 1e3)
    for m, v in res.items():
        print(f"{m:8s} median {statistics.median(v):.4f} ms/step  {[round(u, 4) for u in v]}",
              flush=True)


if __name__ == "__main__":
    main()
