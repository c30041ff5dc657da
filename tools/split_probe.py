"""Probe: C clouds per GPU as G concurrent groups (one host thread, loop stream and side stream
per group), each group stepping its own C/G clouds through the product step (bench.py's step).
The groups' kernels interleave on the device, so one group's kNN query and voxel chain can run
beside another group's noise MLP.  Prints one JSON line: ms per step (all C clouds advanced one
step) for G = 1 and the requested G.

    python tools/split_probe.py --clouds 32 --groups 2 --steps 10 --warmup 3
"""
import argparse
import json
import os
import sys
import threading
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def run(C, G, steps, warmup, points=120000):
    import bench as B
    from pointcloud_style_transfer_amd import _hip
    from pointcloud_style_transfer_amd.models import diffusion_model as dmod
    from pointcloud_style_transfer_amd.synthetic import lidar_like_cloud, standard_normal

    device = torch.device("cuda", 0)
    cfg, model, dp = B.build_model("bf16", device)
    hp, npred = model.hierarchical_processor, model.noise_predictor
    timesteps = torch.linspace(dp.num_timesteps - 1, 0, dp.num_timesteps).long().tolist()
    n = C // G
    bar = threading.Barrier(G + 1)
    errors = []

    def group(g):
        try:
            ids = range(g * n, (g + 1) * n)
            src = torch.from_numpy(np.stack([lidar_like_cloud(1000 + i, points) for i in ids])).to(device)
            cond = torch.from_numpy(np.stack([lidar_like_cloud(2000 + i, points) for i in ids])).to(device)
            xT = torch.from_numpy(np.stack([standard_normal(3000 + i, (points, 3)) for i in ids])).to(device)
            with torch.no_grad():
                style = model.style_encoder(hp.downsample(cond)[0])
                style_in = torch.cat([style, torch.zeros_like(style)])
                pk = npred.packed()
                S = len(timesteps)
                t_rows = torch.tensor(timesteps, dtype=torch.long).repeat_interleave(2 * n)
                t_rows = t_rows.view(S, 2 * n).to(device)
                state = dmod.StepState(device)
                state.begin(torch.cuda.current_stream())
                with torch.cuda.stream(state.loop):
                    knn_ws = _hip.knn_workspace(2 * n, points, cfg.global_points, device=device)
                    vws = _hip.voxel_copies_workspace(n, points, 2, device=device)
                    conds = npred.cond(t_rows.reshape(-1), style_in.repeat(S, 1), pk).view(S, 2 * n, -1)
                    x = xT.clone()
                    x_cat = torch.cat([x, x]).contiguous()
                st = {"x": x, "prepped": False}

                def step(i):
                    t = timesteps[i]
                    t_prev = timesteps[i + 1] if t > 0 else -1
                    cnd = conds[i]
                    xc, xi = hp.downsample_copies(st["x"], 2, vws, st["prepped"])

                    def mlp(xc_, wait=None, start=None):
                        return npred.forward_cond(xc_, cnd, pk, wait, start)

                    prep = dmod.voxel_prep_ok(hp, st["x"], state)
                    st["x"] = dmod.hierarchical_step(hp, mlp, xc, xi, x_cat, st["x"], src, 7.5,
                                                     dp._coeffs(t, t_prev), knn_ws, state,
                                                     fused=True, vox_ws=vws if prep else None)
                    st["prepped"] = prep

                with torch.cuda.stream(state.loop):
                    for i in range(warmup):
                        step(i)
                torch.cuda.synchronize()
                bar.wait()   # warm
                bar.wait()   # go
                with torch.cuda.stream(state.loop):
                    for i in range(steps):
                        step(warmup + i)
                state.end(torch.cuda.current_stream())
                torch.cuda.synchronize()
                state.check()
                bar.wait()   # done
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e))
            bar.abort()

    ths = [threading.Thread(target=group, args=(g,)) for g in range(G)]
    for t in ths:
        t.start()
    bar.wait()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    bar.wait()
    bar.wait()
    el = time.perf_counter() - t0
    for t in ths:
        t.join()
    if errors:
        raise RuntimeError(errors)
    return el / steps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clouds", type=int, default=32)
    ap.add_argument("--groups", type=int, default=2)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    a = ap.parse_args()
    res = {"clouds": a.clouds, "steps": a.steps}
    for G in (1, a.groups, 1, a.groups):
        res.setdefault(f"ms_per_step_g{G}", []).append(round(run(a.clouds, G, a.steps, a.warmup), 3))
    print(json.dumps(res))


if __name__ == "__main__":
    main()
