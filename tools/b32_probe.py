"""Experiment: the kNN build's placement at many clouds per GPU (BASELINE configs[4]'s share).

    python tools/b32_probe.py [--clouds 32] [--steps 10] [--reps 3] [--modes seq,hi_pad,hi_nopad,eq,side_hi]

Runs the bench's denoise step (B clouds of 120k, CFG x2, 30k coarse, bf16, steps from t = 999) in
several layouts, interleaved over `reps` rounds, and prints the median ms/step of each:
  seq       the kNN build inline on the loop stream before the MLP (the product at this size)
  hi_pad    build on a side stream, loop stream high priority, build LDS floor 8192 (the B = 1 layout)
  hi_nopad  same without the LDS floor
  eq        build on a side stream, both streams default priority, no LDS floor
  side_hi   build on a high-priority side stream, loop at default priority, no LDS floor
A development tool (tools/ only)."""
import argparse
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from pointcloud_style_transfer_amd import _hip  # noqa: E402
from pointcloud_style_transfer_amd.synthetic import lidar_like_cloud, standard_normal  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clouds", type=int, default=32)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--modes", default="seq,hi_pad,hi_nopad,eq,side_hi")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    B = a.clouds
    cfg, model, dp = bench.build_model("bf16", dev)
    hp, npred = model.hierarchical_processor, model.noise_predictor
    src = torch.from_numpy(lidar_like_cloud(1000, 120000)[None]).to(dev).repeat(B, 1, 1)
    cond = torch.from_numpy(lidar_like_cloud(2000, 120000)[None]).to(dev)
    xT = torch.from_numpy(standard_normal(3000, (B, 120000, 3))).to(dev)
    streams = {
        "hi": (torch.cuda.Stream(dev, priority=-1), torch.cuda.Stream(dev, priority=0)),
        "eq": (torch.cuda.Stream(dev, priority=0), torch.cuda.Stream(dev, priority=0)),
        "side_hi": (torch.cuda.Stream(dev, priority=0), torch.cuda.Stream(dev, priority=-1)),
    }
    res = {m: [] for m in a.modes.split(",")}
    with torch.no_grad():
        style = model.style_encoder(hp.downsample(cond)[0]).repeat(B, 1)
        style_in = torch.cat([style, torch.zeros_like(style)])
        ts = torch.linspace(999, 0, 1000).long().tolist()
        S = a.steps + 1
        t_rows = torch.tensor(ts[:S], dtype=torch.long).repeat_interleave(2 * B).view(S, 2 * B).to(dev)
        conds = npred.cond(t_rows.reshape(-1), style_in.repeat(S, 1)).view(S, 2 * B, -1)
        blob, bias = npred.packed()[:2]
        ws = _hip.knn_workspace(2 * B, 120000, cfg.global_points, device=dev)
        vws = _hip.voxel_copies_workspace(B, 120000, 2, device=dev)
        ready, built = _hip.DeviceEvent(), _hip.DeviceEvent()
        torch.cuda.synchronize()

        def run(mode, n):
            key = "hi" if mode.startswith("hi") else mode if mode in streams else "hi"
            loop, side = streams[key]
            floor = 8192 if mode == "hi_pad" else 0
            loop.wait_stream(torch.cuda.current_stream())
            torch.manual_seed(11)  # the same voxel-subset draws in every mode
            with torch.cuda.stream(loop):
                x = xT.clone()
                x_cat = torch.cat([x, x]).contiguous()
                for i in range(n):
                    t, tp = ts[i], ts[i + 1]
                    xc, xi = hp.downsample_copies(x, 2, vws)

                    def mlp(c):
                        return _hip.noise_mlp(c.reshape(-1, 3), cfg.global_points, conds[i], blob, bias,
                                              npred.precision_code).view(2 * B, -1, 3)

                    if mode == "seq":
                        h = _hip.knn3_build(x_cat, xi, ws, 0)
                        eps = _hip.knn3_query(mlp(xc), h)
                    else:
                        ready.record(loop)
                        ready.wait(side)
                        with torch.cuda.stream(side):
                            h = _hip.knn3_build(x_cat, xi, ws, floor)
                            built.record(side)
                        nc = mlp(xc)
                        built.wait(loop)
                        eps = _hip.knn3_query(nc, h)
                    x = _hip.cfg_ddim_step(x, eps[:B], eps[B:], src, 7.5, dp._coeffs(t, tp), x_cat=x_cat)
            torch.cuda.current_stream().wait_stream(loop)
            return x

        outs = {}
        for m in res:
            outs[m] = run(m, 2)
        torch.cuda.synchronize()
        ref = next(iter(outs.values()))
        for m, o in outs.items():
            print(f"{m:8s} bit-identical to first mode: {bool(torch.equal(o, ref))}", flush=True)
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
