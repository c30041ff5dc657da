"""Experiment: the guided denoise step replayed from a hipGraph vs the eager two-stream loop.

    python tools/graph_probe.py [--steps 20] [--reps 3]

Same workload as the bench (120k cloud, CFG x2, 30k coarse, bf16, the first `steps` steps from
t = 999).  Modes, interleaved over `reps` rounds, median ms/step printed per mode:
  eager   the product's eager layout (loop stream + side-stream kNN build, device-scope events)
  gseq    one step captured on one stream (kNN build inline) and replayed per step
  gfork   one step captured with the kNN build forked to a side stream during the MLP and joined
          before the query (the eager layout as graph branches)
The per-step scalars (conditioning rows, DDIM coefficients, subset seed) are copied into static
device buffers before each replay, as DiffusionProcess._guided_sample_graph does.  Checks that
every mode ends on the same x (bit-identical).  A development tool (tools/ only)."""
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
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    cfg, model, dp = bench.build_model("bf16", dev)
    hp, npred = model.hierarchical_processor, model.noise_predictor
    G = cfg.global_points
    src = torch.from_numpy(lidar_like_cloud(1000, 120000)[None]).to(dev)
    cond = torch.from_numpy(lidar_like_cloud(2000, 120000)[None]).to(dev)
    xT = torch.from_numpy(standard_normal(3000, (1, 120000, 3))).to(dev)
    loop, side = dmod.step_streams(dev)
    loop.wait_stream(torch.cuda.current_stream())
    S = 1000
    ts = torch.linspace(999, 0, S).long().tolist()
    seeds = [(0x5EED + 7919 * i) & (2**62 - 1) for i in range(S)]
    res = {"eager": [], "gseq": [], "gfork": []}
    finals = {}
    with torch.no_grad(), torch.cuda.stream(loop):
        style = model.style_encoder(hp.downsample(cond)[0])
        style_in = torch.cat([style, torch.zeros_like(style)])
        t_rows = torch.tensor(ts, dtype=torch.long).repeat_interleave(2).view(S, 2).to(dev)
        conds = npred.cond(t_rows.reshape(-1), style_in.repeat(S, 1)).view(S, 2, -1)
        blob, bias = npred.packed()[:2]
        coef_tab = torch.tensor(np.array([dp._coeffs(ts[i], ts[i + 1] if ts[i] > 0 else -1)
                                          for i in range(S)], dtype=np.float32)).to(dev)
        seed_tab = torch.tensor(seeds, dtype=torch.int64).to(dev)
        ws = _hip.knn_workspace(2, 120000, G, device=dev)
        x = xT.clone()
        x_cat = torch.cat([x, x]).contiguous()
        cond_cur = conds[0].clone()
        coef_cur = coef_tab[0].clone()
        seed_cur = seed_tab[:1].clone()
        ready, built = _hip.DeviceEvent(), _hip.DeviceEvent()

        def mlp(c):
            return _hip.noise_mlp(c.reshape(-1, 3), G, cond_cur, blob, bias,
                                  npred.precision_code).view(2, -1, 3)

        def step(fork):
            xc, xi = _hip.voxel_downsample_copies_dseed(x, G, seed_cur, 2)
            if fork:
                main = torch.cuda.current_stream()
                side.wait_stream(main)
                with torch.cuda.stream(side):
                    h = _hip.knn3_build(x_cat, xi, ws, dmod.KNN_BUILD_LDS_FLOOR)
                nc = mlp(xc)
                main.wait_stream(side)
            else:
                h = _hip.knn3_build(x_cat, xi, ws, 0)
                nc = mlp(xc)
            eps = _hip.knn3_query(nc, h)
            _hip.cfg_ddim_step_dcoef(x, eps[:1], eps[1:], src, 7.5, coef_cur, x_cat=x_cat, out=x)

        def eager_step():
            xc, xi = _hip.voxel_downsample_copies_dseed(x, G, seed_cur, 2)
            main = torch.cuda.current_stream()
            ready.record(main)
            ready.wait(side)
            with torch.cuda.stream(side):
                h = _hip.knn3_build(x_cat, xi, ws, dmod.KNN_BUILD_LDS_FLOOR)
                built.record(side)
            nc = mlp(xc)
            built.wait(main)
            eps = _hip.knn3_query(nc, h)
            _hip.cfg_ddim_step_dcoef(x, eps[:1], eps[1:], src, 7.5, coef_cur, x_cat=x_cat, out=x)

        def reset():
            x.copy_(xT)
            x_cat.copy_(torch.cat([xT, xT]))

        def set_step(i):
            cond_cur.copy_(conds[i])
            coef_cur.copy_(coef_tab[i])
            seed_cur.copy_(seed_tab[i:i + 1])

        graphs = {}
        for name, fork in (("gseq", False), ("gfork", True)):
            reset()
            set_step(0)
            step(fork)  # warm (allocations outside the capture)
            g = torch.cuda.CUDAGraph()
            cap = torch.cuda.Stream(device=dev)
            cap.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(cap):
                with torch.cuda.graph(g, stream=cap):
                    step(fork)
            torch.cuda.current_stream().wait_stream(cap)
            graphs[name] = g

        def run(name, n):
            reset()
            for i in range(n):
                set_step(i)
                if name == "eager":
                    eager_step()
                else:
                    graphs[name].replay()

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
                finals[m] = x.clone()
    for m, v in res.items():
        print(f"{m:6s} median {statistics.median(v):.4f} ms/step  {[round(u, 4) for u in v]}",
              flush=True)
    ref = finals["eager"]
    for m in ("gseq", "gfork"):
        print(f"{m} final x bit-identical to eager: {bool(torch.equal(finals[m], ref))}", flush=True)


if __name__ == "__main__":
    main()
