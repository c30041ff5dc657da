"""Experiment: host-side cost of each call of the sampling step (no device sync inside the timing).

    python tools/host_cost.py

Times N back-to-back enqueues of every wrapper the bench's step makes (the device work queues
up behind them; only the host time is measured) and prints the mean host microseconds per call.
A development tool (tools/ only)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from pointcloud_style_transfer_amd import _hip  # noqa: E402
from pointcloud_style_transfer_amd.models import diffusion_model as dmod  # noqa: E402
from pointcloud_style_transfer_amd.synthetic import lidar_like_cloud, standard_normal  # noqa: E402


def timeit(name, fn, n=50):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    print(f"{name:28s} {1e6 * (t1 - t0) / n:8.1f} us host/call", flush=True)


def main():
    dev = torch.device("cuda", 0)
    cfg, model, dp = bench.build_model("bf16", dev)
    hp, npred = model.hierarchical_processor, model.noise_predictor
    G = cfg.global_points
    src = torch.from_numpy(lidar_like_cloud(1000, 120000)[None]).to(dev)
    x = torch.from_numpy(standard_normal(3000, (1, 120000, 3))).to(dev)
    state = dmod.StepState(dev)
    loop, side = state.loop, state.side
    loop.wait_stream(torch.cuda.current_stream())
    with torch.no_grad(), torch.cuda.stream(loop):
        style_in = torch.zeros(2, 256, device=dev)
        ts = torch.linspace(999, 0, 1000).long().tolist()
        t_rows = torch.tensor(ts, dtype=torch.long).repeat_interleave(2).view(1000, 2).to(dev)
        x_cat = torch.cat([x, x]).contiguous()
        ws = _hip.knn_workspace(2, 120000, G, device=dev)
        xc, xi = hp.downsample_copies(x, 2)
        conds = npred.cond(t_rows.reshape(-1), style_in.repeat(1000, 1)).view(1000, 2, -1)
        h = _hip.knn3_build(x_cat, xi, ws, dmod.KNN_BUILD_LDS_FLOOR)
        nc = npred.forward_cond(xc, conds[0])
        eps = _hip.knn3_query(nc, h)
        timeit("packed()", lambda: npred.packed())
        timeit("all_conds (cond x1000)",
               lambda: npred.cond(t_rows.reshape(-1), style_in.repeat(1000, 1)), n=10)
        timeit("downsample_copies", lambda: hp.downsample_copies(x, 2))
        timeit("knn3_build (floor)", lambda: _hip.knn3_build(x_cat, xi, ws, dmod.KNN_BUILD_LDS_FLOOR))
        timeit("knn3_build (no floor)", lambda: _hip.knn3_build(x_cat, xi, ws, 0))
        timeit("forward_cond", lambda: npred.forward_cond(xc, conds[0]))
        timeit("knn3_query", lambda: _hip.knn3_query(nc, h))
        timeit("cfg_ddim_step", lambda: _hip.cfg_ddim_step(x, eps[:1], eps[1:], src, 7.5,
                                                           dp._coeffs(999, 998), x_cat=x_cat))
        ev = _hip.DeviceEvent()
        timeit("DeviceEvent()", lambda: _hip.DeviceEvent(timing=True))
        timeit("event record", lambda: ev.record(loop))
        timeit("event wait", lambda: ev.wait(side))
        timeit("hierarchical_eps", lambda: dmod.hierarchical_eps(
            hp, lambda c: npred.forward_cond(c, conds[0]), xc, xi, x_cat, ws, state))


if __name__ == "__main__":
    main()
