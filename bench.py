"""Benchmark: denoising steps/s of the guided (CFG) sampling loop on 120000-point clouds
(BASELINE.json metric, config 2: 120k sim->real cloud, full 1000-step schedule, bf16 noise
MLP, fp32 geometry), one process per GPU.

A "step" = one iteration of DiffusionProcess.guided_sample_loop (diffusion_model.py:238-260):
voxel downsample of the CFG batch (2 x 120000 -> 2 x 30000; the two rows are copies of x, so
the voxel table is built once and the subset drawn per row), fused noise MLP on 60000 points,
kNN-3 upsample back to 2 x 120000, CFG + DDIM update.  Each rank denoises its own cloud(s)
(independent objects: no data-path collective; scaling "weak").  The one-time style encode is
timed separately and excluded.

Prints ONE JSON line on rank 0 (driver contract), including `roofline` for the dominant
kernel (pcst noise MLP, MFMA-bound) measured with HIP events around its launches inside the
timed region, and `cpu_baseline` (the oracle, a port of the reference path, on host cores).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

FLOP_PER_POINT = 3_540_480          # NoisePredictor MACs x 2
MFMA_BF16_PEAK_TFLOPS = 2500.0      # MI355X dense bf16 (MI355X_MICROARCH.md)
MFMA_F32_PEAK_TFLOPS = 157.3
HBM_PEAK_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # default: one full 1000-step sampling trajectory (t = 999 .. 0)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--clouds-per-gpu", type=int, default=1)
    ap.add_argument("--points", type=int, default=120000)
    ap.add_argument("--precision", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--cpu-steps", type=int, default=3)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--traffic-json", default=os.path.join(REPO, "profiles", "noise_mlp_traffic.json"))
    return ap.parse_args()


def setup_dist(args):
    from pointcloud_style_transfer_amd.distributed import init_from_env

    world, rank, local = init_from_env("nccl")
    if world == 1:
        torch.cuda.set_device(0)
    return world, rank, local


def build_model(precision, device):
    from pointcloud_style_transfer_amd.config.config import Config
    from pointcloud_style_transfer_amd.models.diffusion_model import (DiffusionProcess,
                                                                        PointCloudDiffusionModel)

    cfg = Config(precision=precision, make_dirs=False)
    torch.manual_seed(0)  # random-init weights of the reference architecture
    model = PointCloudDiffusionModel(cfg).to(device).eval()
    return cfg, model, DiffusionProcess(cfg, device=str(device))


def cpu_baseline(args, cfg, model, src, cond, xT):
    """The oracle (numpy + C port of the reference path) on host cores: per-step cost of the
    same guided step on the same 120k clouds, (t(1+k) - t(1)) / k."""
    from oracle import oracle as O

    threads = int(os.environ.get("OMP_NUM_THREADS", str(min(os.cpu_count() or 1, 16))))
    sd = {k: v.detach().float().cpu().numpy() for k, v in model.state_dict().items()}
    sched = O.Schedule()
    ts = O.timesteps_for(1000, 1000)
    rng = np.random.default_rng(6000)

    class RandReplay:  # fresh permutations for every downsample (the oracle never draws itself)
        def next(self, kind):
            raise RuntimeError

    B = 1
    x = xT[:1].copy()
    style = np.zeros((1, 256), np.float32) + 0.1
    style_in = np.concatenate([style, np.zeros_like(style)])

    def step(i):
        nonlocal x
        t = ts[i]
        x_in = np.concatenate([x, x])
        outs, idxs = [], []
        for b in range(2):
            reps, _, _ = O.voxel_reps(x_in[b], cfg.global_points)
            perm = rng.permutation(len(x_in[b]) - len(np.unique(reps))) if len(reps) < cfg.global_points \
                else rng.permutation(len(reps))
            p, ix = O.voxel_downsample(x_in[b:b + 1], cfg.global_points, O.Replay([("randperm", perm)]))
            outs.append(p[0])
            idxs.append(ix[0])
        xc, xi = np.stack(outs), np.stack(idxs)
        nc = O.noise_predictor(sd, xc, np.full(2, t), style_in)
        eps = O.upsample_knn(nc, x_in, xi)
        x = O.guided_update(sched, x, eps[:B], eps[B:], src[:1], t, ts[i + 1], 7.5)

    t0 = time.perf_counter()
    step(0)
    t1 = time.perf_counter()
    for i in range(1, 1 + args.cpu_steps):
        step(i)
    t2 = time.perf_counter()
    per = (t2 - t1) / args.cpu_steps
    return {"value": round(1.0 / per, 4), "unit": "denoising-steps/s", "cores": threads,
            "kind": "port",
            "sample": f"oracle guided step on 1 x {args.points}-pt cloud (CFG x2, 30k coarse), "
                      f"{args.cpu_steps} steps after 1 untimed (first {t1 - t0:.1f}s), "
                      f"{per:.2f} s/step; numpy/OpenBLAS fp32 MLP + C voxel/kNN"}


def encoder_rooflines(xc, device, reps=5):
    """SA1 farthest-point sampling (512 of 30000) and ball query (r 0.2, 32) on the coarse
    condition cloud, timed with HIP events on the launch stream; achieved bandwidth in the
    SURVEY §8d scan model (FPS npoint*N*16 B, ball query S*N*12 B + S*ns*8 B)."""
    from pointcloud_style_transfer_amd import _hip

    B, N, _ = xc.shape
    start = torch.zeros(B, dtype=torch.long, device=device)
    ev = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731
    t_fps, t_bq = [], []
    for _ in range(reps):
        e0, e1, e2 = ev(), ev(), ev()
        e0.record()
        idx = _hip.fps(xc, 512, start)
        e1.record()
        new_xyz = _hip.index_points(xc, idx)
        e2.record()
        _hip.ball_query(0.2, 32, xc, new_xyz)
        e3 = ev()
        e3.record()
        torch.cuda.synchronize()
        t_fps.append(e0.elapsed_time(e1))
        t_bq.append(e2.elapsed_time(e3))
    out = {}
    for name, ms, byts in (("fps", min(t_fps), 512 * N * 16 * B),
                           ("ball_query", min(t_bq), (512 * N * 12 + 512 * 32 * 8) * B)):
        gbs = byts / (ms * 1e-3) / 1e9
        out[name] = {"bound": "hbm (scan model)", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 4), "ms": round(ms, 4),
                     "shape": f"B={B} N={N} S=512"}
    return out


def main():
    args = parse()
    world, rank, local = setup_dist(args)
    device = torch.device("cuda", torch.cuda.current_device())
    from pointcloud_style_transfer_amd import _hip
    from pointcloud_style_transfer_amd.synthetic import lidar_like_cloud, standard_normal

    cfg, model, dp = build_model(args.precision, device)
    from pointcloud_style_transfer_amd.distributed import max_over_ranks, shard

    C = args.clouds_per_gpu
    mine = shard(world * C, rank, world)  # this rank's clouds (SURVEY §8d seeds 1000+i ...)
    src_np = np.stack([lidar_like_cloud(1000 + i, args.points) for i in mine])
    cond_np = np.stack([lidar_like_cloud(2000 + i, args.points) for i in mine])
    xT_np = np.stack([standard_normal(3000 + i, (args.points, 3)) for i in mine])
    src = torch.from_numpy(src_np).to(device)
    cond = torch.from_numpy(cond_np).to(device)
    x = torch.from_numpy(xT_np).to(device)

    hp = model.hierarchical_processor
    npred = model.noise_predictor
    with torch.no_grad():
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        style = model.style_encoder(hp.downsample(cond)[0])
        torch.cuda.synchronize()
        style_s = time.perf_counter() - t0
        style_in = torch.cat([style, torch.zeros_like(style)])
        enc = encoder_rooflines(hp.downsample(cond)[0], device)
        # the same kernels at BASELINE configs[4]'s per-GPU batch (256 clouds / 8 GPUs = 32
        # coarse condition clouds in one launch: one workgroup per cloud)
        xb = torch.from_numpy(np.stack([lidar_like_cloud(2000 + i, cfg.global_points)
                                        for i in range(32)])).to(device)
        enc.update({k + "_b32": v for k, v in encoder_rooflines(xb, device).items()})
        npred.packed()
        timesteps = torch.linspace(dp.num_timesteps - 1, 0, dp.num_timesteps).long().tolist()
        t_rows = torch.tensor(timesteps, dtype=torch.long).repeat_interleave(2 * C)
        t_rows = t_rows.view(len(timesteps), 2 * C).to(device)
        x_cat = torch.cat([x, x]).contiguous()
        ev = []

        def step(i, timed):
            nonlocal x
            t = timesteps[i % len(timesteps)]
            t_prev = timesteps[i % len(timesteps) + 1] if t > 0 else -1
            t_in = t_rows[i % len(timesteps)]
            xc, xi = hp.downsample_copies(x, 2)
            if timed:
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                blob, bias = npred.packed()[:2]
                cnd = npred.cond(t_in, style_in)
                e0.record()
                nc = _hip.noise_mlp(xc.reshape(-1, 3), cfg.global_points, cnd, blob, bias,
                                    npred.precision_code).view(2 * C, -1, 3)
                e1.record()
                ev.append((e0, e1))
            else:
                nc = npred(xc, t_in, style_in)
            eps = hp.upsample_knn(nc, x_cat, xi)
            x = _hip.cfg_ddim_step(x, eps[:C], eps[C:], src, 7.5, dp._coeffs(t, t_prev),
                                   x_cat=x_cat)

        for i in range(args.warmup):
            step(i, False)
        # the timed region restarts the sampling trajectory at t = 999 from x_T
        x = torch.from_numpy(xT_np).to(device)
        x_cat.copy_(torch.cat([x, x]))
        if world > 1:
            import torch.distributed as dist

            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(args.steps):
            step(i, True)
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0
        if world > 1:
            dist.barrier()
            elapsed = max_over_ranks(elapsed, device=device)

    mlp_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    flop = FLOP_PER_POINT * 2 * C * cfg.global_points
    peak = MFMA_BF16_PEAK_TFLOPS if args.precision == "bf16" else MFMA_F32_PEAK_TFLOPS
    achieved = flop / (mlp_ms * 1e-3) / 1e12
    traffic = None
    if os.path.exists(args.traffic_json):
        try:
            with open(args.traffic_json) as f:
                traffic = json.load(f).get("hbm_bytes_per_launch")
        except Exception:
            traffic = None
    total_steps = world * C * args.steps
    value = total_steps / elapsed
    if rank == 0:
        base = None
        if not args.no_cpu_baseline:
            torch.cuda.synchronize()
            base = cpu_baseline(args, cfg, model, src_np, cond_np, xT_np)
        line = {
            "metric": "denoising-steps/sec on 120k-pt cloud",
            "value": round(value, 3),
            "unit": "denoising-steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": args.precision,
            "data": "synthetic (numpy PCG64 anisotropic Gaussian clouds, random-init weights)",
            "config": {"workload": "guided_sample_loop step, 120000-pt sim->real cloud, CFG x2, "
                                   "30000 coarse, full 1000-step schedule (BASELINE configs[1])",
                       "points": args.points, "coarse_points": cfg.global_points,
                       "clouds_per_gpu": C, "guidance_scale": 7.5,
                       "parallelism": f"independent clouds x{world}",
                       "style_encode_s": round(style_s, 4)},
            "roofline": {"kernel": "pcst noise_mlp", "bound": "mfma",
                         "achieved": round(achieved, 2), "peak": peak, "unit": "TFLOP/s",
                         "frac": round(achieved / peak, 4), "traffic": traffic,
                         "algorithmic": f"{FLOP_PER_POINT} FLOP/pt x {2 * C * cfg.global_points} pts",
                         "avg_launch_ms": round(mlp_ms, 4)},
            "cpu_baseline": base,
            "encoder_rooflines": enc,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        import torch.distributed as dist

        dist.destroy_process_group()


if __name__ == "__main__":
    main()
