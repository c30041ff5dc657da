"""Benchmark: denoising steps/s of the guided (CFG) sampling loop on 120000-point clouds
(BASELINE.json metric, config 2: 120k sim->real cloud, full 1000-step schedule, bf16 noise
MLP, fp32 geometry), one process per GPU.

A "step" = one iteration of DiffusionProcess.guided_sample_loop (diffusion_model.py:238-260):
voxel downsample of the CFG batch (2 x 120000 -> 2 x 30000; the two rows are copies of x, so
the voxel table is built once and the subset drawn per row), fused noise MLP on 60000 points,
kNN-3 upsample back to 2 x 120000, CFG + DDIM update.  Each rank denoises its own cloud(s)
(independent objects: no data-path collective; scaling "weak").  The one-time style encode is
timed separately (after one warm-up call) and excluded.

`--gpus N` with N > 1 outside torchrun re-launches itself under
`python -m torch.distributed.run --nproc-per-node N` before anything touches the GPU (the
parent only waits for it); under torchrun the world size must equal N.

Prints ONE JSON line on rank 0 (driver contract), including
  * `roofline` for the dominant kernel (pcst noise MLP, MFMA-bound) from HIP events around its
    launches inside the timed region, with `traffic` from the committed PMC summary;
  * `cpu_baseline` (N=1 only): the oracle -- a numpy + C port of the reference path -- timed
    on the host cores over the same 50-step guided loop that the quality leg compares with;
  * `quality` (N=1 only, outside the timed region): "Chamfer vs ref", the second half of
    BASELINE's metric -- the HIP loop (bf16 and fp32 noise MLP) against the oracle loop on
    the same 120k cloud, x_T and counter-keyed draws (rng.CounterRNG);
  * `encoder_rooflines`: FPS / ball query in the SURVEY §8d scan model AND from PMC counters;
  * `batch32` (N=1 only, after the headline): BASELINE configs[4]'s per-GPU share, 32 clouds x
    120k through DiffusionProcess.guided_sample_loop eager and with graph=True, ms per step;
  * `train_step` (N=1 only, after the headline): BASELINE configs[2], DiffusionTrainer.train_step
    on 8 x 120k clouds under fp16 autocast, ms per step and the top three trainer kernels'
    rooflines.
"""
from __future__ import annotations

import argparse
import contextlib
import json
import os
import socket
import subprocess
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
QUALITY_SEED = 6000                 # replayed permutations


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # default: one full 1000-step sampling trajectory (t = 999 .. 0)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=3)
    # HIP events bracket the noise MLP on every EVENT_EVERY-th timed step (the roofline's live
    # launch duration); every step by default (every 4th measured 2751 / 2745 vs 2742 / 2740
    # steps/s: the events cost nothing measurable, profiles/r05/s2e)
    ap.add_argument("--event-every", type=int, default=1)
    ap.add_argument("--clouds-per-gpu", type=int, default=1)
    ap.add_argument("--points", type=int, default=120000)
    ap.add_argument("--precision", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--quality-steps", type=int, default=50,
                    help="schedule length of the Chamfer-vs-ref / cpu_baseline loop")
    ap.add_argument("--no-cpu-baseline", action="store_true",
                    help="skip the oracle leg (cpu_baseline and quality)")
    ap.add_argument("--no-encoder", action="store_true")
    ap.add_argument("--no-other-precision", action="store_true",
                    help="skip timing the other noise-MLP precision mode after the headline")
    ap.add_argument("--no-extra", action="store_true",
                    help="skip the batch32 (configs[4]) and train_step (configs[2]) legs")
    ap.add_argument("--traffic-json", default=os.path.join(REPO, "profiles", "noise_mlp_traffic.json"))
    ap.add_argument("--encoder-traffic-json",
                    default=os.path.join(REPO, "profiles", "encoder_traffic.json"))
    return ap.parse_args()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def maybe_spawn(args):
    """--gpus N > 1 without a torchrun environment: start the N ranks as a child torchrun job
    (this process has not touched the GPU) and exit with its code."""
    if args.gpus <= 1 or "WORLD_SIZE" in os.environ:
        return
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr", "127.0.0.1",
           "--master-port", str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    sys.exit(subprocess.call(cmd, env=env))


def setup_dist(args):
    from pointcloud_style_transfer_amd.distributed import init_from_env

    world, rank, local = init_from_env("nccl")
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but the launcher started {world} ranks")
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


def host_cpu():
    """CPU model, physical cores, the CPUs this process may run on, and the BLAS threads the
    oracle uses (= min of the affinity set, OMP_NUM_THREADS and the physical cores).  On the GPU
    box the harness exports OMP_NUM_THREADS=16: one GPU's share of the 8-GPU host's cores, which
    other GPUs' jobs use at the same time.  The cap is recorded with its source."""
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        import psutil

        physical = psutil.cpu_count(logical=False) or os.cpu_count()
    except Exception:  # noqa: BLE001
        physical = os.cpu_count()
    visible = len(os.sched_getaffinity(0))
    omp = os.environ.get("OMP_NUM_THREADS")
    cap = int(omp) if omp else visible
    threads = max(1, min(visible, cap, physical or visible))
    rec = {"cpu_model": model, "physical_cores_on_host": physical,
           "cpus_visible_to_process": visible, "OMP_NUM_THREADS": omp, "threads": threads}
    if threads < (physical or threads):
        rec["cap"] = {"threads": threads,
                      "source": "OMP_NUM_THREADS as found in the environment (the GPU box "
                                "exports 16: one GPU's share of the host CPUs)" if omp else
                                "CPU affinity set of this process"}
    return rec


def oracle_leg(args, cfg, model, dp, src_np, cond_np, xT_np, device):
    """The oracle (numpy + C port of the reference path) runs the reference's guided loop on
    host cores: `quality_steps` steps of linspace(999, 0, n) on cloud 0, counter-keyed draws.
    The same schedule, x_T and draws drive the HIP loop in bf16 and fp32.  Returns
    (cpu_baseline, quality)."""
    from oracle import oracle as O
    from pointcloud_style_transfer_amd import rng as R
    from pointcloud_style_transfer_amd.evaluation.metrics import PointCloudMetrics

    cpu = host_cpu()
    try:
        from threadpoolctl import threadpool_limits

        limiter = threadpool_limits(limits=cpu["threads"])
    except Exception:  # noqa: BLE001
        limiter = None
    S = args.quality_steps
    T = cfg.global_points
    sd = {k: v.detach().float().cpu().numpy() for k, v in model.state_dict().items()}
    sched = O.Schedule(cfg.num_timesteps, cfg.beta_schedule, cfg.noise_schedule_offset)
    ts = O.timesteps_for(cfg.num_timesteps, S)
    ctr = R.CounterRNG(QUALITY_SEED)   # the draw order of guided_sample_loop (see rng.py)

    def down(rows):
        """voxel downsample of every row with the next counter-keyed permutation each."""
        outs, idxs = [], []
        for b in range(rows.shape[0]):
            reps, _, _ = O.voxel_reps(rows[b], T)
            U = len(reps)   # reps may repeat an index (two voxels with the same mean index)
            n = U if U > T else (rows.shape[1] - len(np.unique(reps)) if U < T else 0)
            draws = [("randperm", ctr.generator().permutation(n))] if n else []
            p, ix = O.voxel_downsample(rows[b:b + 1], T, O.Replay(draws))
            outs.append(p[0])
            idxs.append(ix[0])
        return np.stack(outs), np.stack(idxs)

    src, cond, x = src_np[:1], cond_np[:1], xT_np[:1].copy()
    t_enc = time.perf_counter()
    cdown, _ = down(cond)
    starts = [("randint", ctr.generator().integers(0, cdown.shape[1], (1,), dtype=np.int64)),
              ("randint", ctr.generator().integers(0, 512, (1,), dtype=np.int64))]
    style = O.style_encoder(sd, cdown, O.Replay(starts))
    t_enc = time.perf_counter() - t_enc
    style_in = np.concatenate([style, np.zeros_like(style)])
    step_s = []
    for i, t in enumerate(ts):
        t0 = time.perf_counter()
        x_in = np.concatenate([x, x])
        xc, xi = down(x_in)
        nc = O.noise_predictor(sd, xc, np.full(2, t), style_in)
        eps = O.upsample_knn(nc, x_in, xi)
        x = O.guided_update(sched, x, eps[:1], eps[1:], src, int(t),
                            int(ts[i + 1]) if t > 0 else -1, 7.5)
        step_s.append(time.perf_counter() - t0)
    if limiter is not None:
        limiter.restore_original_limits()
    per = float(np.median(step_s[1:])) if len(step_s) > 1 else step_s[0]
    base = {"value": round(1.0 / per, 4), "unit": "denoising-steps/s", "cores": cpu["threads"],
            "kind": "port",
            # not measured: what the same run would give if it scaled linearly to every
            # physical core of the host (an upper bound; the oracle's BLAS does not scale so)
            "linear_upper_bound_all_physical_cores": round(
                (1.0 / per) * (cpu["physical_cores_on_host"] or cpu["threads"]) / cpu["threads"], 3),
            "sample": f"oracle (numpy/OpenBLAS fp32 MLP + C voxel/kNN, port of the reference "
                      f"path) guided loop on 1 x {args.points}-pt cloud, CFG x2, 30k coarse, "
                      f"{S}-step schedule; median of steps 2..{S}: {per:.3f} s/step "
                      f"({sum(step_s):.1f} s total, style encode {t_enc:.2f} s)",
            "host": cpu}

    # the HIP loop on the same inputs and draws, bf16 (measured mode) and fp32 (parity mode)
    met = PointCloudMetrics(device=str(device))
    ref = torch.from_numpy(x).to(device)
    quality = {"definition": "evaluation/metrics.py:20-44 Chamfer (Euclidean, both directions, "
                             "/2) between the HIP output and the oracle output",
               "schedule_steps": S, "points": args.points, "guidance_scale": 7.5,
               "draws": f"rng.CounterRNG({QUALITY_SEED}) on both sides; same x_T (seed 3000)"}
    prec0 = cfg.precision
    for prec in ("bf16", "fp32"):
        cfg.precision = prec
        with R.replay(R.CounterRNG(QUALITY_SEED)):
            out = dp.guided_sample_loop(model, torch.from_numpy(src).to(device),
                                        torch.from_numpy(cond).to(device), S, 7.5,
                                        x_T=torch.from_numpy(xT_np[:1]).to(device))
        d = (out.double() - ref.double()).abs()
        scale = ref.abs().max().double()
        within = (d <= 1e-4 * (ref.abs().double() + 0.1 * scale)).double().mean()
        quality[prec] = {
            "chamfer_vs_ref": float(met.chamfer_distance(out, ref)[0]),
            "frac_within_1e-4": round(float(within), 6),
            "max_abs": float(d.max()),
            "mean_abs": float(d.mean()),
        }
    cfg.precision = prec0
    quality["criterion"] = "|hip - oracle| <= 1e-4 * (|oracle| + 0.1 max|oracle|) per element"
    return base, quality


def encoder_rooflines(xc, device, traffic, tag, reps=5):
    """SA1 farthest-point sampling (512 of 30000) and ball query (r 0.2, 32) on coarse
    condition clouds, timed with HIP events on the launch stream.  Two bandwidth figures:
      * `scan_model`: SURVEY §8d's effective bytes (FPS npoint*N*16 B, ball query
        S*N*12 B + S*ns*8 B) over the time -- a comparison figure; > 1.0 of peak is flagged,
        it means the kernel does not re-stream what the model counts;
      * `counters`: HBM bytes per launch from the committed rocprofv3 PMC pass
        (FETCH_SIZE x2 + WRITE_SIZE, profiles/encoder_traffic.json) over the same time."""
    from pointcloud_style_transfer_amd import _hip

    B, N, _ = xc.shape
    start = torch.zeros(B, dtype=torch.long, device=device)
    ev = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731
    idx = _hip.fps(xc, 512, start)
    new_xyz = _hip.index_points(xc, idx)
    _hip.ball_query(0.2, 32, xc, new_xyz)
    torch.cuda.synchronize()
    # each figure: `reps` back-to-back calls between two events, per call (the calls' host work
    # -- argument checks, workspace, launches -- overlaps the previous call's kernel, as in a
    # pipelined encode; one call between events on an idle device would add it to the time)
    t_fps, t_bq = [], []
    for _ in range(3):
        e0, e1, e2, e3 = ev(), ev(), ev(), ev()
        e0.record()
        for _ in range(reps):
            _hip.fps(xc, 512, start)
        e1.record()
        e2.record()
        for _ in range(reps):
            _hip.ball_query(0.2, 32, xc, new_xyz)
        e3.record()
        torch.cuda.synchronize()
        t_fps.append(e0.elapsed_time(e1) / reps)
        t_bq.append(e2.elapsed_time(e3) / reps)
    out = {}
    for name, ms, byts in (("fps", float(np.median(t_fps)), 512 * N * 16 * B),
                           ("ball_query", float(np.median(t_bq)), (512 * N * 12 + 512 * 32 * 8) * B)):
        gbs = byts / (ms * 1e-3) / 1e9
        rec = {"ms": round(ms, 4), "shape": f"B={B} N={N} S=512",
               "scan_model": {"bytes": byts, "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS,
                              "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 4),
                              "exceeds_peak": gbs > HBM_PEAK_GBS}}
        tb = (traffic or {}).get(f"{name}_{tag}")
        if tb:
            g2 = tb / (ms * 1e-3) / 1e9
            rec["counters"] = {"traffic_bytes": tb, "achieved": round(g2, 2), "peak": HBM_PEAK_GBS,
                               "unit": "GB/s", "frac": round(g2 / HBM_PEAK_GBS, 5)}
        else:
            rec["counters"] = None
        if name == "fps":
            rec["per_round_us"] = round(ms * 1e3 / 512, 3)
            rec["bound"] = "latency (512 dependent arg-max rounds)"
        else:
            rec["bound"] = "latency / L2 (one wave per centroid, early exit at nsample)"
        out[name] = rec
    return out


def batch32_leg(cfg, model, dp, device, clouds=32, points=120000, short=5, long=25):
    """BASELINE configs[4]'s per-GPU share: `clouds` clouds x `points` through the product
    sampling loop (DiffusionProcess.guided_sample_loop), eager and graph=True.  Each mode runs a
    `short`- and a `long`-step schedule on the same inputs; ms per step = the wall difference over
    the extra steps, so the one-time costs both runs share (style encode, conditioning rows,
    workspaces, the graph capture) cancel.  Outside the headline's timed region."""
    from pointcloud_style_transfer_amd.synthetic import lidar_like_cloud, standard_normal

    src = torch.from_numpy(np.stack([lidar_like_cloud(1000 + i, points) for i in range(clouds)])).to(device)
    cond = torch.from_numpy(np.stack([lidar_like_cloud(2000 + i, points) for i in range(clouds)])).to(device)
    xT = torch.from_numpy(np.stack([standard_normal(3000 + i, (points, 3)) for i in range(clouds)])).to(device)
    out = {"workload": f"guided_sample_loop, {clouds} x {points}-pt clouds per GPU, CFG x2, "
                       f"{cfg.global_points} coarse (BASELINE configs[4]: 256 clouds / 8 GPUs)",
           "method": f"(wall({long} steps) - wall({short} steps)) / {long - short}, "
                     "torch.cuda.synchronize() around each loop"}
    for mode, graph in (("eager", False), ("graph", True)):
        dp.guided_sample_loop(model, src, cond, 2, 7.5, x_T=xT, graph=graph)  # workspaces, warm-up
        wall = {}
        for n in (short, long):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            dp.guided_sample_loop(model, src, cond, n, 7.5, x_T=xT, graph=graph)
            torch.cuda.synchronize()
            wall[n] = time.perf_counter() - t0
        ms = (wall[long] - wall[short]) / (long - short) * 1e3
        out[mode] = {"ms_per_step": round(ms, 4), "clouds_steps_per_s": round(clouds * 1e3 / ms, 2),
                     "wall_s": {str(k): round(v, 4) for k, v in wall.items()}}
    return out


def train_leg(device, batch=8, points=120000, steps=5, warmup=2):
    """BASELINE configs[2]: one DiffusionTrainer.train_step (trainer.py:70-127, accumulation 1) on
    `batch` x `points` clouds under fp16 autocast (Config defaults), inputs resident in HBM, ms per
    step over `steps` after `warmup` (each step's loss read after the next is queued, as
    train_one_epoch).  Then two more steps with HIP events around the three largest trainer
    kernels (round-4 profile: the fused residual-block backward and forward, the 16-bit weight
    gradient) on their launch stream: algorithmic FLOP over the summed event time, against the
    dense fp16 MFMA peak."""
    import tempfile

    from pointcloud_style_transfer_amd import _hip
    from pointcloud_style_transfer_amd.config.config import Config
    from pointcloud_style_transfer_amd.synthetic import lidar_like_cloud
    from pointcloud_style_transfer_amd.training.trainer import DiffusionTrainer

    logdir = tempfile.mkdtemp(prefix="pcst_bench_train_")
    cfg = Config(make_dirs=False, log_dir=logdir, checkpoint_dir=logdir, gradient_accumulation_steps=1,
                 batch_size=batch)
    torch.manual_seed(0)
    trainer = DiffusionTrainer(cfg, device=str(device))
    trainer.model.train()
    sim = torch.from_numpy(np.stack([lidar_like_cloud(1000 + i, points) for i in range(batch)]))
    real = torch.from_numpy(np.stack([lidar_like_cloud(2000 + i, points) for i in range(batch)]))
    data = {"sim_full": sim.to(device), "real_full": real.to(device)}
    for i in range(warmup):
        trainer.train_step(data, i, 1 << 30, next_batch=data)

    def run(n):
        pending = loss = None
        for i in range(n):
            step = trainer.train_step(data, i, 1 << 30, host_sync=False,
                                      next_batch=data if i + 1 < n else None)
            if pending is not None:
                loss, _ = pending[1].read()
            pending = step
        loss, _ = pending[1].read()
        return loss

    torch.cuda.synchronize()
    t0 = time.perf_counter()
    loss = run(steps)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / steps * 1e3

    # kernel rooflines: wrap the three ABI calls with events on the stream they launch on
    flops = {"resblock_bwd16": lambda a, k: 4 * a[0].shape[0] * 256 * 512,   # dd W2, dz W1
             "resblock_fwd16": lambda a, k: 4 * a[0].shape[0] * 256 * 512,   # x W1^T, h W2^T
             "linear_wgrad_ex": lambda a, k: 2 * a[0].shape[0] * a[0].shape[1] * a[1].shape[1]}
    kernels = {"resblock_bwd16": "resblock_kernel<true, true> (pcst_resblock_bwd16)",
               "resblock_fwd16": "resblock3_kernel (pcst_resblock_fwd16)",
               "linear_wgrad_ex": "wgrad_ex_kernel + combine (pcst_linear_wgrad_ex)"}
    rec = {k: [] for k in flops}
    orig = {k: getattr(_hip, k) for k in flops}

    def wrap(name):
        fn = orig[name]

        def timed(*a, **k):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            r = fn(*a, **k)
            e1.record()
            rec[name].append((e0, e1, flops[name](a, k)))
            return r
        return timed

    try:
        for k in flops:
            setattr(_hip, k, wrap(k))
        run(2)
        torch.cuda.synchronize()
    finally:
        for k, fn in orig.items():
            setattr(_hip, k, fn)
    roof = {}
    for k, ev in rec.items():
        if not ev:
            roof[k] = None
            continue
        t = sum(a.elapsed_time(b) for a, b, _ in ev)
        f = sum(x for _, _, x in ev)
        tf = f / (t * 1e-3) / 1e12
        roof[k] = {"kernel": kernels[k], "bound": "mfma", "calls_per_step": len(ev) // 2,
                   "avg_launch_ms": round(t / len(ev), 4), "achieved": round(tf, 2),
                   "peak": MFMA_BF16_PEAK_TFLOPS, "unit": "TFLOP/s",
                   "frac": round(tf / MFMA_BF16_PEAK_TFLOPS, 4),
                   "algorithmic": "4 M 256 512 FLOP per block" if k != "linear_wgrad_ex" else "2 M I O FLOP"}
    del trainer
    torch.cuda.empty_cache()
    return {"workload": f"DiffusionTrainer.train_step, {batch} x {points}-pt clouds, L1 + Chamfer, "
                        "accumulation 1 (BASELINE configs[2])",
            "dtype": f"fp32 master weights, autocast {cfg.amp_dtype}" if cfg.use_amp else "fp32",
            "steps": steps, "warmup": warmup, "ms_per_step": round(ms, 3),
            "clouds_per_s": round(batch * 1e3 / ms, 3), "final_loss": float(loss), "rooflines": roof}


def main():
    args = parse()
    maybe_spawn(args)
    world, rank, local = setup_dist(args)
    device = torch.device("cuda", torch.cuda.current_device())
    from pointcloud_style_transfer_amd import _hip
    from pointcloud_style_transfer_amd import rng as _rng
    from pointcloud_style_transfer_amd.distributed import max_over_ranks, shard
    from pointcloud_style_transfer_amd.models import diffusion_model as dmod
    from pointcloud_style_transfer_amd.synthetic import lidar_like_cloud, standard_normal

    cfg, model, dp = build_model(args.precision, device)
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
        model.style_encoder(hp.downsample(cond)[0])   # warm-up (first-call costs)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        style = model.style_encoder(hp.downsample(cond)[0])
        torch.cuda.synchronize()
        style_s = time.perf_counter() - t0
        style_in = torch.cat([style, torch.zeros_like(style)])
        enc = None
        if rank == 0 and not args.no_encoder:
            traffic = None
            if os.path.exists(args.encoder_traffic_json):
                with open(args.encoder_traffic_json) as f:
                    traffic = json.load(f).get("bytes_per_launch")
            enc = encoder_rooflines(hp.downsample(cond)[0][:1], device, traffic, "b1")
            # the same kernels at BASELINE configs[4]'s per-GPU batch (256 clouds / 8 GPUs =
            # 32 coarse condition clouds in one launch: one workgroup per cloud)
            xb = torch.from_numpy(np.stack([lidar_like_cloud(2000 + i, cfg.global_points)
                                            for i in range(32)])).to(device)
            enc.update({k + "_b32": v for k, v in
                        encoder_rooflines(xb, device, traffic, "b32").items()})
        npred.packed()
        timesteps = torch.linspace(dp.num_timesteps - 1, 0, dp.num_timesteps).long().tolist()
        t_rows = torch.tensor(timesteps, dtype=torch.long).repeat_interleave(2 * C)
        t_rows = t_rows.view(len(timesteps), 2 * C).to(device)
        x_cat = torch.cat([x, x]).contiguous()
        ev = []

        # the product loop's stream layout (DiffusionProcess.guided_sample_loop): the step on a
        # high-priority stream, the kNN build on a side stream during the noise MLP
        overlap = dmod.overlap_knn_build(2 * C * cfg.global_points)
        state = dmod.StepState(device) if overlap else None
        loop_stream = state.loop if overlap else None
        if overlap:
            state.begin(torch.cuda.current_stream())
            with torch.cuda.stream(loop_stream):
                knn_ws = _hip.knn_workspace(2 * C, args.points, cfg.global_points, device=device)
                rows_ws = (_hip.knn_rows_workspace(C, 2, args.points, cfg.global_points, device)
                           if dmod.rows_layout_ok(2 * C * cfg.global_points) else None)
        else:
            knn_ws = rows_ws = None

        vws = _hip.voxel_copies_workspace(C, args.points, 2, device=device)
        pk = npred.packed()  # the loop changes no weight (as guided_sample_loop)
        S = len(timesteps)
        # device-scope events: no L2 writeback bubble around the timed kernel
        timing_event = lambda: _hip.DeviceEvent(timing=True)  # noqa: E731
        conds = None  # every step's conditioning rows, one launch per loop (as guided_sample_loop)

        def all_conds():
            return npred.cond(t_rows.reshape(-1), style_in.repeat(S, 1), pk).view(S, 2 * C, -1)

        prepped = pool = False
        next_seed = None

        def step(i, timed):
            nonlocal x, prepped, pool, next_seed
            t = timesteps[i % len(timesteps)]
            t_prev = timesteps[i % len(timesteps) + 1] if t > 0 else -1
            cnd = conds[i % len(timesteps)]
            # the rows layout: the kNN's positions-only phase on the side stream beside the
            # downsample (as guided_sample_loop)
            rows, start = (dmod.knn_rows_begin(x, cfg.global_points, state, rows_ws,
                                               by_downsample=prepped)
                           if rows_ws is not None else (None, None))
            xc, xi = hp.downsample_copies(x, 2, vws, prepped, next_seed, pool, start, rows=rows,
                                          rows_wait=state.built_sig if rows is not None else None)

            def mlp(xc_, wait=None, start=None):
                if not timed:
                    return npred.forward_cond(xc_, cnd, pk, wait, start)
                # on the stream the MLP runs on
                e0, e1 = timing_event(), timing_event()
                blob, bias = pk[:2]
                e0.record()
                nc_ = _hip.noise_mlp(xc_.reshape(-1, 3), cfg.global_points, cnd, blob, bias,
                                     npred.precision_code, wait=wait,
                                     signal=start).view(2 * C, -1, 3)
                e1.record()
                ev.append((e0, e1))
                return nc_

            # the update prepares the next step's downsample, its pool histogram for the next
            # subset seed drawn one step ahead included (as guided_sample_loop does)
            prep = dmod.voxel_prep_ok(hp, x, state)
            next_seed = (_rng.source().device_seed() & (2**64 - 1)
                         if prep and dmod.pool_prep_ok(x) else None)
            x = dmod.hierarchical_step(hp, mlp, xc, xi, x_cat, x, src, 7.5, dp._coeffs(t, t_prev),
                                       knn_ws, state, fused=True, vox_ws=vws if prep else None,
                                       pool_seed=next_seed, rows=rows)
            prepped, pool = prep, next_seed is not None

        lctx = torch.cuda.stream(loop_stream) if overlap else contextlib.nullcontext()
        with lctx:
            conds = all_conds()
            for i in range(args.warmup):
                step(i, False)
            # the timed region restarts the sampling trajectory at t = 999 from x_T
            x = torch.from_numpy(xT_np).to(device)
            x_cat.copy_(torch.cat([x, x]))
            prepped = pool = False
            next_seed = None
        if world > 1:
            import torch.distributed as dist

            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with lctx:
            conds = all_conds()  # the loop's one-time conditioning launch, inside the timed region
            for i in range(args.steps):
                step(i, i % max(1, args.event_every) == 0)
        host_elapsed = time.perf_counter() - t0  # the host's enqueue time (the GPU may still run)
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0
        if overlap:
            state.check()  # a timed-out cross-stream wait invalidates the run: raise
        if world > 1:
            dist.barrier()
            elapsed = max_over_ranks(elapsed, device=device)

        # the other precision mode, same loop and stream layout, outside the timed region
        # (N = 1 only): the fp32 (parity) mode's steps/s beside the bf16 headline
        other = None
        if world == 1 and not args.no_other_precision:
            prec0 = cfg.precision
            cfg.precision = "fp32" if prec0 == "bf16" else "bf16"
            pk = npred.packed()  # the other mode's weight stream
            try:
                with lctx:
                    x = torch.from_numpy(xT_np).to(device)
                    x_cat.copy_(torch.cat([x, x]))
                    prepped = pool = False
                    next_seed = None
                    conds = all_conds()
                    for i in range(2):
                        step(i, False)
                torch.cuda.synchronize()
                t1 = time.perf_counter()
                with lctx:
                    conds = all_conds()
                    for i in range(args.steps):
                        step(i, False)
                torch.cuda.synchronize()
                el = time.perf_counter() - t1
                other = {"precision": cfg.precision, "value": round(C * args.steps / el, 3),
                         "ms_per_step": round(el / args.steps * 1e3, 4),
                         "note": "same loop, steps and stream layout as the headline, timed "
                                 "after it (not part of value)"}
            finally:
                cfg.precision = prec0
                pk = npred.packed()
            if overlap:
                state.check()

    mlp_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    # configs[4] and configs[2], after the headline and outside its timed region (N = 1 only)
    batch32 = train_step = None
    if world == 1 and not args.no_extra:
        with torch.no_grad():
            batch32 = batch32_leg(cfg, model, dp, device)
        torch.cuda.empty_cache()
        train_step = train_leg(device)
    flop = FLOP_PER_POINT * 2 * C * cfg.global_points
    peak = MFMA_BF16_PEAK_TFLOPS if args.precision == "bf16" else MFMA_F32_PEAK_TFLOPS
    achieved = flop / (mlp_ms * 1e-3) / 1e12
    traffic = None
    if os.path.exists(args.traffic_json):
        try:
            with open(args.traffic_json) as f:
                traffic = json.load(f).get("hbm_bytes_per_launch")
        except Exception:  # noqa: BLE001
            traffic = None
    total_steps = world * C * args.steps
    value = total_steps / elapsed
    if rank == 0:
        base = quality = None
        if world == 1 and not args.no_cpu_baseline:
            torch.cuda.synchronize()
            with torch.no_grad():
                base, quality = oracle_leg(args, cfg, model, dp, src_np, cond_np, xT_np, device)
        line = {
            "metric": "denoising-steps/sec on 120k-pt cloud",
            "value": round(value, 3),
            "unit": "denoising-steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            # the host's enqueue time of the timed steps (a diagnostic: below ms_per_step, the
            # host runs ahead of the device)
            "host_enqueue_ms_per_step": round(host_elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": args.precision,
            "data": "synthetic (numpy PCG64 anisotropic Gaussian clouds, random-init weights)",
            "config": {"workload": "guided_sample_loop step, 120000-pt sim->real cloud, CFG x2, "
                                   "30000 coarse, full 1000-step schedule (BASELINE configs[1])",
                       "points": args.points, "coarse_points": cfg.global_points,
                       "clouds_per_gpu": C, "guidance_scale": 7.5,
                       "parallelism": f"independent clouds x{world} (one process per GPU)",
                       "style_encode_s": round(style_s, 4)},
            "roofline": {"kernel": "pcst noise_mlp", "bound": "mfma",
                         "achieved": round(achieved, 2), "peak": peak, "unit": "TFLOP/s",
                         "frac": round(achieved / peak, 4), "traffic": traffic,
                         "algorithmic": f"{FLOP_PER_POINT} FLOP/pt x {2 * C * cfg.global_points} pts",
                         "avg_launch_ms": round(mlp_ms, 4),
                         "timed_launches": len(ev),
                         "timing": f"HIP events on the loop stream around every "
                                   f"{max(1, args.event_every)}th timed step's MLP launch"},
            "other_precision": other,
            "cpu_baseline": base,
            "quality": quality,
            "encoder_rooflines": enc,
            "batch32": batch32,
            "train_step": train_step,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        import torch.distributed as dist

        dist.destroy_process_group()


if __name__ == "__main__":
    main()
