"""Worker of tests/test_gpu_ddp.py (not a test module): one DiffusionTrainer process.

    python tests/ddp_worker.py OUT.npz ACCUM MICRO_BATCHES_PER_RANK CLOUDS_PER_MICRO POINTS \
        [AMP GLOBAL_POINTS BACKEND]

Under torch.distributed (RANK / WORLD_SIZE in the environment, gloo backend, every rank on
cuda:0) the trainer wraps the model in DDP; without it the same code is the single-process
reference.  Global micro-batch g (rank r, local step b: g = r * MICRO + b) trains on clouds
[g * CLOUDS, (g + 1) * CLOUDS) with the draws of rng.CounterRNG(100 + g), so both set-ups see
the same samples and the same t / noise / cond-drop / voxel / FPS draws.  The gradient each
optimizer step applies (after clipping) and the parameters after the step are saved (every
rank's parameters: OUT.rankR.npz for R > 0).  AMP=1 (or bf16) runs the trainer under use_amp
with Config.amp_dtype "bfloat16" (the bf16 fused NoisePredictor and GEMMs) and the GradScaler
disabled, so gradients compare unscaled; AMP=fp16 runs the reference's float16 autocast with the
GradScaler at a fixed scale (its unscale_ is exact: a power of two).
BACKEND=nccl (world 1, no RANK / WORLD_SIZE in the environment): a one-rank RCCL process group
on cuda:0 and DiffusionTrainer(ddp=True), so DDP's reducer all-reduces through RCCL (the smoke
of the transport the 8-GPU node uses); the libraries the process mapped are saved as `libs`.
"""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    out, accum, micro, clouds, points = sys.argv[1], *map(int, sys.argv[2:6])
    amp_arg = sys.argv[6] if len(sys.argv) > 6 else "0"
    amp = amp_arg != "0"
    amp_dtype = "float16" if amp_arg == "fp16" else "bfloat16"
    global_points = int(sys.argv[7]) if len(sys.argv) > 7 else 2048
    backend = sys.argv[8] if len(sys.argv) > 8 else "gloo"
    from pointcloud_style_transfer_amd import distributed as D
    from pointcloud_style_transfer_amd import rng
    from pointcloud_style_transfer_amd.config.config import Config
    from pointcloud_style_transfer_amd.synthetic import lidar_like_cloud
    from pointcloud_style_transfer_amd.training.trainer import DiffusionTrainer

    if backend == "nccl":
        import torch.distributed as dist

        world, rank = 1, 0
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda:0"),
                                init_method=f"tcp://127.0.0.1:{os.environ['MASTER_PORT']}")
    else:
        world, rank, _ = D.init_from_env("gloo")
    torch.cuda.set_device(0)
    tmp = os.path.dirname(os.path.abspath(out))
    os.chdir(tmp)
    cfg = Config(make_dirs=False, log_dir=tmp, checkpoint_dir=tmp, use_amp=amp,
                 gradient_accumulation_steps=accum, global_points=global_points,
                 precision="fp32", amp_dtype=amp_dtype)
    torch.manual_seed(0)
    tr = DiffusionTrainer(cfg, device="cuda:0", ddp=True if backend == "nccl" else None)
    assert tr.distributed == (world > 1 or backend == "nccl")
    for m in tr.model.modules():
        if isinstance(m, torch.nn.Dropout):
            m.p = 0.0
    tr.model.train()
    if amp:
        tr.scaler = (torch.amp.GradScaler(init_scale=2.0 ** 14, growth_interval=10 ** 9)
                     if amp_dtype == "float16" else torch.amp.GradScaler(enabled=False))
    grads = {}
    o_step = tr.optimizer.step

    def step(*a, **k):
        for n, p in tr.model.named_parameters():
            grads[n] = p.grad.detach().cpu().numpy().copy()
        return o_step(*a, **k)

    tr.optimizer.step = step
    losses = []
    for b in range(micro):
        g = rank * micro + b
        ids = range(g * clouds, (g + 1) * clouds)
        sim = torch.from_numpy(np.stack([lidar_like_cloud(1000 + i, points) for i in ids]))
        real = torch.from_numpy(np.stack([lidar_like_cloud(2000 + i, points) for i in ids]))
        with rng.replay(rng.CounterRNG(100 + g)):
            loss, _ = tr.train_step({"sim_full": sim.cuda(), "real_full": real.cuda()}, b, micro)
        losses.append(float(loss.detach()))
    torch.cuda.synchronize()
    params = {f"param:{n}": p.detach().cpu().numpy() for n, p in tr.model.named_parameters()}
    with open("/proc/self/maps") as f:
        libs = sorted({ln.split()[-1] for ln in f if ".so" in ln.split()[-1]})
    if rank == 0:
        np.savez(out, losses=np.array(losses), libs=np.array(libs),
                 **{f"grad:{k}": v for k, v in grads.items()}, **params)
    else:
        np.savez(f"{out[:-4]}.rank{rank}.npz", **params)
    if world > 1:
        torch.distributed.barrier()
    if torch.distributed.is_initialized():
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
