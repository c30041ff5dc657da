"""Experiment: host enqueue time of DiffusionTrainer.train_step vs its device time (configs[2]:
8 x 120k clouds).  Steps are queued with host_sync=False and no readback; prints the host time
spent in each train_step call and the wall time per step once the device has drained.
A development tool (tools/ only)."""
import os
import sys
import tempfile
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pointcloud_style_transfer_amd.config.config import Config  # noqa: E402
from pointcloud_style_transfer_amd.synthetic import lidar_like_cloud  # noqa: E402
from pointcloud_style_transfer_amd.training.trainer import DiffusionTrainer  # noqa: E402

d = tempfile.mkdtemp()
cfg = Config(make_dirs=False, log_dir=d, checkpoint_dir=d, use_amp=True, gradient_accumulation_steps=1,
             batch_size=8)
torch.manual_seed(0)
tr = DiffusionTrainer(cfg, device="cuda")
tr.model.train()
dev = torch.device("cuda")
sim = torch.from_numpy(np.stack([lidar_like_cloud(1000 + i, 120000) for i in range(8)])).to(dev)
real = torch.from_numpy(np.stack([lidar_like_cloud(2000 + i, 120000) for i in range(8)])).to(dev)
batch = {"sim_full": sim, "real_full": real}
for i in range(3):
    tr.train_step(batch, i, 1 << 30, next_batch=batch)
torch.cuda.synchronize()
for rep in range(2):
    host = []
    t0 = time.perf_counter()
    for i in range(6):
        h0 = time.perf_counter()
        tr.train_step(batch, i, 1 << 30, host_sync=False, next_batch=batch)
        host.append(time.perf_counter() - h0)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"host per train_step {[round(1e3 * h, 2) for h in host]} ms; wall {1e3 * (t2 - t0) / 6:.2f} "
          f"ms/step; device drained {1e3 * (t2 - t1):.1f} ms after the last enqueue", flush=True)
