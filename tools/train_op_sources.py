"""Where a trainer step's small PyTorch kernels come from: runs a few DiffusionTrainer steps
(tools/bench_train.py's setup) under torch.profiler with python stacks and prints, for the
ops that launch fills and device copies (aten::fill_ / zero_ / copy_ / zeros / ...), the count
per step by the innermost frame inside this repository.

    python tools/train_op_sources.py --steps 2 --warmup 2
"""
import argparse
import collections
import json
import os
import sys
import tempfile

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

OPS = ("aten::fill_", "aten::zero_", "aten::copy_", "aten::zeros", "aten::zeros_like", "aten::clone",
       "aten::contiguous", "aten::to", "aten::_to_copy", "aten::index_put_", "aten::cat", "aten::stack",
       "aten::add_", "aten::mul_", "aten::mul", "aten::add", "aten::sub", "aten::div", "aten::sum",
       "aten::mean", "aten::abs", "aten::copy")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--points", type=int, default=120000)
    ap.add_argument("--batch", type=int, default=8)
    a = ap.parse_args()
    from pointcloud_style_transfer_amd.config.config import Config
    from pointcloud_style_transfer_amd.synthetic import lidar_like_cloud
    from pointcloud_style_transfer_amd.training.trainer import DiffusionTrainer

    device = torch.device("cuda", 0)
    logdir = tempfile.mkdtemp(prefix="pcst_opsrc_")
    cfg = Config(make_dirs=False, log_dir=logdir, checkpoint_dir=logdir, use_amp=True,
                 gradient_accumulation_steps=1, batch_size=a.batch, amp_dtype="float16")
    torch.manual_seed(0)
    tr = DiffusionTrainer(cfg, device=str(device))
    tr.model.train()
    sim = torch.from_numpy(np.stack([lidar_like_cloud(1000 + i, a.points) for i in range(a.batch)]))
    real = torch.from_numpy(np.stack([lidar_like_cloud(2000 + i, a.points) for i in range(a.batch)]))
    batch = {"sim_full": sim.to(device), "real_full": real.to(device)}
    for i in range(a.warmup):
        tr.train_step(batch, i, 1 << 30, next_batch=batch)
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile

    with profile(activities=[ProfilerActivity.CPU], with_stack=True, record_shapes=True) as prof:
        for i in range(a.steps):
            tr.train_step(batch, i, 1 << 30, next_batch=batch if i + 1 < a.steps else None)
        torch.cuda.synchronize()
    counts = collections.Counter()
    for ev in prof.key_averages(group_by_stack_n=12):
        if ev.key not in OPS:
            continue
        frame = "?"
        for fr in ev.stack or []:
            if "pointcloud_style_transfer_amd" in fr or "/tools/" in fr:
                frame = fr.replace(REPO + "/", "")
                break
        counts[(ev.key, frame)] += ev.count
    out = [{"op": k[0], "where": k[1], "per_step": v / a.steps} for k, v in counts.most_common(70)]
    # without python stacks (some builds record none): the same ops by input shapes
    shapes = collections.Counter()
    for ev in prof.key_averages(group_by_input_shape=True):
        if ev.key in OPS:
            shapes[(ev.key, str(ev.input_shapes)[:160])] += ev.count
    out += [{"op": k[0], "shapes": k[1], "per_step": v / a.steps} for k, v in shapes.most_common(60)]
    sys.stdout.write(json.dumps(out, indent=0) + "\n")


if __name__ == "__main__":
    main()
