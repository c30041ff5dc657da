"""Experiment harness: time knn3_interp on recorded inputs of the bench trajectory.
  python tools/knn_replay.py record FILE   (production library: records 8 steps' inputs)
  PCST_LIB=... python tools/knn_replay.py time FILE   (times each recorded call, 20 reps)"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pointcloud_style_transfer_amd import _hip  # noqa: E402

mode, path = sys.argv[1], sys.argv[2]
if mode == "record":
    from pointcloud_style_transfer_amd.config.config import Config
    from pointcloud_style_transfer_amd.models.diffusion_model import (DiffusionProcess,
                                                                        PointCloudDiffusionModel)
    from pointcloud_style_transfer_amd.synthetic import lidar_like_cloud, standard_normal
    cfg = Config(precision="bf16", make_dirs=False)
    torch.manual_seed(0)
    m = PointCloudDiffusionModel(cfg).cuda().eval()
    dp = DiffusionProcess(cfg, "cuda")
    src = torch.from_numpy(lidar_like_cloud(1000, 120000)[None]).cuda()
    cond = torch.from_numpy(lidar_like_cloud(2000, 120000)[None]).cuda()
    x = torch.from_numpy(standard_normal(3000, (1, 120000, 3))).cuda()
    hp, npred = m.hierarchical_processor, m.noise_predictor
    keep = {0, 1, 5, 50, 200, 500, 800, 999}
    rec = []
    with torch.no_grad():
        style = m.style_encoder(hp.downsample(cond)[0])
        style_in = torch.cat([style, torch.zeros_like(style)])
        ts = torch.linspace(999, 0, 1000).long().tolist()
        x_cat = torch.cat([x, x]).contiguous()
        for i, t in enumerate(ts):
            tp = ts[i + 1] if t > 0 else -1
            xc, xi = hp.downsample(x_cat)
            nc = npred(xc, torch.full((2,), t, device="cuda"), style_in)
            eps = _hip.knn3_interp(nc, x_cat, xi)
            if i in keep:
                rec.append((i, nc.cpu(), x_cat.cpu(), xi.cpu(), eps.cpu()))
            x = _hip.cfg_ddim_step(x, eps[:1], eps[1:], src, 7.5, dp._coeffs(t, tp), x_cat=x_cat)
    torch.save(rec, path)
    print("recorded", [r[0] for r in rec])
else:
    rec = torch.load(path, weights_only=True)
    tot = 0.0
    line = []
    bad = 0
    for i, nc, xcat, xi, ref in rec:
        nc, xcat, xi = nc.cuda(), xcat.cuda(), xi.cuda()
        out = _hip.knn3_interp(nc, xcat, xi)
        bad += int((out.cpu() != ref).any())
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        torch.cuda.synchronize()
        ev[0].record()
        for _ in range(20):
            _hip.knn3_interp(nc, xcat, xi)
        ev[1].record()
        torch.cuda.synchronize()
        us = ev[0].elapsed_time(ev[1]) / 20 * 1e3
        tot += us
        line.append(f"{i}:{us:.0f}")
    print(f"mean {tot / len(rec):.1f} us/call  mismatching steps {bad}  [" + " ".join(line) + "]")
