"""Experiment harness: per-query records of the brick-shell outlier search on the bench's first
trajectory steps.  PCST_LIB=pointcloud_style_transfer_amd/libpcst_hip_v_trace.so 
python tools/knn_otrace.py   (library built with -DKNN_TRACE)."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pointcloud_style_transfer_amd import _hip  # noqa: E402
from pointcloud_style_transfer_amd.config.config import Config  # noqa: E402
from pointcloud_style_transfer_amd.models.diffusion_model import (DiffusionProcess,  # noqa: E402
                                                                    PointCloudDiffusionModel)
from pointcloud_style_transfer_amd.synthetic import lidar_like_cloud, standard_normal  # noqa: E402

L = _hip.lib()
dump = L.pcst_knn_otrace_dump
dump.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
buf = np.zeros(2 * 4096 * 4, np.uint64)
cfg = Config(precision="bf16", make_dirs=False)
torch.manual_seed(0)
m = PointCloudDiffusionModel(cfg).cuda().eval()
dp = DiffusionProcess(cfg, "cuda")
src = torch.from_numpy(lidar_like_cloud(1000, 120000)[None]).cuda()
cond = torch.from_numpy(lidar_like_cloud(2000, 120000)[None]).cuda()
x = torch.from_numpy(standard_normal(3000, (1, 120000, 3))).cuda()
hp, npred = m.hierarchical_processor, m.noise_predictor
with torch.no_grad():
    style = m.style_encoder(hp.downsample(cond)[0])
    style_in = torch.cat([style, torch.zeros_like(style)])
    ts = torch.linspace(999, 0, 1000).long().tolist()
    x_cat = torch.cat([x, x]).contiguous()
    for i, t in enumerate(ts[:21]):
        tp = ts[i + 1] if t > 0 else -1
        xc, xi = hp.downsample(x_cat)
        nc = npred(xc, torch.full((2,), t, device="cuda"), style_in)
        dump(None, 0)
        st = []
        eps = _hip.knn3_interp(nc, x_cat, xi, stats=st)
        dump(buf.ctypes.data, buf.nbytes)
        if i in (1, 5, 10, 20):
            r = buf.reshape(2, 4096, 4).astype(np.int64)
            for b in range(2):
                rb = r[b][r[b][:, 1] > 0]
                if len(rb) == 0:
                    continue
                t0 = rb[:, 0].min()
                dur = (rb[:, 1] - rb[:, 0]) / 100.0  # us (100 MHz)
                fin = (rb[:, 1] - t0) / 100.0
                sh, lr, stg = rb[:, 2] >> 32, rb[:, 2] & 0xffffffff, rb[:, 3]
                o = np.argsort(dur)[-4:]
                print(f"step {i} row {b}: outliers {st[0]['outliers'][b]} span {fin.max():.1f} us; "
                      f"per query us mean {dur.mean():.1f} p90 {np.percentile(dur, 90):.1f} max {dur.max():.1f}; "
                      f"shells mean {sh.mean():.2f} max {sh.max()}; last r max {lr.max()}; staged mean "
                      f"{stg.mean():.0f} max {stg.max()}", flush=True)
                for j in o:
                    print(f"    slow: {dur[j]:.1f} us shells {sh[j]} r {lr[j]} staged {stg[j]} start {(rb[j, 0]-t0)/100:.1f}")
        x = _hip.cfg_ddim_step(x, eps[:1], eps[1:], src, 7.5, dp._coeffs(t, tp), x_cat=x_cat)
