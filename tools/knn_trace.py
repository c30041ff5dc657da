"""Experiment harness: per-chunk pass timings of the kNN query kernel on the bench trajectory.
  PCST_LIB=pointcloud_style_transfer_amd/libpcst_hip_v_trace.so python tools/knn_trace.py OUT.npz
(the library must be built with -DKNN_TRACE).  Saves, for a few trajectory steps, the raw
per-chunk records (see knn.hip: queries, open lanes after passes 1/2, clock64 stamps, refs
staged per pass, outlier lanes, ball-union volume)."""
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
dump = L.pcst_knn_trace_dump
dump.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
NREC = 2 * 32768 * 8
buf = np.zeros(NREC, np.uint64)

cfg = Config(precision="bf16", make_dirs=False)
torch.manual_seed(0)
m = PointCloudDiffusionModel(cfg).cuda().eval()
dp = DiffusionProcess(cfg, "cuda")
src = torch.from_numpy(lidar_like_cloud(1000, 120000)[None]).cuda()
cond = torch.from_numpy(lidar_like_cloud(2000, 120000)[None]).cuda()
x = torch.from_numpy(standard_normal(3000, (1, 120000, 3))).cuda()
hp, npred = m.hierarchical_processor, m.noise_predictor
keep = {1, 5, 50, 300, 700}
out = {}
with torch.no_grad():
    style = m.style_encoder(hp.downsample(cond)[0])
    style_in = torch.cat([style, torch.zeros_like(style)])
    ts = torch.linspace(999, 0, 1000).long().tolist()
    x_cat = torch.cat([x, x]).contiguous()
    for i, t in enumerate(ts[:max(keep) + 1]):
        tp = ts[i + 1] if t > 0 else -1
        xc, xi = hp.downsample(x_cat)
        nc = npred(xc, torch.full((2,), t, device="cuda"), style_in)
        if i in keep:
            dump(None, 0)
        eps = _hip.knn3_interp(nc, x_cat, xi)
        if i in keep:
            dump(buf.ctypes.data, buf.nbytes)
            out[f"s{i}"] = buf.reshape(2, 32768, 8).copy()
        x = _hip.cfg_ddim_step(x, eps[:1], eps[1:], src, 7.5, dp._coeffs(t, tp), x_cat=x_cat)
np.savez_compressed(sys.argv[1], **out)
for k, r in out.items():
    r = r.reshape(-1, 8)
    r = r[(r[:, 0] & 1) == 1].astype(np.int64)
    t = r[:, 5] - r[:, 2]
    p1, p2, p3 = r[:, 3] - r[:, 2], r[:, 4] - r[:, 3], r[:, 5] - r[:, 4]
    s1, s2, s3 = r[:, 6] >> 32, r[:, 6] & 0xffffffff, r[:, 7] >> 32
    o = (r[:, 7] >> 16) & 0xffff
    top = np.argsort(t)[-5:]
    print(f"{k}: chunks {len(r)} cyc mean {t.mean():.0f} p99 {np.percentile(t, 99):.0f} max {t.max()} | "
          f"pass1 mean {p1.mean():.0f} max {p1.max()} | pass2 mean {p2.mean():.0f} max {p2.max()} | "
          f"pass3 mean {p3.mean():.0f} max {p3.max()} | staged1 mean {s1.mean():.0f} max {s1.max()} | "
          f"outliers {o.sum()}")
    for j in top:
        print("   slow:", t[j], "q", r[j, 0] >> 32, "open", r[j, 1] >> 32, r[j, 1] & 0xffffffff,
              "staged", s1[j], s2[j], s3[j], "ballvol", r[j, 7] & 0xffff, "out", o[j],
              "cyc", p1[j], p2[j], p3[j])
