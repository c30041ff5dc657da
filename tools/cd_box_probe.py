"""Overflow-row statistics of the hybrid Chamfer forward (experiment build with
-DPCST_X_CG_BOX_STATS: list rows report min = -1 and the number of boxes they scanned as the
argmin).  Pairs: a lidar-like target and pred = target + noise x scale (the trainer's pred_x0 at
growing timesteps).  Prints one JSON line per scale: list rows per side and mean / p90 / max boxes.

    PCST_LIB=.../libpcst_hip_v_boxstats.so python tools/cd_box_probe.py
"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from pointcloud_style_transfer_amd import _hip
    from pointcloud_style_transfer_amd.synthetic import lidar_like_cloud

    B, N = 8, 30000
    rng = np.random.default_rng(0)
    q = np.stack([lidar_like_cloud(300 + i, N) for i in range(B)]).astype(np.float32)
    Q = torch.from_numpy(q).cuda()
    for scale in (0.02, 0.1, 0.3, 1.0, 3.0, 10.0, 30.0, 100.0):
        p = (q + rng.standard_normal(q.shape) * scale).astype(np.float32)
        P = torch.from_numpy(p).cuda()
        B_, N_, _ = P.shape
        min1 = torch.empty(B, N, device="cuda")
        min2 = torch.empty(B, N, device="cuda")
        a1 = torch.empty(B, N, dtype=torch.int32, device="cuda")
        a2 = torch.empty(B, N, dtype=torch.int32, device="cuda")
        ws = _hip._workspace("pcst_chamfer_fwd_workspace_size", B, N, N, device=P.device)
        _hip._call("pcst_chamfer_fwd", _hip._ptr(P), _hip._ptr(Q), B, N, N, _hip._ptr(min1),
                   _hip._ptr(a1), _hip._ptr(min2), _hip._ptr(a2), None, 3, _hip._ptr(ws),
                   _hip._stream())
        torch.cuda.synchronize()
        out = {"scale": scale, "extent": float(np.abs(q).max())}
        for name, m, a in (("pred_rows", min1, a1), ("target_rows", min2, a2)):
            sel = (m == -1.0)
            cnt = a[sel].float().cpu().numpy()
            out[name] = {"list": int(sel.sum()), "mean_boxes": float(cnt.mean()) if cnt.size else 0.0,
                         "p90": float(np.percentile(cnt, 90)) if cnt.size else 0.0,
                         "max": float(cnt.max()) if cnt.size else 0.0}
        t0 = torch.cuda.Event(enable_timing=True)
        t1 = torch.cuda.Event(enable_timing=True)
        t0.record()
        for _ in range(5):
            _hip.chamfer_fwd(P, Q, 3)
        t1.record()
        torch.cuda.synchronize()
        out["fwd_ms"] = t0.elapsed_time(t1) / 5
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
