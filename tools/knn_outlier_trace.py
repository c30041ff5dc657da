"""Experiment: per-query timing of the rows-layout kNN outlier launch (an experiment build with
-DPCST_KNN_OUTLIER_TRACE, loaded through PCST_LIB).

    make -C pointcloud_style_transfer_amd/csrc OUT=../libpcst_hip_v_otrace.so BUILD=build_v_otrace \\
        "XDEF=-DPCST_KNN_OUTLIER_TRACE"
    PCST_LIB=$PWD/pointcloud_style_transfer_amd/libpcst_hip_v_otrace.so python tools/knn_outlier_trace.py

The bench's first-step cloud (x_T, 120k, CFG x2, 30k device-drawn coarse points per row) and two
later-looking clouds (a lidar-like slab, a clustered cloud): per outlier query its start / end in
10 ns ticks, the brick shells it scanned, whether it started without a bound (the query pass found
fewer than 3 refs), its final radius and the refs it staged.  A development tool (tools/ only)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import knobs  # noqa: E402

knobs.apply()
from pointcloud_style_transfer_amd import _hip  # noqa: E402
from pointcloud_style_transfer_amd.synthetic import standard_normal  # noqa: E402
from knn_chunk_trace import rows_obound_offset  # noqa: E402


def trace(x, M, label):
    dev = x.device
    N = x.shape[1]
    ws = _hip.knn_rows_workspace(1, 2, N, M, dev)
    coarse = torch.randn(2, M, 3, device=dev)
    off = rows_obound_offset(1, 2, N, M)
    for rep in range(3):
        xc, xi = _hip.voxel_downsample(x, M, seed=rep, copies=2)
        h = _hip.knn3_rows_build(x, M, 2, ws)
        _hip.knn3_rows_refs(h, xi)
        for b in range(2):
            o = off + (b * N + 80000) * 4
            ws[o:o + 8192 * 16].zero_()
        _hip.knn3_rows_query(coarse, h)
        torch.cuda.synchronize()
    st = _hip.knn_rows_stats(h)
    tr = []
    for b in range(2):
        n = min(st["outliers"][b], 8192)
        o = off + (b * N + 80000) * 4
        tr.append(ws[o:o + n * 16].view(torch.int32).view(n, 4).cpu().numpy().astype(np.int64))
    tr = np.concatenate(tr)
    if len(tr) == 0:
        print(label, "no outliers")
        return
    t0, t1 = tr[:, 0] & 0xFFFFFFFF, tr[:, 1] & 0xFFFFFFFF
    base = t0.min()
    s, e = (t0 - base) / 100.0, (t1 - base) / 100.0
    d = e - s
    shells, inf, rad, staged = tr[:, 2] & 0x7FFF, (tr[:, 2] >> 15) & 1, tr[:, 2] >> 16, tr[:, 3]
    q = lambda a: " ".join(f"{np.percentile(a, p):.1f}" for p in (10, 50, 90, 99, 100))  # noqa: E731
    print(f"== {label}: outliers {st['outliers']}, launch span {e.max():.1f} us")
    print("  duration p10/50/90/99/max:", q(d))
    print("  start    p10/50/90/99/max:", q(s))
    print("  shells   p10/50/90/99/max:", q(shells), " histogram", np.bincount(shells)[:12].tolist())
    print("  staged   p10/50/90/99/max:", q(staged))
    print(f"  no bound at start: {inf.mean():.3f}; duration with / without bound: "
          f"{d[inf == 0].mean() if (inf == 0).any() else 0:.1f} / {d[inf == 1].mean() if inf.any() else 0:.1f}")
    for k in range(1, 8):
        sel = shells == k
        if sel.any():
            print(f"  shells {k}: n {sel.sum()}, dur mean {d[sel].mean():.1f}, staged mean {staged[sel].mean():.0f}, "
                  f"radius mean {rad[sel].mean():.1f}")
    top = np.argsort(-d)[:5]
    print("  longest:", [(round(float(d[i]), 1), int(shells[i]), int(inf[i]), int(rad[i]), int(staged[i]))
                         for i in top])


def main():
    dev = torch.device("cuda", 0)
    N, M = 120000, 30000
    trace(torch.from_numpy(standard_normal(3000, (1, N, 3))).to(dev), M, "x_T (bench first step)")
    rng = np.random.default_rng(5)
    lid = rng.standard_normal((1, N, 3)).astype(np.float32) * np.array([20.0, 20.0, 1.0], np.float32)
    trace(torch.from_numpy(lid).to(dev), M, "lidar-like slab")
    cen = rng.standard_normal((64, 3)).astype(np.float32) * 5
    cl = (cen[rng.integers(0, 64, N)] + rng.standard_normal((N, 3)).astype(np.float32) * 0.3)[None]
    trace(torch.from_numpy(np.ascontiguousarray(cl)).to(dev), M, "64 clusters")


if __name__ == "__main__":
    main()
