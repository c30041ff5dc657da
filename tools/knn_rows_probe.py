"""kNN layouts side by side on a sampling step's inputs (experiments only): the compact build +
query (pcst_knn3_build / _query) and the rows layout (pcst_knn3_rows_*), on the bench's 120k
cloud at the start of the trajectory (x_T, Gaussian) and on a late-trajectory-like cloud (the
LiDAR-like source), CFG batch of 2 rows with the voxel downsample's own indices.  Prints per
layout: chunks, outliers, overflow refs and the HIP-event time of each phase.

    python tools/knn_rows_probe.py
"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from pointcloud_style_transfer_amd import _hip  # noqa: E402
from pointcloud_style_transfer_amd.synthetic import lidar_like_cloud, standard_normal  # noqa: E402


def timed(fn, reps=5, before=None):
    """median HIP-event time of fn (us); `before` runs untimed ahead of every repetition (a
    query's outlier counter accumulates: each timed query gets a fresh build)"""
    ts = []
    out = None
    for _ in range(reps):
        if before is not None:
            before()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        out = fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    return out, float(np.median(ts))


def main():
    dev = torch.device("cuda", 0)
    N, T = 120000, 30000
    for name, x_np in (("x_T gaussian", standard_normal(3000, (1, N, 3))),
                       ("lidar-like", lidar_like_cloud(1000, N)[None])):
        x = torch.from_numpy(np.ascontiguousarray(x_np, np.float32)).to(dev)
        for src in ("voxel", "distinct"):
            if src == "voxel":
                _, idx = _hip.voxel_downsample(x, T, seed=77, copies=2)
            else:  # distinct indices: no repeats, no overflow
                g = torch.Generator(device="cpu").manual_seed(5)
                idx = torch.stack([torch.randperm(N, generator=g)[:T] for _ in range(2)]).to(dev)
            probe(name, src, x, idx.contiguous(), N, T, dev)


def probe(name, src, x, idx, N, T, dev):
    x_cat = torch.cat([x, x]).contiguous()
    coarse = torch.randn(2, T, 3, device=dev)
    rec = {"cloud": name, "idx": src,
           "dup_refs": [int(T - torch.unique(idx[b]).numel()) for b in range(2)]}
    ws = _hip.knn_workspace(2, N, T, dev)
    h, rec["compact_build_us"] = timed(lambda: _hip.knn3_build(x_cat, idx, ws))
    ref, rec["compact_query_us"] = timed(lambda: _hip.knn3_query(coarse, h),
                                         before=lambda: _hip.knn3_build(x_cat, idx, ws))
    st = torch.zeros(5, dtype=torch.int32, device=dev)
    _hip.lib().pcst_knn_stats(_hip._ptr(ws), 2, N, T, _hip._ptr(st), _hip._stream())
    st = st.cpu().tolist()
    rec["compact"] = {"err": st[0], "chunks": st[1:3], "outliers": st[3:5]}
    rws = _hip.knn_rows_workspace(1, 2, N, T, dev)
    hr, rec["rows_build_us"] = timed(lambda: _hip.knn3_rows_build(x, T, 2, rws))
    _, rec["rows_refs_us"] = timed(lambda: _hip.knn3_rows_refs(hr, idx),
                                   before=lambda: _hip.knn3_rows_build(x, T, 2, rws))
    got, rec["rows_query_us"] = timed(
        lambda: _hip.knn3_rows_query(coarse, hr),
        before=lambda: _hip.knn3_rows_refs(_hip.knn3_rows_build(x, T, 2, rws), idx))
    rec["rows"] = _hip.knn_rows_stats(hr)
    rec["bit_identical"] = bool(torch.equal(got, ref))
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
