"""Experiment: the device-drawn voxel downsample's kernels alone and beside the kNN rows build
(phase A) on a second stream, on the bench's noise cloud (120k, CFG x2, 30k coarse).

    rocprofv3 --kernel-trace --stats -d OUT -o run -- python tools/voxel_probe.py [--reps 20]

mode alone: downsample_copies only; mode beside: each downsample with phase A of the kNN rows
build queued on a side stream at the same time (as the sampling step runs them).
A development tool (tools/ only)."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pointcloud_style_transfer_amd import _hip  # noqa: E402
from pointcloud_style_transfer_amd.synthetic import standard_normal  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--modes", default="alone,beside")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    x = torch.from_numpy(standard_normal(3000, (1, 120000, 3))).to(dev)
    ws = _hip.voxel_copies_workspace(1, 120000, 2, dev)
    kws = _hip.knn_rows_workspace(1, 2, 120000, 30000, dev)
    side = torch.cuda.Stream(device=dev)
    eps = torch.cat([x, x]).contiguous()
    x_cat = torch.cat([x, x]).contiguous()
    coeffs = (0.0, 1.0, 0.0, 1.0)  # x' = eps = x: the bench's noise cloud every rep
    for mode in a.modes.split(","):
        for r in range(a.reps):
            # the product's prepared path: the update makes the statistics, zeroing and pool
            # histogram, the downsample then skips them
            x = _hip.cfg_ddim_voxel_prep(x, eps, None, 7.5, coeffs, x_cat, ws, pool_seed=r)
            if mode == "beside":
                side.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(side):
                    _hip.knn3_rows_build(x, 30000, 2, kws)
            _hip.voxel_downsample(x, 30000, seed=r, copies=2, ws=ws, prepped=True, pool=True)
            torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        print(mode, "done", flush=True)


if __name__ == "__main__":
    main()
