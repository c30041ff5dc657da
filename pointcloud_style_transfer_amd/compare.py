"""`compare.py` (reference repo root, compare.py:1-98): precision / recall / F-score of two
.npy clouds at a distance threshold, with the nearest-neighbour queries on the device
(`pcst_knn_dist`, exact float64 distances) instead of two host cKDTrees.

    python -m pointcloud_style_transfer_amd.compare a.npy b.npy [--threshold 0.2]
"""
from __future__ import annotations

import argparse
import os

import numpy as np
import torch

from . import _hip


def calculate_similarity(pcd1: np.ndarray, pcd2: np.ndarray, threshold: float,
                         device: str = "cuda") -> tuple:
    """compare.py:6-43 -> (precision %, recall %, F1).  pcd1 is the reference cloud."""
    a = torch.as_tensor(np.asarray(pcd1, dtype=np.float32)).to(device)[None]
    b = torch.as_tensor(np.asarray(pcd2, dtype=np.float32)).to(device)[None]
    d21 = _hip.knn_dist(b, a, 1)[0, :, 0]
    d12 = _hip.knn_dist(a, b, 1)[0, :, 0]
    precision = np.mean((d21 < threshold).cpu().numpy())
    recall = np.mean((d12 < threshold).cpu().numpy())
    if precision + recall == 0:
        f_score = 0.0
    else:
        f_score = 2 * (precision * recall) / (precision + recall)
    return precision * 100, recall * 100, f_score


def main():
    parser = argparse.ArgumentParser(description="Point counts and similarity of two .npy clouds.")
    parser.add_argument("file1", type=str, help="reference cloud (.npy, N x 3)")
    parser.add_argument("file2", type=str, help="generated cloud (.npy, N x 3)")
    parser.add_argument("--threshold", type=float, default=0.2,
                        help="distance threshold (metres), default 0.2")
    args = parser.parse_args()
    for f in (args.file1, args.file2):
        if not os.path.exists(f):
            print(f"error: file not found -> {f}")
            return
    try:
        pcd1 = np.load(args.file1)
        pcd2 = np.load(args.file2)
        for f, p in ((args.file1, pcd1), (args.file2, pcd2)):
            if p.ndim != 2 or p.shape[1] != 3:
                print(f"error: {os.path.basename(f)} has shape {p.shape}, not (N, 3)")
                return
    except Exception as e:  # noqa: BLE001 (mirrors the reference's catch-all)
        print(f"error loading .npy: {e}")
        return
    print("-" * 50)
    print("point counts:")
    print(f"  - file 1 ({os.path.basename(args.file1)}): {len(pcd1)} points")
    print(f"  - file 2 ({os.path.basename(args.file2)}): {len(pcd2)} points")
    print("-" * 50)
    precision, recall, f_score = calculate_similarity(pcd1, pcd2, args.threshold)
    print(f"similarity (threshold = {args.threshold} m):")
    print(f"  - precision: {precision:.2f}%")
    print(f"  - recall:    {recall:.2f}%")
    print(f"  - F1-score:  {f_score:.4f}")
    print("-" * 50)


if __name__ == "__main__":
    main()
