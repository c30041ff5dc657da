"""`PointCloudPreprocessor` (data/preprocessing.py:9-175): host normalisation plus the offline
hierarchical preprocessing that writes the `*_hierarchical.pt` training files.

  * normalize / denormalize (:21-42): float64 numpy, as the reference;
  * _voxel_grid_downsample_numpy (:45-104): the per-point voxel coordinates and centre
    distances come from `pcst_voxel_center_dist` (csrc/preprocess.hip); the grouping (first-
    appearance voxel order, nearest-to-centre point with the lowest index on ties) is a stable
    sort of the device arrays.  The representative set is bit-exact with the reference.  The
    random pad / subsample draws use `rng` (numpy Generator or RandomState, default the global
    numpy RNG like the reference's np.random.choice) over the pool in ascending order; the
    reference's pool is a Python set, whose iteration order is not reproduced;
  * consistent_upsample (:106-119): the float64 3-NN IDW of `pcst_knn3_interp` (bit-exact with
    sklearn's KD-tree);
  * create_hierarchical_data / save_hierarchical_data (:121-175): the same dict and file name.
"""
from __future__ import annotations

import os
from typing import Dict, Tuple

import numpy as np
import torch

from .. import _hip
from ..synthetic import denormalize_point_cloud, normalize_point_cloud


class PointCloudPreprocessor:
    def __init__(self, total_points: int = 120000, global_points: int = 30000,
                 device: str = "cuda", rng=None):
        self.total_points = total_points
        self.global_points = global_points
        self.device = torch.device(device)
        self.rng = rng if rng is not None else np.random

    def normalize_point_cloud(self, points: np.ndarray, target_range: float = 1.8):
        return normalize_point_cloud(points, target_range)

    def denormalize_point_cloud(self, points: np.ndarray, norm_params: dict) -> np.ndarray:
        return denormalize_point_cloud(points, norm_params)

    # ------------------------------------------------------------------ voxel downsample
    def voxel_representatives(self, points: np.ndarray, target_size: int) -> np.ndarray:
        """Indices of the voxel representatives in first-appearance voxel order
        (preprocessing.py:56-93); float32 voxel grid math as numpy does it."""
        points = np.ascontiguousarray(points)
        xyz_min = points.min(axis=0)
        xyz_range = points.max(axis=0) - xyz_min
        xyz_range[xyz_range < 1e-6] = 1.0
        voxel_size = (xyz_range.prod() / target_size) ** (1 / 3) * 1.2
        if voxel_size < 1e-6:
            voxel_size = np.float32(1e-3)  # the reference's python float acts as float32 here
        if points.dtype != np.float32 or np.asarray(voxel_size).dtype != np.float32:
            raise RuntimeError("voxel downsample: the device path reproduces float32 inputs only")
        pts = torch.from_numpy(points).to(self.device)
        key, dist = _hip.voxel_center_dist(pts, xyz_min, voxel_size)
        n = key.shape[0]
        idx = torch.arange(n, device=self.device)
        # lexicographic (key, dist, idx): stable sorts from the least significant field
        o = torch.sort(dist, stable=True)[1]
        o = o[torch.sort(key[o], stable=True)[1]]
        ks = key[o]
        head = torch.ones(n, dtype=torch.bool, device=self.device)
        head[1:] = ks[1:] != ks[:-1]
        reps = o[head]                                  # nearest-to-centre point per voxel
        gid = torch.cumsum(head.long(), 0) - 1          # voxel group of each sorted point
        first = torch.full((int(head.sum()),), n, dtype=torch.long, device=self.device)
        first = first.scatter_reduce(0, gid, idx[o], reduce="amin")
        return reps[torch.argsort(first)].cpu().numpy()  # dict insertion order

    def _voxel_grid_downsample_numpy(self, points: np.ndarray,
                                     target_size: int) -> Tuple[np.ndarray, np.ndarray]:
        n_points = points.shape[0]
        if n_points <= target_size:
            return points, np.arange(n_points)
        selected = self.voxel_representatives(points, target_size)
        if len(selected) < target_size:
            keep = np.ones(n_points, dtype=bool)
            keep[selected] = False
            pool = np.nonzero(keep)[0]
            if len(pool) > 0:
                extra = self.rng.choice(pool, min(target_size - len(selected), len(pool)),
                                        replace=False)
                selected = np.concatenate([selected, extra])
        elif len(selected) > target_size:
            selected = self.rng.choice(selected, target_size, replace=False)
        final = np.asarray(selected, dtype=int)
        return points[final], final

    def consistent_downsample(self, points: np.ndarray,
                              target_size: int) -> Tuple[np.ndarray, np.ndarray]:
        return self._voxel_grid_downsample_numpy(points, target_size)

    def consistent_upsample(self, coarse_points: np.ndarray, original_points: np.ndarray,
                            coarse_indices: np.ndarray) -> np.ndarray:
        dev = self.device
        out = _hip.knn3_interp(torch.from_numpy(np.asarray(coarse_points, np.float32))[None].to(dev),
                               torch.from_numpy(np.asarray(original_points, np.float32))[None].to(dev),
                               torch.from_numpy(np.asarray(coarse_indices, np.int64))[None].to(dev))
        return out[0].cpu().numpy()

    # ------------------------------------------------------------------ files
    def create_hierarchical_data(self, points: np.ndarray) -> Dict:
        points_norm, norm_params = self.normalize_point_cloud(points)
        points_norm = points_norm.astype(np.float32)
        global_points, global_indices = self.consistent_downsample(points_norm, self.global_points)
        return {"full_points": points_norm, "global_points": global_points,
                "global_indices": global_indices, "norm_params": norm_params}

    def _resample(self, points: np.ndarray) -> np.ndarray:
        if len(points) > self.total_points:
            return self._voxel_grid_downsample_numpy(points, self.total_points)[0]
        return points[self.rng.choice(len(points), self.total_points, replace=True)]

    def save_hierarchical_data(self, sim_points: np.ndarray, real_points: np.ndarray,
                               output_dir: str, file_id: str) -> str:
        os.makedirs(output_dir, exist_ok=True)
        if len(sim_points) != self.total_points:
            sim_points = self._resample(sim_points)
        if len(real_points) != self.total_points:
            real_points = self._resample(real_points)
        sim = self.create_hierarchical_data(sim_points)
        real = self.create_hierarchical_data(real_points)
        data = {
            "sim_full": sim["full_points"], "sim_global": sim["global_points"],
            "sim_global_indices": sim["global_indices"], "sim_norm_params": sim["norm_params"],
            "real_full": real["full_points"], "real_global": real["global_points"],
            "real_global_indices": real["global_indices"], "real_norm_params": real["norm_params"],
            "total_points": self.total_points, "global_points": self.global_points,
        }
        path = os.path.join(output_dir, f"{file_id}_hierarchical.pt")
        torch.save(data, path)
        return path
