"""Synthetic LiDAR-like point clouds.

All inputs are drawn with numpy PCG64 (stable across platforms) and normalised
exactly like the reference's host-side normaliser
(`data/preprocessing.py:21-38`: centre = mean, scale = 1.8 / max|p - c|,
float64 math, then cast to float32).

Seeds: sim clouds 1000+i, real clouds 2000+i, x_T 3000+i,
trainer t 4000, trainer eps 5000, replayed permutations 6000.
"""
from __future__ import annotations

import numpy as np

SIM_SEED = 1000
REAL_SEED = 2000
XT_SEED = 3000


def normalize_point_cloud(points: np.ndarray, target_range: float = 1.8):
    """Mirror of `PointCloudPreprocessor.normalize_point_cloud` (`data/preprocessing.py:21-38`)."""
    center = points.mean(axis=0)
    centered = points - center
    max_abs = np.max(np.abs(centered))
    scale = 1.0 if max_abs < 1e-6 else target_range / max_abs
    return centered * scale, {"center": center, "scale": scale,
                              "method": "isotropic", "target_range": target_range}


def denormalize_point_cloud(points: np.ndarray, params: dict) -> np.ndarray:
    """Mirror of `PointCloudPreprocessor.denormalize_point_cloud` (`data/preprocessing.py:40-42`)."""
    return (points / params["scale"]) + params["center"]


def lidar_like_cloud(seed: int, n: int = 120000, sigma=(1.0, 1.0, 0.15)) -> np.ndarray:
    """Anisotropic Gaussian cloud, normalised to +-1.8, float32 [n, 3]."""
    rng = np.random.Generator(np.random.PCG64(seed))
    pts = rng.standard_normal((n, 3)) * np.asarray(sigma, dtype=np.float64)
    return normalize_point_cloud(pts)[0].astype(np.float32)


def standard_normal(seed: int, shape) -> np.ndarray:
    rng = np.random.Generator(np.random.PCG64(seed))
    return rng.standard_normal(shape).astype(np.float32)
