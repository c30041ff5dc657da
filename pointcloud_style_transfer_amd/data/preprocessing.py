"""Host-side normalisation used by the inference entry point (`data/preprocessing.py:21-42`):
centre = mean, scale = 1.8 / max|p - c| in float64.  The offline numpy voxel preprocessing of
the reference (:45-175) is out of scope."""
import numpy as np

from ..synthetic import denormalize_point_cloud, normalize_point_cloud


class PointCloudPreprocessor:
    def __init__(self, total_points: int = 120000, global_points: int = 30000):
        self.total_points = total_points
        self.global_points = global_points

    def normalize_point_cloud(self, points: np.ndarray, target_range: float = 1.8):
        return normalize_point_cloud(points, target_range)

    def denormalize_point_cloud(self, points: np.ndarray, norm_params: dict) -> np.ndarray:
        return denormalize_point_cloud(points, norm_params)
