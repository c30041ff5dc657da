from .preprocessing import PointCloudPreprocessor

__all__ = ["PointCloudPreprocessor"]
