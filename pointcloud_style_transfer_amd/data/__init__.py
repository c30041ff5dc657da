from .dataset import HierarchicalPointCloudDataset, create_dataloaders
from .preprocessing import PointCloudPreprocessor

__all__ = ["PointCloudPreprocessor", "HierarchicalPointCloudDataset", "create_dataloaders"]
