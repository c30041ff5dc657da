"""Drop-in for the reference's `models/__init__.py:3-33` re-export surface."""
from .diffusion_model import (
    TimeEmbedding,
    StyleEncoder,
    NoisePredictor,
    HierarchicalProcessor,
    PointCloudDiffusionModel,
    DiffusionProcess,
)
from .losses import DiffusionLoss
from .pointnet2_encoder import PointNet2Encoder

__all__ = [
    "TimeEmbedding",
    "StyleEncoder",
    "NoisePredictor",
    "HierarchicalProcessor",
    "PointCloudDiffusionModel",
    "DiffusionProcess",
    "DiffusionLoss",
    "PointNet2Encoder",
]
