"""MI355X-native PointNet++-conditioned diffusion hot path of PointCloud_style_transfer.

Mirrors the reference's module tree (config, models, data.preprocessing, utils,
scripts/inference.py, training/trainer.py); compute runs in libpcst_hip.so
(hand-written gfx950 HIP kernels behind the C ABI in include/pcst.h)."""
from .config.config import Config

__all__ = ["Config", "PointCloudDiffusionModel", "DiffusionProcess", "DiffusionTrainer"]


def __getattr__(name):  # lazy: importing the package must not require the native library
    if name in ("PointCloudDiffusionModel", "DiffusionProcess"):
        from .models import diffusion_model

        return getattr(diffusion_model, name)
    if name == "DiffusionTrainer":
        from .training.trainer import DiffusionTrainer

        return DiffusionTrainer
    raise AttributeError(name)
