"""Host utilities of the hot path's entry points (reference `utils/__init__.py:1-11`; the
matplotlib/open3d visualiser is out of scope)."""
from .checkpoint import CheckpointManager
from .ema import ExponentialMovingAverage
from .logger import Logger

__all__ = ["Logger", "CheckpointManager", "ExponentialMovingAverage"]
