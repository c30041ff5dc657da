"""`evaluation` (evaluation/__init__.py): the metrics on the device.  DiffusionTester
(evaluation/tester.py) is broken at the reference's HEAD and has no counterpart."""
from .metrics import PointCloudMetrics

__all__ = ["PointCloudMetrics"]
