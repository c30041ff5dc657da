"""tools/voxel_probe.py with tools/knobs.py applied first (PCST_LIB experiment builds)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import knobs  # noqa: E402

knobs.apply()
import voxel_probe  # noqa: E402

voxel_probe.main()
