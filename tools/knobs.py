"""A/B knobs for experiment runs (tools/ only; the product modules read no environment).

    import knobs; knobs.apply()

reads PCST_KNN_OVERLAP=0|1, PCST_KNN_BUILD_LDS_FLOOR=<bytes>, PCST_ROWS_LAYOUT=0|1,
PCST_ROWS_MAX_MLP_POINTS=<n>,
PCST_VOXEL_PREP / _POOL_PREP=0|1, PCST_FUSED_BLOCK_FWD / _BWD=0|1 (models._autograd) and sets the
matching module constants of models.diffusion_model.  Kernel-side variants are
experiment builds (csrc/Makefile XDEF): PCST_LIB=<path> points _hip.LIB_PATH at one before the
library is loaded (the product _hip reads no environment)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def apply():
    from pointcloud_style_transfer_amd import _hip
    from pointcloud_style_transfer_amd.models import diffusion_model as dm

    e = os.environ
    if e.get("PCST_LIB"):
        if _hip._lib is not None:
            raise RuntimeError("knobs.apply(): PCST_LIB must be applied before the library loads")
        _hip.LIB_PATH = e["PCST_LIB"]
    if "PCST_KNN_OVERLAP" in e:
        dm.OVERLAP_KNN_BUILD = e["PCST_KNN_OVERLAP"] != "0"
    if "PCST_KNN_BUILD_LDS_FLOOR" in e:
        dm.KNN_BUILD_LDS_FLOOR = int(e["PCST_KNN_BUILD_LDS_FLOOR"])
    if "PCST_VOXEL_PREP" in e:
        dm.VOXEL_PREP = e["PCST_VOXEL_PREP"] != "0"
    if "PCST_POOL_PREP" in e:
        dm.POOL_PREP = e["PCST_POOL_PREP"] != "0"
    if "PCST_ROWS_LAYOUT" in e:  # the step's kNN in the rows layout (0: the compact build)
        dm.ROWS_LAYOUT = e["PCST_ROWS_LAYOUT"] != "0"
    if "PCST_GRAPH_FORK_BUILD" in e:  # the graph step's kNN build on a forked branch (0: inline)
        dm.GRAPH_FORK_BUILD = e["PCST_GRAPH_FORK_BUILD"] != "0"
    if "PCST_KNN_BUILD_MAX_WG" in e:  # the compact build's work-groups per launch (0: natural)
        dm.KNN_BUILD_MAX_WG = int(e["PCST_KNN_BUILD_MAX_WG"])
    if "PCST_ROWS_MAX_MLP_POINTS" in e:  # the rows layout up to this many MLP points per launch
        dm.ROWS_MAX_MLP_POINTS = int(e["PCST_ROWS_MAX_MLP_POINTS"])
    if "PCST_FUSED_BLOCK_FWD" in e:
        from pointcloud_style_transfer_amd.models import _autograd
        _autograd.FUSED_BLOCK_FWD = e["PCST_FUSED_BLOCK_FWD"] != "0"
    if "PCST_FUSED_BLOCK_BWD" in e:
        from pointcloud_style_transfer_amd.models import _autograd
        _autograd.FUSED_BLOCK_BWD = e["PCST_FUSED_BLOCK_BWD"] != "0"
    if "PCST_MASK_BITS" in e:
        from pointcloud_style_transfer_amd.models import _autograd
        _autograd.MASK_BITS = e["PCST_MASK_BITS"] != "0"
    if "PCST_FUSED_BN_STATS" in e:
        from pointcloud_style_transfer_amd.models import _autograd
        _autograd.FUSED_BN_STATS = e["PCST_FUSED_BN_STATS"] != "0"
    if "PCST_BATCH_CAST" in e:
        from pointcloud_style_transfer_amd.models import _autograd
        _autograd.BATCH_CAST = e["PCST_BATCH_CAST"] != "0"
