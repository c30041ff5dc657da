"""Offline hierarchical preprocessing (data/preprocessing.py:45-175,
data/dataset.py): the voxel representatives are bit-exact with the reference (golden
preprocess.npz from gen_preprocess.py); the random pad/subsample draw is checked by its
properties (the reference draws from a Python set, whose order is not reproduced); the .pt
file round-trips through the dataset loader."""
import numpy as np
import pytest

from oracle import oracle as O


@pytest.fixture(scope="module")
def G(golden):
    return golden("preprocess.npz")


def test_oracle_voxel_reps_vs_reference(G):
    assert np.array_equal(O.voxel_center_reps(G["pad_points"], 4096), G["pad_reps"])
    assert np.array_equal(O.voxel_center_reps(G["sub_points"], 4096), G["sub_reps"])


def test_dataset_roundtrip_and_collate(tmp_path):
    import torch

    from pointcloud_style_transfer_amd.data.dataset import (HierarchicalPointCloudDataset,
                                                             create_dataloaders)

    for split in ("train", "val"):
        d = tmp_path / split
        d.mkdir()
        for i in range(3):
            rng = np.random.default_rng(i)
            data = {"sim_full": rng.standard_normal((64, 3)).astype(np.float32),
                    "real_full": rng.standard_normal((64, 3)).astype(np.float32),
                    "sim_global": np.zeros((16, 3), np.float32), "real_global": np.zeros((16, 3), np.float32),
                    "sim_global_indices": np.arange(16), "real_global_indices": np.arange(16),
                    "sim_norm_params": {"center": np.zeros(3), "scale": 1.0, "method": "isotropic",
                                        "target_range": 1.8},
                    "real_norm_params": {"center": np.ones(3), "scale": np.float64(2.0), "method": "isotropic",
                                         "target_range": 1.8},
                    "total_points": 64, "global_points": 16}
            torch.save(data, d / f"{i:03d}_hierarchical.pt")
    ds = HierarchicalPointCloudDataset(str(tmp_path / "train"))
    assert len(ds) == 3
    item = ds[1]
    assert item["sim_full"].dtype == torch.float32 and item["sim_global_indices"].dtype == torch.int64
    assert np.array_equal(item["sim_full"].numpy(),
                          np.random.default_rng(1).standard_normal((64, 3)).astype(np.float32))
    assert item["real_norm_params"]["scale"] == 2.0
    tr, va = create_dataloaders(str(tmp_path), batch_size=2, num_workers=0)
    b = next(iter(tr))
    assert b["sim_full"].shape == (2, 64, 3) and len(b["sim_norm_params"]) == 2
    assert len(tr) == 1 and len(va) == 2          # drop_last on train only
    simple = HierarchicalPointCloudDataset(str(tmp_path / "val"), use_hierarchical=False)
    assert set(simple[0]) == {"sim_full", "real_full"}


def test_dataset_missing_dir(tmp_path):
    from pointcloud_style_transfer_amd.data.dataset import HierarchicalPointCloudDataset

    with pytest.raises(FileNotFoundError):
        HierarchicalPointCloudDataset(str(tmp_path))


@pytest.mark.gpu
def test_device_voxel_downsample_vs_reference(G):
    from pointcloud_style_transfer_amd.data.preprocessing import PointCloudPreprocessor

    pre = PointCloudPreprocessor(20000, 4096, rng=np.random.default_rng(0))
    for name in ("pad", "sub"):
        pts = G[f"{name}_points"]
        reps = pre.voxel_representatives(pts, 4096)
        assert np.array_equal(reps, G[f"{name}_reps"])
        out_pts, idx = pre.consistent_downsample(pts, 4096)
        assert len(idx) == 4096 and len(np.unique(idx)) == 4096
        assert np.array_equal(out_pts, pts[idx])
        if name == "pad":   # all representatives first, in order, then distinct non-representatives
            assert np.array_equal(idx[:len(reps)], reps)
        else:               # a subset of the representatives
            assert np.isin(idx, reps).all()


@pytest.mark.gpu
def test_device_consistent_upsample_vs_reference(G):
    from pointcloud_style_transfer_amd.data.preprocessing import PointCloudPreprocessor

    pre = PointCloudPreprocessor(20000, 4096)
    out = pre.consistent_upsample(G["up_coarse"], G["pad_points"], G["pad_idx"])
    assert np.array_equal(out, G["up_result"])


@pytest.mark.gpu
def test_save_hierarchical_file_loads(tmp_path):
    from pointcloud_style_transfer_amd.data.dataset import HierarchicalPointCloudDataset
    from pointcloud_style_transfer_amd.data.preprocessing import PointCloudPreprocessor

    rng = np.random.default_rng(3)
    pre = PointCloudPreprocessor(8000, 2048, rng=rng)
    sim = (rng.standard_normal((9000, 3)) * [5, 5, 1]).astype(np.float32)   # voxel resample
    real = (rng.standard_normal((7000, 3)) * [5, 5, 1]).astype(np.float32)  # choice resample
    pre.save_hierarchical_data(sim, real, str(tmp_path), "s0")
    item = HierarchicalPointCloudDataset(str(tmp_path))[0]
    assert item["sim_full"].shape == (8000, 3) and item["real_global"].shape == (2048, 3)
    assert np.abs(item["sim_full"].numpy()).max() == pytest.approx(1.8, rel=1e-6)
    assert np.array_equal(item["sim_global"].numpy(),
                          item["sim_full"].numpy()[item["sim_global_indices"].numpy()])
