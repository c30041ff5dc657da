"""`HierarchicalPointCloudDataset` / `create_dataloaders` (data/dataset.py:10-176): the
`*_hierarchical.pt` training files written by PointCloudPreprocessor.save_hierarchical_data.

Same keys, dtypes, default items and collate as the reference.  Differences, by design:
  * files load with `torch.load(weights_only=True)` and an allowlist of the numpy types the
    format holds (arrays, dtypes, scalars), never a full unpickler;
  * under torch.distributed the train loader takes a DistributedSampler, so every rank of the
    DDP trainer reads its own shard of the files;
  * pin_memory only when a HIP device is present.
"""
from __future__ import annotations

import glob
import os
from typing import Dict, Tuple

import numpy as np
import torch
import torch.distributed as dist
from torch.utils.data import DataLoader, Dataset
from torch.utils.data.distributed import DistributedSampler


def _numpy_safe_globals():
    import numpy.dtypes as ndt

    try:
        from numpy._core.multiarray import _reconstruct, scalar
    except ImportError:  # numpy < 2
        from numpy.core.multiarray import _reconstruct, scalar
    kinds = [getattr(ndt, n) for n in dir(ndt) if n.endswith("DType")]
    return [_reconstruct, scalar, np.ndarray, np.dtype] + kinds


def load_hierarchical_file(path: str) -> dict:
    """One `*_hierarchical.pt` dict, loaded without executing code from the file."""
    with torch.serialization.safe_globals(_numpy_safe_globals()):
        return torch.load(path, weights_only=True)


class HierarchicalPointCloudDataset(Dataset):
    """data/dataset.py:10-101."""

    def __init__(self, processed_dir: str, use_hierarchical: bool = True):
        self.processed_dir = processed_dir
        self.use_hierarchical = use_hierarchical
        self.file_paths = sorted(glob.glob(os.path.join(processed_dir, "*_hierarchical.pt")))
        if not self.file_paths:
            raise FileNotFoundError(
                f"No hierarchical data files ('*_hierarchical.pt') found in {processed_dir}. "
                "Please run the preprocess_data.py script first.")

    def __len__(self):
        return len(self.file_paths)

    def __getitem__(self, idx) -> Dict[str, torch.Tensor]:
        path = self.file_paths[idx]
        try:
            data = load_hierarchical_file(path)
            required = ["sim_full", "real_full"]
            if self.use_hierarchical:
                required += ["sim_global", "sim_global_indices", "sim_norm_params",
                             "real_global", "real_global_indices", "real_norm_params"]
            missing = [k for k in required if k not in data]
            if missing:
                raise KeyError(f"Missing keys in {path}: {missing}")
            out = {"sim_full": torch.from_numpy(np.asarray(data["sim_full"])).float(),
                   "real_full": torch.from_numpy(np.asarray(data["real_full"])).float()}
            if self.use_hierarchical:
                out.update({
                    "sim_global": torch.from_numpy(np.asarray(data["sim_global"])).float(),
                    "real_global": torch.from_numpy(np.asarray(data["real_global"])).float(),
                    "sim_global_indices": torch.from_numpy(np.asarray(data["sim_global_indices"])).long(),
                    "real_global_indices": torch.from_numpy(np.asarray(data["real_global_indices"])).long(),
                    "sim_norm_params": data["sim_norm_params"],
                    "real_norm_params": data["real_norm_params"],
                    "total_points": data.get("total_points", 120000),
                    "global_points": data.get("global_points", 30000),
                })
            return out
        except Exception as e:  # noqa: BLE001 -- the reference substitutes a default item
            print(f"Error loading {path}: {e}")
            return (self._get_default_hierarchical_item() if self.use_hierarchical
                    else self._get_default_simple_item())

    def _get_default_simple_item(self) -> Dict[str, torch.Tensor]:
        return {"sim_full": torch.zeros(120000, 3), "real_full": torch.zeros(120000, 3)}

    def _get_default_hierarchical_item(self) -> Dict[str, torch.Tensor]:
        return {
            "sim_full": torch.zeros(120000, 3), "real_full": torch.zeros(120000, 3),
            "sim_global": torch.zeros(30000, 3), "real_global": torch.zeros(30000, 3),
            "sim_global_indices": torch.arange(30000), "real_global_indices": torch.arange(30000),
            "sim_norm_params": {"center": np.zeros(3), "scale": 1.0, "method": "isotropic"},
            "real_norm_params": {"center": np.zeros(3), "scale": 1.0, "method": "isotropic"},
            "total_points": 120000, "global_points": 30000,
        }


def _collate(use_hierarchical: bool):
    def hierarchical_collate_fn(batch):
        """data/dataset.py:136-157."""
        if not batch:
            return {}
        first = batch[0]
        keys = ["sim_full", "real_full"]
        if use_hierarchical:
            keys += ["sim_global", "real_global", "sim_global_indices", "real_global_indices"]
        out = {k: torch.stack([b[k] for b in batch]) for k in keys if k in first}
        if use_hierarchical:
            for k in ("sim_norm_params", "real_norm_params", "total_points", "global_points"):
                if k in first:
                    out[k] = [b[k] for b in batch]
        return out

    return hierarchical_collate_fn


def create_dataloaders(processed_dir: str, batch_size: int, num_workers: int,
                       use_hierarchical: bool = True) -> Tuple[DataLoader, DataLoader]:
    """data/dataset.py:104-176; train/ and val/ under processed_dir."""
    train_dir = os.path.join(processed_dir, "train")
    val_dir = os.path.join(processed_dir, "val")
    if not os.path.isdir(train_dir) or not os.path.isdir(val_dir):
        raise FileNotFoundError(f"Train/Val directories not found in {processed_dir}. "
                                "Please run preprocessing first.")
    train_ds = HierarchicalPointCloudDataset(train_dir, use_hierarchical)
    val_ds = HierarchicalPointCloudDataset(val_dir, use_hierarchical)
    collate = _collate(use_hierarchical) if use_hierarchical else None
    pin = torch.cuda.is_available()
    sampler = None
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        sampler = DistributedSampler(train_ds, shuffle=True, drop_last=True)
    train = DataLoader(train_ds, batch_size=batch_size, shuffle=sampler is None, sampler=sampler,
                       num_workers=num_workers, pin_memory=pin, drop_last=True, collate_fn=collate)
    val = DataLoader(val_ds, batch_size=batch_size, shuffle=False, num_workers=num_workers,
                     pin_memory=pin, collate_fn=collate)
    return train, val
