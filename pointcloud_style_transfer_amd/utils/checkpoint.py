"""Checkpoint I/O in the reference's format (`utils/checkpoint.py:12-151`):
ckpt_epoch_XXXX.pth / best_model.pth holding {epoch, model_state_dict,
optimizer_state_dict, config, ema_state_dict}.

The config is pickled under the reference's class path `config.config.Config`, so the
reference can read our checkpoints and we read theirs.  Loading never unpickles code:
torch.load(weights_only=True) with our Config allow-listed under that name.
"""
from __future__ import annotations

import contextlib
import glob
import os
import sys
from typing import Optional

import torch

from ..config import config as _config_mod
from ..config.config import Config
from .ema import ExponentialMovingAverage
from .logger import Logger

REF_CONFIG_PATH = "config.config.Config"


@contextlib.contextmanager
def reference_pickle_names():
    """While saving: pickle Config as `config.config.Config` (the reference's module path)."""
    added = []
    for name, mod in (("config", sys.modules[_config_mod.__name__.rsplit(".", 1)[0]]),
                      ("config.config", _config_mod)):
        if name not in sys.modules:
            sys.modules[name] = mod
            added.append(name)
    same = sys.modules.get("config.config") is _config_mod
    old = Config.__module__
    if same:
        Config.__module__ = "config.config"
    try:
        yield
    finally:
        Config.__module__ = old
        for name in added:
            sys.modules.pop(name, None)


def safe_load(path, map_location="cpu"):
    """torch.load(weights_only=True) that maps the reference's pickled Config onto ours."""
    with torch.serialization.safe_globals([(Config, REF_CONFIG_PATH), Config]):
        return torch.load(path, map_location=map_location, weights_only=True)


def save_checkpoint(state: dict, path: str):
    with reference_pickle_names():
        torch.save(state, path)


class CheckpointManager:
    def __init__(self, checkpoint_dir: str, experiment_name: str):
        self.base_dir = os.path.join(checkpoint_dir, experiment_name)
        os.makedirs(self.base_dir, exist_ok=True)
        self.logger = Logger(name="CheckpointManager", log_dir="logs", experiment_name=experiment_name)

    def save(self, model, optimizer: torch.optim.Optimizer,
             ema: Optional[ExponentialMovingAverage], epoch: int, is_best: bool = False):
        model = getattr(model, "module", model)  # unwrap DDP
        state = {"epoch": epoch, "model_state_dict": model.state_dict(),
                 "optimizer_state_dict": optimizer.state_dict(),
                 "config": model.config if hasattr(model, "config") else None}
        if ema:
            state["ema_state_dict"] = ema.state_dict()
        path = os.path.join(self.base_dir, f"ckpt_epoch_{epoch:04d}.pth")
        save_checkpoint(state, path)
        self.logger.info(f"Checkpoint saved to {path}")
        if is_best:
            save_checkpoint(state, os.path.join(self.base_dir, "best_model.pth"))

    def load(self, model, optimizer: torch.optim.Optimizer,
             ema: Optional[ExponentialMovingAverage]) -> int:
        latest = self._find_latest_checkpoint()
        if not latest:
            self.logger.info("No checkpoint found. Starting training from scratch.")
            return 0
        try:
            ck = safe_load(latest)
            missing = [k for k in ("model_state_dict", "optimizer_state_dict", "epoch") if k not in ck]
            if missing:
                self.logger.error(f"Checkpoint missing required keys: {missing}")
                return 0
            getattr(model, "module", model).load_state_dict(ck["model_state_dict"])
            try:
                optimizer.load_state_dict(ck["optimizer_state_dict"])
            except Exception as e:  # noqa: BLE001 -- reference semantics: continue
                self.logger.warning(f"Failed to load optimizer state: {e}")
            if ema and "ema_state_dict" in ck:
                try:
                    ema.load_state_dict(ck["ema_state_dict"])
                except Exception as e:  # noqa: BLE001
                    self.logger.warning(f"Failed to load EMA state: {e}")
            return ck.get("epoch", -1) + 1
        except Exception as e:  # noqa: BLE001 -- reference falls back to scratch
            self.logger.error(f"Failed to load checkpoint: {e}. Starting from scratch.")
            return 0

    def _find_latest_checkpoint(self) -> Optional[str]:
        files = glob.glob(os.path.join(self.base_dir, "ckpt_epoch_*.pth"))
        if not files:
            return None

        def ep(f):
            try:
                return int(os.path.basename(f).replace("ckpt_epoch_", "").replace(".pth", ""))
            except ValueError:
                return -1
        return max(files, key=ep)

    def get_best_model_path(self) -> Optional[str]:
        p = os.path.join(self.base_dir, "best_model.pth")
        return p if os.path.exists(p) else None
