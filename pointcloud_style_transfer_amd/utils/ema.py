"""Exponential moving average of the trainable parameters, state-compatible with the
reference (`utils/ema.py:7-151`): shadows kept as an ordered list of the requires_grad
parameters; state_dict = {'decay', 'shadow_params' (CPU tensors)}.  Updates run as device
tensor ops (torch._foreach) on the parameters' device."""
from __future__ import annotations

from typing import Iterable

import torch


class ExponentialMovingAverage:
    def __init__(self, parameters: Iterable[torch.nn.Parameter], decay: float = 0.995):
        if decay < 0.0 or decay > 1.0:
            raise ValueError("Decay must be between 0 and 1")
        self.parameters = list(parameters)
        self.decay = decay
        self.collected_params = []
        with torch.no_grad():
            self.shadow_params = [p.clone().detach() for p in self.parameters if p.requires_grad]
        self.param_names = [f"param_{i}" for i, p in enumerate(self.parameters) if p.requires_grad]

    def _trainable(self):
        return [p for p in self.parameters if p.requires_grad]

    def update(self):
        """shadow = decay * shadow + (1 - decay) * param  (ema.py:39-53)."""
        if not self.shadow_params:
            return
        with torch.no_grad():
            params = [p.data for p in self._trainable()][: len(self.shadow_params)]
            torch._foreach_mul_(self.shadow_params, self.decay)
            torch._foreach_add_(self.shadow_params, params, alpha=1 - self.decay)

    def apply_shadow(self):
        if not self.shadow_params:
            return
        with torch.no_grad():
            self.collected_params = [p.detach().clone() for p in self._trainable()]
            # p.copy_ (not p.data.copy_) bumps the parameter's version counter, so weight
            # caches keyed on it (NoisePredictor.packed) see the swap
            for p, s in zip(self._trainable(), self.shadow_params):
                p.copy_(s)

    def restore(self):
        if not self.collected_params:
            return
        with torch.no_grad():
            for p, c in zip(self._trainable(), self.collected_params):
                p.copy_(c)
        self.collected_params = []

    def state_dict(self) -> dict:
        return {"decay": self.decay,
                "shadow_params": [p.clone().detach().cpu() for p in self.shadow_params]}

    def load_state_dict(self, state_dict: dict):
        """ema.py:100-151, including the partial-load fallback on a count mismatch."""
        if "shadow_params" not in state_dict:
            raise KeyError("Invalid EMA state_dict: missing 'shadow_params'")
        self.decay = state_dict["decay"]
        loaded = state_dict["shadow_params"]
        trainable = self._trainable()
        if len(loaded) != len(trainable):
            n = min(len(loaded), len(trainable), len(self.shadow_params))
            if n > 0:
                dev = self.parameters[0].device if self.parameters else "cpu"
                for i in range(n):
                    self.shadow_params[i] = loaded[i].to(dev)
                return
            self.__init__(self.parameters, self.decay)
            return
        shadows = []
        for p, s in zip(trainable, loaded):
            s = s.to(p.device)
            shadows.append(s if s.shape == p.shape else p.clone().detach())
        self.shadow_params = shadows
