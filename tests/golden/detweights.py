"""Closed-form deterministic weights for the golden fixtures.

The reference model (2,549,827 parameters) is far too large to commit, so the
fixture generator and the tests both fill every state_dict entry from numpy
PCG64 keyed by (seed, position in state_dict order).  The reference's
state_dict order (`models/diffusion_model.py:156-163`, `pointnet2_encoder.py:61-121`)
is reproduced by our module tree, so the same function yields the same weights
on both sides.
"""
from __future__ import annotations

import numpy as np


def deterministic_state(named_shapes, seed: int = 1234):
    """named_shapes: iterable of (name, shape tuple). Returns {name: np.ndarray}."""
    out = {}
    for i, (name, shape) in enumerate(named_shapes):
        rng = np.random.Generator(np.random.PCG64([seed, i]))
        shape = tuple(shape)
        if name.endswith("num_batches_tracked"):
            out[name] = np.zeros(shape, dtype=np.int64)
            continue
        if name.endswith("running_mean"):
            v = rng.uniform(-0.2, 0.2, shape)
        elif name.endswith("running_var"):
            v = rng.uniform(0.5, 1.5, shape)
        elif "mlp_bns" in name and name.endswith("weight"):
            v = rng.uniform(0.8, 1.2, shape)
        elif "mlp_bns" in name and name.endswith("bias"):
            v = rng.uniform(-0.1, 0.1, shape)
        elif name.endswith("bias"):
            v = rng.uniform(-0.05, 0.05, shape)
        else:
            fan_in = int(np.prod(shape[1:])) if len(shape) > 1 else 1
            bound = 1.0 / np.sqrt(fan_in)
            v = rng.uniform(-bound, bound, shape)
        out[name] = v.astype(np.float32)
    return out


def load_into(module, seed: int = 1234):
    """Fill a torch module's state_dict in place (works for reference and ours)."""
    import torch

    sd = module.state_dict()
    vals = deterministic_state([(k, tuple(v.shape)) for k, v in sd.items()], seed)
    module.load_state_dict({k: torch.from_numpy(v) for k, v in vals.items()})
    return module
