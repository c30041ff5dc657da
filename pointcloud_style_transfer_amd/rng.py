"""Random draws of the hot path, routed through one switchable source.

The reference draws with torch's generators at fixed call sites
(FPS start `pointnet2_encoder.py:36` on the CPU generator; `randperm` in the voxel
downsample `diffusion_model.py:101,111`; x_T `randn` `:234`; the cond-drop
`rand` `:177`; trainer `randint`/`randn_like` `trainer.py:75-76`,
`diffusion_model.py:214`).  Our code makes the same draws, in the same order,
through `source()`.  Parity tests install a `replay(...)` source that feeds back
the draws recorded from the reference, so a device run can be compared
bit-for-bit with the reference's outputs.

On the performance path the voxel downsample does not call `randperm` at all: it
draws its random subset on the device (Philox keys + sort, `csrc/voxel.hip`),
seeded from `device_seed()`.
"""
from __future__ import annotations

import contextlib
import threading

import numpy as np
import torch


class TorchRNG:
    replaying = False

    def randint(self, low, high, size, device=None):
        return torch.randint(low, high, size, dtype=torch.long, device=device)

    def randperm(self, n, device=None):
        return torch.randperm(n, device=device)

    def randn(self, shape, device=None):
        return torch.randn(shape, device=device)

    def rand(self, shape, device=None):
        return torch.rand(shape, device=device)

    def randn_like(self, x):
        return torch.randn_like(x)

    def device_seed(self):
        return int(torch.randint(0, 2**62, (1,), dtype=torch.long).item())


class ReplayRNG:
    """Returns recorded draws in call order; the kind of every draw is checked."""

    replaying = True

    def __init__(self, draws):
        self.draws = [(str(n), np.asarray(v)) for n, v in draws]
        self.pos = 0

    @classmethod
    def from_npz(cls, z, prefix):
        names = list(z[f"{prefix}_names"])
        return cls([(str(n), z[f"{prefix}_{i}"]) for i, n in enumerate(names)])

    def _next(self, kind):
        if self.pos >= len(self.draws):
            raise RuntimeError(f"replay exhausted at draw {self.pos} ({kind})")
        name, val = self.draws[self.pos]
        if name != kind:
            raise RuntimeError(f"replay: expected {kind}, recorded {name} at draw {self.pos}")
        self.pos += 1
        return val

    def randint(self, low, high, size, device=None):
        return torch.from_numpy(self._next("randint").astype(np.int64)).to(device)

    def randperm(self, n, device=None):
        v = self._next("randperm")
        if len(v) != n:
            raise RuntimeError(f"replay: randperm length {len(v)} recorded, {n} requested")
        return torch.from_numpy(v.astype(np.int64)).to(device)

    def randn(self, shape, device=None):
        return torch.from_numpy(self._next("randn").astype(np.float32)).to(device)

    def rand(self, shape, device=None):
        return torch.from_numpy(self._next("rand").astype(np.float32)).to(device)

    def randn_like(self, x):
        return torch.from_numpy(self._next("randn_like").astype(np.float32)).to(x.device)

    def device_seed(self):
        return 0

    @property
    def exhausted(self):
        return self.pos == len(self.draws)


class CounterRNG:
    """Counter-keyed draws for side-by-side runs (bench.py's "Chamfer vs ref" leg): the k-th
    draw, whatever its kind, comes from numpy PCG64 seeded with (seed, k).  Two runs that make
    their draws in the same order get the same values, and a permutation drawn for a different
    length n (a voxel count that moved by a point) still comes from the same key.  Installed
    with `replay(...)`, so the sampler takes its replay paths (host-drawn permutations)."""

    replaying = True

    def __init__(self, seed: int):
        self.seed = int(seed)
        self.k = 0

    def generator(self) -> np.random.Generator:
        g = np.random.default_rng([self.seed, self.k])
        self.k += 1
        return g

    def randint(self, low, high, size, device=None):
        return torch.from_numpy(self.generator().integers(low, high, size, dtype=np.int64)).to(device)

    def randperm(self, n, device=None):
        return torch.from_numpy(self.generator().permutation(int(n)).astype(np.int64)).to(device)

    def randn(self, shape, device=None):
        return torch.from_numpy(self.generator().standard_normal(shape, dtype=np.float32)).to(device)

    def rand(self, shape, device=None):
        return torch.from_numpy(self.generator().random(shape, dtype=np.float32)).to(device)

    def randn_like(self, x):
        return self.randn(tuple(x.shape), x.device)

    def device_seed(self):
        return 0


class GeneratorRNG(TorchRNG):
    """torch's draws from a private, seeded CPU generator (moved to the device), on the
    non-replay (device) paths: the draws of one sampling loop do not depend on what other host
    threads draw at the same time (tests of concurrent loops).  Installed with `use(...)`."""

    def __init__(self, seed: int):
        self.g = torch.Generator().manual_seed(int(seed))

    def randint(self, low, high, size, device=None):
        return torch.randint(low, high, size, dtype=torch.long, generator=self.g).to(device)

    def randperm(self, n, device=None):
        return torch.randperm(n, generator=self.g).to(device)

    def randn(self, shape, device=None):
        return torch.randn(shape, generator=self.g).to(device)

    def rand(self, shape, device=None):
        return torch.rand(shape, generator=self.g).to(device)

    def randn_like(self, x):  # x's dtype, as TorchRNG.randn_like (torch.randn_like)
        return torch.randn(tuple(x.shape), generator=self.g, dtype=x.dtype).to(x.device)

    def device_seed(self):
        return int(torch.randint(0, 2**62, (1,), dtype=torch.long, generator=self.g).item())


_default = TorchRNG()
# the installed source is per host thread (a loop in one thread never consumes another
# thread's replayed or seeded draws); threads without one use torch's global generators
_local = threading.local()


def source():
    return getattr(_local, "source", None) or _default


@contextlib.contextmanager
def use(rng):
    """Install `rng` as the calling thread's source for the duration of the block."""
    prev = getattr(_local, "source", None)
    _local.source = rng
    try:
        yield rng
    finally:
        _local.source = prev


@contextlib.contextmanager
def replay(draws_or_rng):
    """Install a replay source (recorded draws, a ReplayRNG or a CounterRNG) for this thread."""
    rng = (draws_or_rng if isinstance(draws_or_rng, (ReplayRNG, CounterRNG))
           else ReplayRNG(draws_or_rng))
    with use(rng):
        yield rng
