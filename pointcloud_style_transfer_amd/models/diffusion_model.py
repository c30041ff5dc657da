"""Diffusion model of the style-transfer hot path on the MI355X kernels -- drop-in for the
reference's `models/diffusion_model.py` (same classes, constructor arguments, parameter
names/shapes, forward signatures and sampler loops).

  TimeEmbedding / NoisePredictor      -> csrc/noise_mlp.hip (one fused MFMA launch + cond)
  HierarchicalProcessor.downsample    -> csrc/voxel.hip     (device voxel hash, no host sync)
  HierarchicalProcessor.upsample_knn  -> csrc/knn.hip       (device float64 kNN-3, no D2H/H2D)
  guided_sample_loop / ddim update    -> csrc/sampler.hip   (fused CFG + DDIM)
  StyleEncoder                        -> models/pointnet2_encoder.py kernels + pointwise linear

Keyword-only additions (defaults unchanged): `x_T=` on the sampler loops (inject the
initial noise).  Random draws go through `rng.source()` so parity runs can replay the
reference's draws; on the perf path the voxel subset is drawn on the device.
"""
from __future__ import annotations

import contextlib
import math
import threading
from typing import Optional, Tuple

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import _hip
from .. import packing
from .. import rng as _rng
from ..config.config import Config
from . import _autograd as _ag
from .pointnet2_encoder import PointNet2Encoder


class TimeEmbedding(nn.Module):
    """`TimeEmbedding` (diffusion_model.py:15-26).  Inside NoisePredictor the embedding is
    computed by pcst_noise_cond; this standalone forward exists for API parity."""

    def __init__(self, dim: int):
        super().__init__()
        self.dim = dim

    def freqs(self, device) -> torch.Tensor:
        # kept per device: a pageable host->device copy synchronises the stream (every training
        # step would wait for the work queued before it); not a buffer, so the state_dict stays
        # the reference's
        cache = self.__dict__.setdefault("_freqs", {})
        key = str(torch.device(device))
        if key not in cache:
            cache[key] = packing.time_freqs(self.dim).to(device)
        return cache[key]

    def forward(self, t: torch.Tensor) -> torch.Tensor:
        _hip.require_device(t)
        e = t[:, None].float() * self.freqs(t.device)[None, :]
        return torch.cat((e.sin(), e.cos()), dim=-1)


def _linear(x: torch.Tensor, lin: nn.Linear, relu: bool) -> torch.Tensor:
    """nn.Linear (+ReLU) on the pointwise MFMA kernel (x [rows, in])."""
    return _hip.pointwise_linear(x, lin.weight.detach(), None, lin.bias.detach(), relu, 0)


class StyleEncoder(nn.Module):
    """`StyleEncoder` (diffusion_model.py:28-36): PointNet++ encoder + style MLP."""

    def __init__(self, feature_dim: int = 256):
        super().__init__()
        self.encoder = PointNet2Encoder(input_channels=3, feature_dim=feature_dim)
        self.style_mlp = nn.Sequential(nn.Linear(feature_dim, 512), nn.ReLU(), nn.Dropout(0.1),
                                       nn.Linear(512, feature_dim), nn.ReLU())

    def forward(self, points: torch.Tensor, geometry: Optional[list] = None) -> torch.Tensor:
        f = self.encoder(points, geometry)
        if _ag.needs_grad(self):
            h = _ag.linear(f, self.style_mlp[0], True)
            h = self.style_mlp[2](h)
            return _ag.linear(h, self.style_mlp[3], True)
        h = _linear(f, self.style_mlp[0], True)
        if self.training and self.style_mlp[2].p > 0:
            h = F.dropout(h, self.style_mlp[2].p, True)
        return _linear(h, self.style_mlp[3], True)


class NoisePredictor(nn.Module):
    """`NoisePredictor` (diffusion_model.py:38-61); forward = pcst_noise_cond + pcst_noise_mlp."""

    def __init__(self, config: Config):
        super().__init__()
        if config.feature_dim != 256 or config.time_embed_dim != 128:
            raise NotImplementedError("the fused MI355X noise MLP is built for feature_dim=256, "
                                      "time_embed_dim=128 (the reference Config defaults)")
        self.config = config
        fd = config.feature_dim
        self.point_encoder = nn.Sequential(nn.Linear(3, 128), nn.ReLU(), nn.Linear(128, 256),
                                           nn.ReLU(), nn.Linear(256, fd))
        self.time_embedding = TimeEmbedding(config.time_embed_dim)
        self.time_proj = nn.Linear(config.time_embed_dim, fd)
        self.style_proj = nn.Linear(fd, fd)
        self.layers = nn.ModuleList([
            nn.Sequential(nn.Linear(fd, fd * 2), nn.ReLU(), nn.Linear(fd * 2, fd), nn.Dropout(0.1))
            for _ in range(6)])
        self.output_mlp = nn.Sequential(nn.Linear(fd, 256), nn.ReLU(), nn.Linear(256, 128),
                                        nn.ReLU(), nn.Linear(128, 3))
        self._pack_key = None
        self._packed = None

    @property
    def precision_code(self) -> int:
        """ABI precision code: "bf16" runs the bf16 (solo) kernel, "fp32" the exact-f32 parity
        kernel."""
        p = getattr(self.config, "precision", "fp32")
        return packing.BF16 if p == "bf16" else packing.F32

    def packed(self):
        """Packed MFMA weight stream + bias table, rebuilt when any weight changes."""
        params = list(self.parameters())
        dev = params[0].device
        key = (self.precision_code, str(dev), tuple((p.data_ptr(), p._version) for p in params))
        if key != self._pack_key:
            sd = {f"noise_predictor.{k}": v.detach().float().cpu().numpy()
                  for k, v in self.state_dict().items()}
            blob = torch.from_numpy(packing.pack_blob(sd, self.precision_code)).to(dev)
            bias = torch.from_numpy(packing.pack_bias(sd)).to(dev)
            freqs = self.time_embedding.freqs(dev)
            wt_t = self.time_proj.weight.detach().float().t().contiguous()
            ws_t = self.style_proj.weight.detach().float().t().contiguous()
            self._packed = (blob, bias, freqs, wt_t, ws_t)
            self._pack_key = key
        return self._packed

    def cond(self, timestep: torch.Tensor, style_feat: torch.Tensor,
             packed: Optional[tuple] = None) -> torch.Tensor:
        _, _, freqs, wt_t, ws_t = packed if packed is not None else self.packed()
        return _hip.noise_cond(timestep, style_feat, freqs, wt_t, self.time_proj.bias.detach(),
                               ws_t, self.style_proj.bias.detach(),
                               self.point_encoder[4].bias.detach())

    def _fused_params(self):
        """Weights in NoisePredictorFn's order: point encoder, 6 x (Linear1, Linear2), output."""
        mods = [self.point_encoder[0], self.point_encoder[2], self.point_encoder[4]]
        for layer in self.layers:
            mods += [layer[0], layer[2]]
        mods += [self.output_mlp[0], self.output_mlp[2], self.output_mlp[4]]
        out = []
        for m in mods:
            out += [m.weight, m.bias]
        return out

    def _dropout_active(self) -> bool:
        return self.training and any(l[3].p > 0 for l in self.layers)

    def _forward_autograd(self, noisy_points, timestep, style_feat):
        """Differentiable path (training): every linear on the MFMA GEMM kernel with its
        backward (models/_autograd.py); residual adds / dropout as device tensor ops."""
        pe = self.point_encoder
        tf = _ag.linear(self.time_embedding(timestep.to(noisy_points.device)), self.time_proj)
        sf = _ag.linear(style_feat, self.style_proj)
        if noisy_points.is_cuda and torch.is_autocast_enabled("cuda"):
            # the whole per-point network on the 16-bit-storage fused GEMMs (NoisePredictorFn,
            # autocast's dtype);
            # each residual block keeps its own Dropout rate
            ps = tuple(float(l[3].p) if self.training else 0.0 for l in self.layers)
            cond = torch.stack([tf.float(), sf.float()], 1)
            return _ag.NoisePredictorFn.apply(noisy_points.float(), cond, ps,
                                              *self._fused_params())
        h = _ag.linear(noisy_points, pe[0], True)
        h = _ag.linear(h, pe[2], True)
        pf = _ag.linear(h, pe[4])
        x = pf + tf.unsqueeze(1) + sf.unsqueeze(1)
        for layer in self.layers:
            d = _ag.linear(_ag.linear(x, layer[0], True), layer[2])
            x = layer[3](d) + x
        h = _ag.linear(x, self.output_mlp[0], True)
        h = _ag.linear(h, self.output_mlp[2], True)
        return _ag.linear(h, self.output_mlp[4])

    def fused_inference(self, style_feat: torch.Tensor) -> bool:
        """True when forward() runs the fused inference kernel (no autograd, no dropout)."""
        return not (_ag.needs_grad(self) or self._dropout_active()
                    or (style_feat.requires_grad and torch.is_grad_enabled()))

    def forward_cond(self, noisy_points: torch.Tensor, cond: torch.Tensor,
                     packed: Optional[tuple] = None, wait=None, signal=None) -> torch.Tensor:
        """The fused inference forward with precomputed conditioning rows (`cond()` of the
        same timesteps and style features): the sampling loops compute every step's rows in one
        launch before the loop.  `packed` (this module's `packed()`, fetched once before a loop
        that does not change the weights) skips the per-call weight-version check.  `wait` (a
        DeviceSignal): later work on this stream also waits for it; `signal` (a DeviceSignal's
        next_value()): published as the launch begins (_hip.noise_mlp)."""
        B, N, _ = noisy_points.shape
        blob, bias = (packed if packed is not None else self.packed())[:2]
        out = _hip.noise_mlp(noisy_points.reshape(B * N, 3), N, cond, blob, bias,
                             self.precision_code, wait=wait, signal=signal)
        return out.view(B, N, 3)

    def forward(self, noisy_points: torch.Tensor, timestep: torch.Tensor,
                style_feat: torch.Tensor) -> torch.Tensor:
        if not self.fused_inference(style_feat):
            return self._forward_autograd(noisy_points, timestep, style_feat)
        cond = self.cond(timestep.to(noisy_points.device), style_feat)
        return self.forward_cond(noisy_points, cond)


class HierarchicalProcessor:
    """`HierarchicalProcessor` (diffusion_model.py:64-153) on the device."""

    def __init__(self, total_points: int = 120000, global_points: int = 30000):
        self.total_points = total_points
        self.global_points = global_points

    def _voxel_grid_downsample_torch(self, points: torch.Tensor,
                                     target_size: int) -> Tuple[torch.Tensor, torch.Tensor]:
        if points.shape[1] <= target_size:
            idx = torch.arange(points.shape[1], device=points.device)
            return points, idx.expand(points.shape[0], -1)
        src = _rng.source()
        if src.replaying:
            return _hip.voxel_downsample(points, target_size,
                                         perm_provider=lambda b, n: src.randperm(n, points.device))
        return _hip.voxel_downsample(points, target_size, seed=src.device_seed())

    def downsample(self, points: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        return self._voxel_grid_downsample_torch(points, self.global_points)

    def downsample_copies(self, points: torch.Tensor, copies: int,
                          ws: Optional[torch.Tensor] = None,
                          prepped: bool = False, seed: Optional[int] = None,
                          pool: bool = False, start=None, rows=None,
                          rows_wait=None) -> Tuple[torch.Tensor, torch.Tensor]:
        """downsample(torch.cat([points] * copies)) -- the CFG batch of guided_sample_loop
        (diffusion_model.py:244-247) -- without building or re-hashing the copies.  Replay runs
        take the concatenated path: the reference draws one permutation per row.  `ws`
        (_hip.voxel_copies_workspace of the same shape) is reused instead of allocated;
        prepped: `ws` was prepared for `points` by the previous step's update
        (_hip.cfg_ddim_voxel_prep).  seed: the subset seed drawn ahead by the loop (the one the
        previous step's update made the pool histogram for: pool=True); None draws it here.
        start (prepped only): a signal value the launch publishes as it begins (knn_rows_begin).
        rows / rows_wait: the step's kNN rows handle and its refs signal -- the downsample's emit
        places the coarse refs itself (phase B; the device-drawn path only: a replayed or
        concatenated downsample leaves rows.placed False)."""
        src = _rng.source()
        if points.shape[1] <= self.global_points or src.replaying:
            return self.downsample(torch.cat([points] * copies))
        return _hip.voxel_downsample(points, self.global_points,
                                     seed=src.device_seed() if seed is None else seed,
                                     copies=copies, ws=ws, prepped=prepped, pool=pool, start=start,
                                     rows=rows, rows_wait=rows_wait)

    def step_prep(self, points: torch.Tensor) -> bool:
        """Whether the next downsample_copies of `points` can take a workspace prepared by the
        step's update (the device-drawn path; replay runs concatenate)."""
        return points.shape[1] > self.global_points and not _rng.source().replaying

    def upsample_knn(self, coarse_points: torch.Tensor, original_points: torch.Tensor,
                     coarse_indices: torch.Tensor) -> torch.Tensor:
        return _hip.knn3_interp(coarse_points, original_points, coarse_indices)


# The sampling step's stream layout.  The kNN upsample's build (grid, counts,
# sort: positions only) does not depend on the noise MLP's output, so it runs on a side stream:
#   - rows layout (one MLP round of work-groups, <= ROWS_MAX_MLP_POINTS: one cloud): the side
#     stream bins every point of x (phase A) while the loop stream runs the voxel downsample,
#     whose emit launch places the coarse refs (phase B) once phase A's refs flag is up, and the
#     MLP launch's last work-group waits for phase A's end, so the query's work-groups only check
#     the flag;
#   - compact layout (many MLP rounds: 32 clouds per GPU): the whole build beside the MLP, its
#     work-groups held to an LDS floor of KNN_BUILD_LDS_FLOOR bytes while the MLP needs at most
#     two rounds of work-groups (so they only take the CUs the MLP's last round leaves idle), and
#     unpadded beyond (they take CUs as MLP work-groups retire: 8.78 -> 8.31 ms per 32-cloud step
#     against the build inline, tools/b32_probe.py).
# Cross-stream dependencies are device flags (_hip.DeviceSignal): an event that another queue
# waits on stalls the recording queue ~17 us, a flag ~3 us (tools/sync_probe.hip); the loop ->
# side flag is published by the launch that needs its input final (the voxel insert's or the MLP's
# start signal), so no signal launch sits on the loop queue.  Results are bit-identical to the
# single-stream loop.  Module constants: the design's fixed choices; tools/knobs.py overrides
# them for A/B runs only.
OVERLAP_KNN_BUILD = True
_OVERLAP_MAX_MLP_POINTS = 2 * 128 * 256
# LDS floor of the compact build's work-groups (pcst_knn3_build's lds_floor): above what an MLP
# work-group leaves free on its CU, so the build never co-resides with the MLP, and 16 KiB rather
# than the smallest such floor (8 KiB): 2718 / 2722 / 2733 / 2706 vs 2685 / 2709 / 2717 / 2693
# steps/s in four alternating pairs over two boxes (profiles/r04/a56, a57).
KNN_BUILD_LDS_FLOOR = 16384
# Work-groups per launch of the compact build beside the MLP (pcst_knn3_build's max_wg; 0: the
# natural grids).  Beside a many-round MLP (32 clouds: 7500 work-groups) every build work-group
# that takes a slot as MLP work-groups retire holds it through its memory waits; 256 work-groups
# that each stride over more of the build take fewer slots: 32-cloud step 7.17-7.28 vs 7.38-7.53 ms
# (four pairs, profiles/r06/r6mw, r6mw2).  tools/knobs.py overrides it for A/B runs.
KNN_BUILD_MAX_WG = 256
# The hipGraph step (guided_sample_loop(graph=True)): the compact kNN build on a forked branch of
# the captured graph beside the MLP, capped as above, instead of inline before it.
GRAPH_FORK_BUILD = True


def overlap_knn_build(mlp_points: int) -> bool:
    return OVERLAP_KNN_BUILD


def knn_build_lds_floor(mlp_points: int) -> int:
    """The side-stream build's LDS floor for an MLP launch over `mlp_points` points."""
    return KNN_BUILD_LDS_FLOOR if mlp_points <= _OVERLAP_MAX_MLP_POINTS else 0


_THREAD_STREAMS = threading.local()


def step_streams(device) -> Tuple[torch.cuda.Stream, torch.cuda.Stream]:
    """(high-priority loop stream, default-priority side stream) of the calling host thread on a
    device, created once per thread (pcst_stream_create).  Two sampling loops running at the same
    time from two threads never share a queue: their flag waits, interleaved on one queue, could
    wait on each other."""
    idx = torch.device(device).index
    idx = torch.cuda.current_device() if idx is None else idx
    per_dev = getattr(_THREAD_STREAMS, "by_device", None)
    if per_dev is None:
        per_dev = _THREAD_STREAMS.by_device = {}
    if idx not in per_dev:
        per_dev[idx] = (_hip.DeviceStream(idx, priority=-1), _hip.DeviceStream(idx, priority=0))
    loop, side = per_dev[idx]
    return loop.stream, side.stream


# At most one overlapped loop per device at a time.  HIP maps streams onto at most
# GPU_MAX_HW_QUEUES hardware queues per priority (4 on the MI355X boxes), so per-thread stream
# pairs do not keep concurrent loops apart: with more loops than queues, one loop's in-queue flag
# wait can sit ahead of the other loop's producer on a shared queue -- a cycle that only the poll
# bound breaks (a SignalTimeout).  A loop that finds the device's overlapped slot taken runs the
# single-stream layout (no cross-stream waits; the same bits).
_OVERLAP_LOCKS = {}
_OVERLAP_LOCKS_GUARD = threading.Lock()


def overlap_slot(device):
    """The device's overlapped-loop lock (acquire non-blocking; release when the loop ends)."""
    idx = torch.device(device).index
    idx = torch.cuda.current_device() if idx is None else idx
    with _OVERLAP_LOCKS_GUARD:
        return _OVERLAP_LOCKS.setdefault(idx, threading.Lock())


# Poll bound of the step's device waits (0: the library's default, ~10 s).  Tests lower it.
SIGNAL_MAX_POLLS = 0


class StepState:
    """The overlapped step's streams and cross-stream dependencies for ONE sampling loop (or one
    bench run): the calling thread's loop / side streams and three device flags (0: loop -> side,
    the step's input is final -- compact layout: the voxel output, rows layout: x; 1: side ->
    loop, compact layout: the kNN build is done, rows layout: phase B may run; 2: rows layout,
    phase A is done).  The flags share one allocation, so `check()` reads every timeout word with
    one copy; it raises _hip.SignalTimeout when a wait gave up (the loop's results are then
    invalid).  Per loop, so concurrent loops never share a flag and a flag's host counter starts
    at zero every loop."""

    def __init__(self, device, max_polls=None):
        self.loop, self.side = step_streams(device)
        polls = SIGNAL_MAX_POLLS if max_polls is None else max_polls
        self._flags = torch.zeros(3, 4, dtype=torch.int32, device=device)
        self.ready_sig = _hip.DeviceSignal(device, polls, self._flags[0])
        self.built_sig = _hip.DeviceSignal(device, polls, self._flags[1])
        self.done_sig = _hip.DeviceSignal(device, polls, self._flags[2])

    def begin(self, caller):
        """Order both streams after the caller's work so far (the flags' zero fill included)."""
        self.loop.wait_stream(caller)
        self.side.wait_stream(caller)

    def end(self, caller):
        """Order the caller after every loop- and side-stream kernel (also on an exception: the
        tensors the caller frees must not be reused while they run)."""
        caller.wait_stream(self.loop)
        caller.wait_stream(self.side)

    def check(self):
        """After end(): raise if any of the step's device waits timed out."""
        if bool(self._flags[:, 1].cpu().any()):
            raise _hip.SignalTimeout(
                "pcst: a cross-stream device wait of the sampling step timed out (the kNN build or "
                "the voxel output it waited for never signalled); the loop's output is invalid")


# The step's kNN in the rows layout (pcst_knn3_rows_*) while the MLP is one round of work-groups
# (<= ROWS_MAX_MLP_POINTS): with the one-round bf16 MLP (235 work-groups of 512 threads and every
# VGPR of their CUs) nothing beside it finds a CU, so the compact build could only run after it
# (round 5: ~75 us on the step's critical path); here its positions-only part overlaps the
# latency-bound voxel chain instead.  Bit-identical to the compact layout
# (tests/test_gpu_knn_rows.py).  With many MLP rounds (32 clouds per GPU) the compact build still
# hides under the MLP and the rows layout's query, which visits every point (34 % more chunks),
# loses (b1 2706 vs 2614 steps/s, b32 8.26 vs 7.61 ms, profiles/r05/r5c).  tools/knobs.py may
# turn it off for A/B runs.
ROWS_LAYOUT = True
ROWS_MAX_MLP_POINTS = 256 * 256


def rows_layout_ok(mlp_points: int) -> bool:
    return ROWS_LAYOUT and mlp_points <= ROWS_MAX_MLP_POINTS


def knn_rows_begin(x, M, state, ws, by_downsample=False):
    """Phase A of the step's kNN on the side stream, ordered after the loop stream's work so far
    (x is ready): -> (the rows handle for hierarchical_eps(rows=...), start).  by_downsample: the
    next launch on the loop stream, the prepared voxel downsample, publishes the loop -> side flag
    as it begins (pass `start` to downsample_copies) instead of a signal launch here; else start is
    None.  The side stream signals state.built_sig once phase B may run and state.done_sig when
    phase A is done."""
    start = None
    if by_downsample:
        start = state.ready_sig.next_value()
    else:
        state.ready_sig.signal(torch.cuda.current_stream())
    state.ready_sig.wait(state.side)
    with torch.cuda.stream(state.side):
        h = _hip.knn3_rows_build(x, M, 2, ws, refs_sig=state.built_sig, done_sig=state.done_sig)
    return h, start


def hierarchical_eps(hp, mlp, xc, xi, x_cat, knn_ws=None, state=None, fused=False, rows=None):
    """eps for the CFG batch: mlp(xc) on the current stream, upsampled to the full clouds by
    kNN-3 (HierarchicalProcessor.upsample_knn).  With a StepState (and a preallocated
    workspace) the kNN build runs on its side stream (the layouts above).  fused: `mlp` is the
    fused-conditioning MLP, which takes wait= (its last work-group waits for a DeviceSignal) and
    start= (its launch publishes a DeviceSignal value as it begins).  rows: the knn_rows_begin
    handle of this step (the rows layout)."""
    if state is None:
        return hp.upsample_knn(mlp(xc), x_cat, xi)
    main = torch.cuda.current_stream()
    if rows is not None:  # the rows layout: phase A ran beside the downsample (knn_rows_begin)
        if not rows.placed:  # (the device-drawn downsample's emit placed the refs itself)
            _hip.knn3_rows_refs(rows, xi, wait=state.built_sig)  # (waits for phase A in-kernel)
        if fused:  # the MLP's last work-group waits for phase A's end; the query only checks it
            return _hip.knn3_rows_query(mlp(xc, wait=state.done_sig), rows, state.done_sig,
                                        waited=True)
        # else one wait launch (one work-group polls) before the query, never the query's own
        # work-groups: at 4 per CU they hold every VGPR of the device, and phase A's last launches
        # could then find no CU ("Forward progress")
        nc = mlp(xc)
        state.done_sig.wait(main)
        return _hip.knn3_rows_query(nc, rows, state.done_sig, waited=True)
    ready, built = state.ready_sig, state.built_sig
    start = None
    if fused:
        start = ready.next_value()  # written by the MLP launch as it begins (pcst_noise_mlp_ex)
    else:
        ready.signal(main)
    ready.wait(state.side)
    with torch.cuda.stream(state.side):
        handle = _hip.knn3_build(x_cat, xi, knn_ws, knn_build_lds_floor(xc.shape[0] * xc.shape[1]),
                                 KNN_BUILD_MAX_WG)
        built.signal(state.side)
    nc = mlp(xc, start=start) if fused else mlp(xc)
    built.wait(main)
    return _hip.knn3_query(nc, handle, built)


def pool_prep_ok(x) -> bool:
    """Whether a prepared update also makes the next downsample's pool histogram (POOL_PREP;
    the prep kernel's histogram holds the 1024 bins of clouds up to 4M points)."""
    return POOL_PREP and x.shape[1] <= (4 << 20)


def voxel_prep_ok(hp, x, state) -> bool:
    """Whether hierarchical_step's update prepares the next downsample_copies of x (VOXEL_PREP)."""
    return VOXEL_PREP and hp.step_prep(x)


def hierarchical_step(hp, mlp, xc, xi, x_cat, x, source, guidance_scale, coeffs, knn_ws=None,
                      state=None, fused=False, vox_ws=None, pool_seed=None, rows=None):
    """One guided step of the hierarchical branch (diffusion_model.py:240-260): eps of the CFG
    batch (mlp(xc) upsampled by kNN-3), then the fused CFG + DDIM update of x (x_cat takes the
    new x twice).  Returns the new x.  state: a StepState (overlapped layout) or None.
    vox_ws: the voxel workspace of the next step's downsample_copies, prepared by this update
    (_hip.cfg_ddim_voxel_prep: one launch fewer); that call must then pass prepped=True.
    pool_seed (with vox_ws): the seed of that downsample, drawn ahead; the update also makes its
    pool-key histogram (POOL_PREP), and the downsample must then pass seed=pool_seed, pool=True.
    rows: the knn_rows_begin handle of this step (the rows layout)."""
    C = x.shape[0]
    eps = hierarchical_eps(hp, mlp, xc, xi, x_cat, knn_ws, state, fused, rows)
    if vox_ws is not None:
        return _hip.cfg_ddim_voxel_prep(x, eps, source, guidance_scale, coeffs, x_cat, vox_ws,
                                        pool_seed=pool_seed)
    return _hip.cfg_ddim_step(x, eps[:C], eps[C:], source, guidance_scale, coeffs, x_cat=x_cat)


# The step's CFG + DDIM update also prepares the next step's voxel downsample (its statistics and
# zeroing: pcst_cfg_ddim_voxel_prep), one launch fewer per step; bit-identical.
VOXEL_PREP = True
# The update also makes the next downsample's pool-key histogram (its keys depend on the subset
# seed, the row and the point index only), so the voxel insert on the step's critical path skips
# it; the loop draws each step's subset seed one step ahead (one draw per step either way, in the
# same order: the draws, hence the results, are unchanged).  POOL_PREP needs VOXEL_PREP.
POOL_PREP = True


class PointCloudDiffusionModel(nn.Module):
    """`PointCloudDiffusionModel` (diffusion_model.py:156-190)."""

    def __init__(self, config: Config):
        super().__init__()
        self.config = config
        self.style_encoder = StyleEncoder(feature_dim=config.feature_dim)
        self.noise_predictor = NoisePredictor(config)
        self.hierarchical_processor = HierarchicalProcessor(total_points=config.total_points,
                                                            global_points=config.global_points)

    def style_geometry(self, condition_points: torch.Tensor, use_hierarchical: bool = True):
        """The positions-only part of the style branch of forward(): the condition cloud's
        downsample and the encoder's FPS / ball-query indices, in forward()'s draw order.
        Passing it back as forward(style_geometry=...) skips recomputing it."""
        if use_hierarchical and condition_points.shape[1] > self.config.global_points:
            xyz = self.hierarchical_processor.downsample(condition_points)[0]
        else:
            xyz = condition_points
        return xyz, self.style_encoder.encoder.geometry(xyz)

    def forward(self, noisy_points: torch.Tensor, timestep: torch.Tensor,
                condition_points: torch.Tensor, cond_drop_prob: float = 0.0,
                use_hierarchical: bool = True,
                style_geometry: Optional[tuple] = None) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
        hp = self.hierarchical_processor
        if style_geometry is not None:  # style_geometry(condition_points, use_hierarchical)
            style_feat = self.style_encoder(*style_geometry)
        elif use_hierarchical and condition_points.shape[1] > self.config.global_points:
            style_feat = self.style_encoder(hp.downsample(condition_points)[0])
        else:
            style_feat = self.style_encoder(condition_points)
        if cond_drop_prob > 0:
            mask = _rng.source().rand((style_feat.shape[0], 1), style_feat.device) > cond_drop_prob
            style_feat = style_feat * mask
        if use_hierarchical and noisy_points.shape[1] > self.config.global_points:
            noisy_down, idx = hp.downsample(noisy_points)
            return self.noise_predictor(noisy_down, timestep, style_feat), idx
        return self.noise_predictor(noisy_points, timestep, style_feat), None


class DiffusionProcess:
    """`DiffusionProcess` (diffusion_model.py:193-293)."""

    def __init__(self, config: Config, device: str = "cuda"):
        self.num_timesteps = config.num_timesteps
        self.device = device
        # tables evaluated with the reference's own torch CPU ops (bit-exact), then moved
        self._cpu_device = "cpu"
        betas = self._get_beta_schedule(config.beta_schedule, config.noise_schedule_offset)
        alphas = 1.0 - betas
        ac = torch.cumprod(alphas, axis=0)
        self._ac_host = ac.numpy().astype(np.float32)
        self.betas = betas.to(device)
        self.alphas = alphas.to(device)
        self.alphas_cumprod = ac.to(device)
        self.alphas_cumprod_prev = F.pad(ac[:-1], (1, 0), value=1.0).to(device)
        self.sqrt_alphas_cumprod = torch.sqrt(ac).to(device)
        self.sqrt_one_minus_alphas_cumprod = torch.sqrt(1.0 - ac).to(device)

    def _get_beta_schedule(self, schedule_name: str, offset: float = 0.0) -> torch.Tensor:
        """`_get_beta_schedule` (diffusion_model.py:204-211), on the CPU."""
        if schedule_name == "cosine":
            steps = self.num_timesteps + 1
            x = torch.linspace(0, self.num_timesteps, steps)
            ac = torch.cos(((x / self.num_timesteps) + 0.008 + offset) / 1.008 * torch.pi * 0.5) ** 2
            ac = ac / ac[0]
            betas = 1 - (ac[1:] / ac[:-1])
            return torch.clip(betas, 0.0001, 0.9999)
        if schedule_name == "linear":
            return torch.linspace(0.0001, 0.02, self.num_timesteps)
        raise NotImplementedError(f"unknown beta schedule: {schedule_name}")

    def q_sample(self, x_start: torch.Tensor, t: torch.Tensor,
                 noise: torch.Tensor = None) -> Tuple[torch.Tensor, torch.Tensor]:
        """`q_sample` (diffusion_model.py:213-218)."""
        if noise is None:
            noise = _rng.source().randn_like(x_start)
        t = torch.clamp(t, 0, self.num_timesteps - 1)
        a = self.sqrt_alphas_cumprod[t].view(-1, 1, 1)
        b = self.sqrt_one_minus_alphas_cumprod[t].view(-1, 1, 1)
        return a * x_start + b * noise, noise

    def _apply_geometric_constraints(self, points: torch.Tensor,
                                     target_range: float = 1.8) -> torch.Tensor:
        return torch.tanh(points / target_range) * target_range

    def _timesteps(self, num_inference_steps: int):
        """The guided loop's schedule: CPU linspace(999, 0, n).long() (diffusion_model.py:236)."""
        return torch.linspace(self.num_timesteps - 1, 0, num_inference_steps).long().tolist()

    def _coeffs(self, t: int, t_prev: int):
        """fp32 scalars of the update, as the reference's 0-d tensor ops produce them."""
        one = np.float32(1.0)
        a = self._ac_host[t]
        ap = self._ac_host[t_prev] if t_prev >= 0 else one
        return (np.sqrt(one - a), np.sqrt(a) + np.float32(1e-8), np.sqrt(ap), np.sqrt(one - ap))

    @torch.no_grad()
    def guided_sample_loop(self, model: PointCloudDiffusionModel, source_points: torch.Tensor,
                           condition_points: torch.Tensor, num_inference_steps: int = 50,
                           guidance_scale: float = 7.5, *,
                           x_T: Optional[torch.Tensor] = None, graph: bool = False) -> torch.Tensor:
        """`guided_sample_loop` (diffusion_model.py:224-261).

        graph=True (keyword-only, BASELINE configs[4]): the hierarchical denoise step is captured
        once into a hipGraph and replayed per timestep; the per-step scalars (timestep rows, DDIM
        coefficients, subset seed) are copied into static device buffers between replays.  Same
        draws and kernels as the eager loop, so the result is bit-identical."""
        if graph and source_points.shape[1] > model.config.global_points \
                and not _rng.source().replaying:
            return self._guided_sample_graph(model, source_points, condition_points,
                                             num_inference_steps, guidance_scale, x_T)
        device = source_points.device
        shape = source_points.shape
        B = shape[0]
        hp = model.hierarchical_processor
        style_feat = model.style_encoder(hp.downsample(condition_points)[0])
        style_in = torch.cat([style_feat, torch.zeros_like(style_feat)])
        x = x_T.to(device).float() if x_T is not None else _rng.source().randn(shape, device)
        timesteps = self._timesteps(num_inference_steps)
        use_hierarchical = shape[1] > model.config.global_points
        npred = model.noise_predictor
        # the CFG batch's timestep rows for the whole schedule, built once (one copy, no
        # per-step fill kernel)
        t_rows = torch.tensor(timesteps, dtype=torch.long).repeat_interleave(2 * B)
        t_rows = t_rows.view(len(timesteps), 2 * B).to(device)
        # the reference's t_prev lookup (first occurrence of t, diffusion_model.py:252)
        t_prevs = [timesteps[timesteps.index(t) + 1] if t > 0 else -1 for t in timesteps]
        # every step's conditioning rows (time_proj + style_proj + b4, per CFG row) in one launch:
        # they depend only on t and the style features, not on x
        conds = pk = None
        if npred.fused_inference(style_in):
            S = len(timesteps)
            pk = npred.packed()  # the loop changes no weight
            conds = npred.cond(t_rows.reshape(-1), style_in.repeat(S, 1), pk).view(S, 2 * B, -1)
        overlap = use_hierarchical and overlap_knn_build(2 * B * model.config.global_points)
        slot = overlap_slot(device) if overlap else None
        if slot is not None and not slot.acquire(blocking=False):
            overlap, slot = False, None  # another loop holds the device's overlapped layout
        try:
            return self._guided_loop_body(model, source_points, B, shape, hp, style_in, x, timesteps,
                                          use_hierarchical, npred, t_rows, t_prevs, conds, pk,
                                          overlap, guidance_scale, device)
        finally:
            if slot is not None:
                slot.release()

    def _guided_loop_body(self, model, source_points, B, shape, hp, style_in, x, timesteps,
                          use_hierarchical, npred, t_rows, t_prevs, conds, pk, overlap,
                          guidance_scale, device):
        source = source_points.float().contiguous()
        x_cat = torch.cat([x, x]).contiguous()
        state = ws = vws = None
        ctx = contextlib.nullcontext()
        if overlap:
            state = StepState(device)
            caller = torch.cuda.current_stream(device)
            state.begin(caller)
            ctx = torch.cuda.stream(state.loop)
        rows_ws = None
        with ctx:
            if overlap and rows_layout_ok(2 * B * model.config.global_points):
                rows_ws = _hip.knn_rows_workspace(B, 2, shape[1], model.config.global_points, device)
            elif overlap:
                ws = _hip.knn_workspace(2 * B, shape[1], model.config.global_points, device=device)
            if use_hierarchical:
                vws = _hip.voxel_copies_workspace(B, shape[1], 2, device=device)
            prepped = pool = False
            next_seed = None
            try:
                for i, t in enumerate(timesteps):
                    t_in = t_rows[i]
                    if conds is not None:
                        cond_i = conds[i]
                        mlp = lambda c, wait=None, start=None: (  # noqa: E731
                            npred.forward_cond(c, cond_i, pk, wait, start))
                    else:
                        mlp = lambda c: npred(c, t_in, style_in)  # noqa: E731
                    coeffs = self._coeffs(t, t_prevs[i])
                    if use_hierarchical:
                        rows, start = (knn_rows_begin(x, model.config.global_points, state,
                                                      rows_ws, by_downsample=prepped)
                                       if rows_ws is not None else (None, None))
                        xc, xi = hp.downsample_copies(x, 2, vws, prepped, next_seed, pool, start,
                                                      rows=rows,
                                                      rows_wait=state.built_sig if rows else None)
                        prep = i + 1 < len(timesteps) and voxel_prep_ok(hp, x, state)
                        # the next step's subset seed, drawn one step ahead for its pool histogram
                        next_seed = (_rng.source().device_seed() & (2**64 - 1)
                                     if prep and pool_prep_ok(x) else None)
                        x = hierarchical_step(hp, mlp, xc, xi, x_cat, x, source, guidance_scale,
                                              coeffs, ws, state, fused=conds is not None,
                                              vox_ws=vws if prep else None, pool_seed=next_seed,
                                              rows=rows)
                        prepped, pool = prep, next_seed is not None
                    else:
                        eps = mlp(x_cat)
                        x = _hip.cfg_ddim_step(x, eps[:B], eps[B:], source, guidance_scale,
                                               coeffs, x_cat=x_cat)
            finally:
                # also when a step raises: tensors the caller frees must not be reused while
                # loop-stream and side-stream kernels still run
                if overlap:
                    state.end(caller)
        if overlap:
            state.check()  # a timed-out device wait is an error, never a silent wrong result
        return x

    def _guided_sample_graph(self, model, source_points, condition_points, num_inference_steps,
                             guidance_scale, x_T):
        device = source_points.device
        shape = source_points.shape
        B = shape[0]
        hp = model.hierarchical_processor
        npred = model.noise_predictor
        style_feat = model.style_encoder(hp.downsample(condition_points)[0])
        style_in = torch.cat([style_feat, torch.zeros_like(style_feat)])
        x = (x_T.to(device).float() if x_T is not None
             else _rng.source().randn(shape, device)).contiguous().clone()
        timesteps = self._timesteps(num_inference_steps)
        t_prevs = [timesteps[timesteps.index(t) + 1] if t > 0 else -1 for t in timesteps]
        source = source_points.float().contiguous()
        x_cat = torch.cat([x, x]).contiguous()
        S = len(timesteps)
        # per-step scalars, drawn/computed in the eager loop's order, resident on the device
        seeds = [_rng.source().device_seed() & (2**64 - 1) for _ in range(S)]
        seed_tab = torch.tensor([v - 2**64 if v >= 2**63 else v for v in seeds],
                                dtype=torch.int64).to(device)
        coef_tab = torch.tensor(np.array([self._coeffs(t, tp) for t, tp in zip(timesteps, t_prevs)],
                                         dtype=np.float32)).to(device)
        t_tab = torch.tensor(timesteps, dtype=torch.long).repeat_interleave(2 * B)
        t_tab = t_tab.view(S, 2 * B).to(device)
        t_cur, coef_cur, seed_cur = t_tab[0].clone(), coef_tab[0].clone(), seed_tab[:1].clone()
        npred.packed()  # weight packing happens outside the capture
        M = model.config.global_points

        # the kNN build on a forked graph branch beside the MLP (GRAPH_FORK_BUILD; uncapped it
        # measured slower than inline at 32 clouds: 7.65-7.86 vs 7.38-7.50 ms per step,
        # profiles/r05/s2o, s2p)
        capture = torch.cuda.Stream(device=device)
        branch = torch.cuda.Stream(device=device)
        knn_ws = _hip.knn_workspace(2 * B, x_cat.shape[1], M, device)

        def step():
            xc, xi = _hip.voxel_downsample_copies_dseed(x, M, seed_cur, 2)
            if GRAPH_FORK_BUILD:
                # the build (positions only) on a graph branch beside the MLP, joined before the query
                branch.wait_stream(capture)
                with torch.cuda.stream(branch):
                    handle = _hip.knn3_build(x_cat, xi, knn_ws, knn_build_lds_floor(xc.shape[0] * xc.shape[1]),
                                             KNN_BUILD_MAX_WG)
                nc = npred(xc, t_cur, style_in)
                capture.wait_stream(branch)
                eps = _hip.knn3_query(nc, handle)
            else:
                eps = hp.upsample_knn(npred(xc, t_cur, style_in), x_cat, xi)
            _hip.cfg_ddim_step_dcoef(x, eps[:B], eps[B:], source, guidance_scale, coef_cur,
                                     x_cat=x_cat, out=x)

        g = torch.cuda.CUDAGraph()
        capture.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(capture):
            with torch.cuda.graph(g, stream=capture):
                step()
        torch.cuda.current_stream().wait_stream(capture)
        for i in range(S):
            t_cur.copy_(t_tab[i])
            coef_cur.copy_(coef_tab[i])
            seed_cur.copy_(seed_tab[i:i + 1])
            g.replay()
        return x

    @torch.no_grad()
    def ddim_sample_loop(self, model: PointCloudDiffusionModel, shape: Tuple,
                         condition_points: torch.Tensor, num_inference_steps: int = 50, *,
                         x_T: Optional[torch.Tensor] = None) -> torch.Tensor:
        """`ddim_sample_loop` (diffusion_model.py:263-293): full model.forward every step."""
        device = condition_points.device
        x = x_T.to(device).float() if x_T is not None else _rng.source().randn(shape, device)
        timesteps = torch.linspace(self.num_timesteps - 1, 0, num_inference_steps,
                                   dtype=torch.long).tolist()
        use_hierarchical = shape[1] > model.config.global_points
        for i, t in enumerate(timesteps):
            prev_t = timesteps[i + 1] if i < len(timesteps) - 1 else -1
            batch_t = torch.full((shape[0],), t, device=device, dtype=torch.long)
            if use_hierarchical:
                nc, idx = model(x, batch_t, condition_points, cond_drop_prob=0,
                                use_hierarchical=True)
                eps = model.hierarchical_processor.upsample_knn(nc, x, idx)
            else:
                eps, _ = model(x, batch_t, condition_points, cond_drop_prob=0,
                               use_hierarchical=False)
            x = _hip.cfg_ddim_step(x, eps, None, None, 0.0, self._coeffs(t, prev_t))
        return x
