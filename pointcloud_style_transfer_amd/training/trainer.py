"""Training entry point -- drop-in for the reference's `training/trainer.py` (DiffusionTrainer,
CosineWithWarmupLR: same constructor, epoch/step semantics, loss, clipping, AdamW, EMA and
checkpoint cadence).

Compute runs on the MI355X kernels: voxel downsample, FPS / ball query, the per-point linear
layers (forward AND backward, models/_autograd.py), Chamfer / L1 losses (csrc/chamfer.hip).
Data parallelism: when torch.distributed is initialised with world_size > 1
the model is wrapped in DistributedDataParallel (RCCL all-reduce of the fp32 gradients over
xGMI, overlapped with backward); BN statistics stay rank-local as in the reference (no
SyncBN); clip/AdamW/EMA run replicated after the all-reduce, so ranks stay identical.

Under DDP: micro-steps that do not end an accumulation window run under `no_sync()`, so the
gradient all-reduce happens once per optimizer step (the summed micro-batch gradients equal the
reference's accumulation over the same samples, trainer.py:115-125); ranks > 0 re-seed the
torch generators with `initial_seed() + rank`, so each rank draws its own t, noise, dropout
and voxel subsets; the EMA is built after the DDP wrap, from rank 0's broadcast weights; the
validation loss is averaged over ranks before the best/patience decision, so every rank stops
at the same epoch; the train sampler's epoch is set every epoch.

Precision under `use_amp` (the reference's default): the per-point linear layers run on 16-bit
MFMA with fp32 accumulation (models/_autograd.py -> pcst_gemm_ex / pcst_gemm_nt_bf16 /
pcst_linear_wgrad_bf16) in `Config.amp_dtype`: float16 by default, the reference's CUDA
autocast (trainer.py:50,78; 11 mantissa bits, the GradScaler guards the range), or bfloat16
(8 bits, fp32's exponent range); both run at the same MFMA rate.  Geometry, BN statistics,
Chamfer and L1 stay fp32.  `use_amp=False` runs every product in exact f32 (the gradient
parity tests).
The GradScaler logic is kept as is.  TensorBoard is optional (not installed here).
"""
from __future__ import annotations

import contextlib
import math
import os
from typing import Optional

import numpy as np
import torch
import torch.distributed as dist
import torch.optim as optim
from torch.amp import GradScaler, autocast

from .. import _hip
from .. import rng as _rng
from ..config.config import Config
from ..models.diffusion_model import DiffusionProcess, PointCloudDiffusionModel
from ..models.losses import DiffusionLoss
from ..utils.checkpoint import CheckpointManager
from ..utils.ema import ExponentialMovingAverage
from ..utils.logger import Logger

try:  # trainer.py:5 -- optional here
    from torch.utils.tensorboard import SummaryWriter
except Exception:  # noqa: BLE001
    class SummaryWriter:  # type: ignore
        def __init__(self, *a, **k):
            pass

        def add_scalar(self, *a, **k):
            pass

        def close(self):
            pass


class CosineWithWarmupLR:
    """`CosineWithWarmupLR` (trainer.py:20-34)."""

    def __init__(self, optimizer, warmup_epochs, total_epochs, min_lr_ratio=0.01):
        self.optimizer = optimizer
        self.warmup_epochs = warmup_epochs
        self.total_epochs = total_epochs
        self.min_lr_ratio = min_lr_ratio
        self.base_lrs = [g["lr"] for g in optimizer.param_groups]
        self.current_epoch = 0

    def step(self):
        self.current_epoch += 1
        if self.current_epoch <= self.warmup_epochs:
            scale = self.current_epoch / self.warmup_epochs
        else:
            progress = (self.current_epoch - self.warmup_epochs) / (self.total_epochs - self.warmup_epochs)
            scale = self.min_lr_ratio + 0.5 * (1 - self.min_lr_ratio) * (1 + math.cos(math.pi * progress))
        for g, base in zip(self.optimizer.param_groups, self.base_lrs):
            g["lr"] = base * scale


def keep_fused(optimizer, state_dict):
    """load_state_dict pre-hook of the fused AdamW: Optimizer.load_state_dict replaces the
    param groups with the saved ones, and a checkpoint written by the reference (or by a
    non-fused optimizer) carries fused=None.  The optimizer would then step with the foreach
    kernel while GradScaler, seeing a fused optimizer, hands it found_inf -- which that kernel
    rejects.  Keep the groups fused; `step` is then loaded onto the device as float32 (torch's
    rule for fused state)."""
    sd = dict(state_dict)
    sd["param_groups"] = [dict(g, fused=True, foreach=None) for g in state_dict["param_groups"]]
    return sd


def _progress(it, desc):
    try:
        from tqdm import tqdm

        return tqdm(it, desc=desc)
    except Exception:  # noqa: BLE001
        return it


class DeferredLosses:
    """One step's loss values, copied to pinned host memory behind the step (no host wait):
    read() waits for that copy only -- a `.item()` on the step's tensors would be ordered behind
    everything queued after the step as well."""

    def __init__(self, loss: torch.Tensor, terms: dict):
        self.keys = list(terms)
        vals = torch.stack([loss.detach().float().reshape(())]
                           + [terms[k].detach().float().reshape(()) for k in self.keys])
        self.buf = torch.empty(len(self.keys) + 1, dtype=torch.float32, pin_memory=True)
        self.buf.copy_(vals, non_blocking=True)
        self.ready = torch.cuda.Event()
        self.ready.record()

    def read(self):
        """(loss, {term: value}) as python floats (the values `.item()` gives)."""
        self.ready.synchronize()
        v = self.buf.tolist()
        return v[0], dict(zip(self.keys, v[1:]))


class DiffusionTrainer:
    """`DiffusionTrainer` (trainer.py:36-232)."""

    def __init__(self, config: Config, device: str = "cuda", *, ddp: Optional[bool] = None):
        """ddp (keyword-only): None wraps the model in DDP when a process group of world size
        > 1 is initialised; True wraps it whenever a process group is initialised, world size 1
        included (the RCCL smoke test: DDP's reducer then all-reduces through a one-rank
        communicator)."""
        self.config = config
        self.device = torch.device(device)
        self.device_type = "cuda" if "cuda" in str(self.device) else "cpu"
        group = dist.is_available() and dist.is_initialized()
        self.distributed = group and (dist.get_world_size() > 1 or bool(ddp))
        self.rank = dist.get_rank() if self.distributed else 0
        self.logger = Logger(name="DiffusionTrainer", log_dir=config.log_dir,
                             experiment_name=config.experiment_name, file_output=self.rank == 0)
        self.model = PointCloudDiffusionModel(config).to(self.device)
        self.diffusion_process = DiffusionProcess(config, device=str(self.device))
        self.loss_fn = DiffusionLoss(noise_weight=1.0, chamfer_weight=config.lambda_chamfer)
        # fused AdamW on the GPU: one kernel for all parameters, and GradScaler hands it
        # found_inf on the device instead of synchronising on it (torch's amp-scaling protocol)
        fused = self.device_type == "cuda"
        self.optimizer = optim.AdamW(self.model.parameters(), lr=config.learning_rate,
                                     weight_decay=config.weight_decay, betas=(0.9, 0.95),
                                     fused=fused)
        if fused:
            self.optimizer.register_load_state_dict_pre_hook(keep_fused)
        if config.lr_scheduler == "cosine_with_warmup":
            self.scheduler = CosineWithWarmupLR(self.optimizer, config.warmup_epochs,
                                                config.num_epochs, config.min_lr_ratio)
        else:
            self.scheduler = optim.lr_scheduler.CosineAnnealingLR(
                self.optimizer, T_max=config.num_epochs, eta_min=config.learning_rate * 0.01)
        self.scaler = GradScaler(enabled=(config.use_amp and self.device_type == "cuda"))
        self.writer = SummaryWriter(log_dir=os.path.join(config.log_dir, config.experiment_name))
        self.checkpoint_manager = CheckpointManager(config.checkpoint_dir, config.experiment_name)
        self.best_val_loss = float("inf")
        self.current_epoch = 0
        self.patience_counter = 0
        self.max_patience = 20
        self.gradient_accumulation_steps = config.gradient_accumulation_steps
        self.gradient_clip_norm = 1.0
        self.ddp_model = self.model
        # train_step(next_batch=...): the next batch's style geometry (condition-cloud downsample,
        # FPS, ball query: positions only) is queued on a side stream at the start of a step and
        # runs beside it; the next step's forward then starts at the SA MLPs.  Off while draws
        # are replayed (the parity tests follow the reference's draw order).
        # Draw order: with prefetch on, batch k+1's geometry draws (the condition cloud's voxel
        # subset seed, the SA1/SA2 FPS starts) are made at the start of step k, BEFORE step k's
        # timestep / noise / cond-drop / dropout draws.  A seeded epoch therefore consumes the
        # global generator in a different order than the same train_step calls without
        # next_batch (and than the reference, trainer.py:70-127): the runs are equally valid
        # samples but intentionally not draw-for-draw identical.  Set this to False for the
        # reference's order (every parity test runs with it off or under a replay source).
        self.prefetch_style_geometry = self.device_type == "cuda"
        self._geo_next = None  # (condition tensor it was computed for, geometry, ready event)
        self._geo_stream = None
        self._geo_dstream = None
        if self.distributed:
            from torch.nn.parallel import DistributedDataParallel as DDP

            self.ddp_model = DDP(self.model, device_ids=[self.device.index] if self.device.index is not None else None,
                                 broadcast_buffers=False, bucket_cap_mb=16)
            # every rank draws its own t / noise / dropout / voxel subsets
            if self.rank > 0:
                torch.manual_seed(torch.initial_seed() + self.rank)
        # after the wrap: DDP has broadcast rank 0's weights, so every rank's shadows agree
        self.ema = ExponentialMovingAverage(self.model.parameters(), decay=config.ema_decay)

    # ------------------------------------------------------------------ one step
    def _is_sync_step(self, batch_idx: int, num_batches: int) -> bool:
        return ((batch_idx + 1) % self.gradient_accumulation_steps == 0
                or batch_idx == num_batches - 1)

    def train_step(self, batch, batch_idx: int, num_batches: int, *, host_sync: bool = True,
                   next_batch=None):
        """Body of the per-batch loop of train_one_epoch (trainer.py:70-127).

        host_sync=False (keyword-only) returns (loss tensor, DeferredLosses) instead of the
        reference's python floats: nothing waits for the device, so the caller can queue the
        next step before reading this one's values (train_one_epoch does; see _log_step).
        next_batch (keyword-only): the batch the next call will get; its style geometry is
        computed beside this step (prefetch_style_geometry)."""
        sync = self._is_sync_step(batch_idx, num_batches)
        geo = self._take_geometry(batch)
        if next_batch is not None:
            self._queue_geometry(next_batch)
        # DDP: all-reduce only on the micro-step that ends the accumulation window
        ctx = (self.ddp_model.no_sync() if self.distributed and not sync
               else contextlib.nullcontext())
        with ctx:
            loss, terms = self._forward_backward(batch, geo)
        if sync:
            self.scaler.unscale_(self.optimizer)
            torch.nn.utils.clip_grad_norm_(self.model.parameters(), self.gradient_clip_norm)
            self.scaler.step(self.optimizer)
            self.scaler.update()
            self.optimizer.zero_grad()
            self.ema.update()
        if not host_sync:
            return loss.detach(), DeferredLosses(loss, terms)
        # the reference's loss dict of python floats (losses.py:93-102), read once the whole
        # step is queued: its syncs then wait on work already in flight
        loss_dict = {k: v.item() for k, v in terms.items()}
        return loss, loss_dict

    def _prefetching(self) -> bool:
        return (self.prefetch_style_geometry and self.device_type == "cuda"
                and not _rng.source().replaying)

    def _queue_geometry(self, batch):
        """Queue batch's style geometry on the side stream, ordered after the work queued so far
        (not after this step's forward and backward, which are queued next)."""
        if not self._prefetching():
            return
        real = batch["real_full"]
        main = torch.cuda.current_stream(self.device)
        if self._geo_stream is None:
            # a stream of its own at the device's greatest priority: a pool stream
            # (torch.cuda.Stream) can land on the hardware queue of the main stream, depending on
            # how many streams the process created before (a forked hipGraph branch earlier in the
            # bench made the step 9.7 -> 10.4 ms: the prefetch then serialised with the step)
            self._geo_dstream = _hip.DeviceStream(self.device, priority=-1)
            self._geo_stream = self._geo_dstream.stream
        side = self._geo_stream
        side.wait_stream(main)
        with torch.cuda.stream(side), torch.no_grad():
            real_dev = real.to(self.device, non_blocking=True)
            geo = self.model.style_geometry(real_dev, self.config.use_hierarchical)
            ready = torch.cuda.Event()
            ready.record(side)
        self._geo_next = (real, (real_dev, geo), ready)

    def _take_geometry(self, batch):
        """The prefetched geometry if it was computed for this batch's condition cloud."""
        pending, self._geo_next = self._geo_next, None
        if pending is None or pending[0] is not batch["real_full"] or not self._prefetching():
            return None
        real_dev, (xyz, geo) = pending[1]
        main = torch.cuda.current_stream(self.device)
        main.wait_event(pending[2])
        for t in [real_dev, xyz] + [u for g in geo for u in g]:
            t.record_stream(main)  # made on the side stream, used and freed on this one
        return real_dev, (xyz, geo)

    def _log_step(self, pbar, loss, deferred) -> float:
        """One step's contribution to the epoch's loss sum and its progress-bar line."""
        loss_value, loss_dict = deferred.read()
        if hasattr(pbar, "set_postfix"):
            pbar.set_postfix({"Loss": f"{loss_dict.get('total_loss', 0):.4f}",
                              "L1": f"{loss_dict.get('noise_loss', 0):.4f}",
                              "CD": f"{loss_dict.get('chamfer_loss', 0):.4f}",
                              "LR": f"{self.optimizer.param_groups[0]['lr']:.2e}"})
        return loss_value * self.gradient_accumulation_steps

    def _amp_dtype(self):
        name = getattr(self.config, "amp_dtype", "float16")
        if name not in ("float16", "bfloat16"):
            raise ValueError(f"Config.amp_dtype must be 'float16' or 'bfloat16', got {name!r}")
        return getattr(torch, name)

    def _forward_backward(self, batch, geo=None):
        # non_blocking: from a pinned loader batch the copies do not stall the host
        sim = batch["sim_full"].to(self.device, non_blocking=True)
        real = batch["real_full"].to(self.device, non_blocking=True) if geo is None else geo[0]
        B, N, C = sim.shape
        src = _rng.source()
        t = src.randint(0, self.config.num_timesteps, (B,), device=self.device).long()
        noisy, actual_noise = self.diffusion_process.q_sample(sim, t)
        with autocast(device_type=self.device_type, enabled=self.config.use_amp,
                      dtype=self._amp_dtype()):
            pred, indices = self.ddp_model(noisy_points=noisy, timestep=t, condition_points=real,
                                           cond_drop_prob=self.config.cond_drop_prob,
                                           use_hierarchical=self.config.use_hierarchical,
                                           style_geometry=None if geo is None else geo[1])
            if indices is not None:
                ie = indices.unsqueeze(-1).expand(-1, -1, C)
                actual_coarse = torch.gather(actual_noise, 1, ie)
                pred_x0_coarse = sim_coarse = None
                if self.config.lambda_chamfer > 0:
                    noisy_coarse = torch.gather(noisy, 1, ie)
                    sim_coarse = torch.gather(sim, 1, ie)
                    a = self.diffusion_process.sqrt_alphas_cumprod[t].view(B, 1, 1)
                    b = self.diffusion_process.sqrt_one_minus_alphas_cumprod[t].view(B, 1, 1)
                    pred_x0_coarse = (noisy_coarse - b * pred) / (a + 1e-8)
                loss, terms = self.loss_fn.forward_tensors(
                    predicted_noise=pred, actual_noise=actual_coarse,
                    predicted_points_coarse=pred_x0_coarse, target_points_coarse=sim_coarse)
            else:
                loss, terms = self.loss_fn.forward_tensors(predicted_noise=pred,
                                                           actual_noise=actual_noise)
            loss = loss / self.gradient_accumulation_steps
        self.scaler.scale(loss).backward()
        return loss, terms

    def train_one_epoch(self, data_loader):
        self.model.train()
        total = 0.0
        pbar = _progress(data_loader, f"Epoch {self.current_epoch}/{self.config.num_epochs} [Train]")
        self.optimizer.zero_grad()
        n = len(data_loader)
        # The reference reads each step's loss with .item() right after the step (a device sync
        # that leaves the GPU idle while the host queues the next step's many small launches).
        # Here step k's values are read after step k + 1 is queued: the same sum and the same
        # progress-bar values, one step later.
        pending = None
        items = enumerate(pbar)
        cur = next(items, None)
        while cur is not None:
            nxt = next(items, None)  # one batch ahead: its style geometry runs beside this step
            batch_idx, batch = cur
            step = self.train_step(batch, batch_idx, n, host_sync=False,
                                   next_batch=None if nxt is None else nxt[1])
            if pending is not None:
                total += self._log_step(pbar, *pending)
            pending = step
            cur = nxt
        if pending is not None:
            total += self._log_step(pbar, *pending)
        avg = total / n
        self.writer.add_scalar("Loss/Train", avg, self.current_epoch)
        return avg

    @torch.no_grad()
    def validate_one_epoch(self, data_loader):
        """trainer.py:140-174 (EMA weights, eval mode, noise loss only)."""
        self.ema.apply_shadow()
        try:
            self.model.eval()
            total = 0.0
            for batch in _progress(data_loader, f"Epoch {self.current_epoch} [Val]"):
                loss = self._val_loss(batch)
                if math.isfinite(loss):
                    total += loss
            avg = total / len(data_loader)
            if self.distributed:
                # one decision for every rank (best / patience / stop), else a rank that
                # breaks early leaves the others hanging in the gradient all-reduce
                t = torch.tensor([avg], dtype=torch.float64, device=self.device)
                dist.all_reduce(t, op=dist.ReduceOp.SUM)
                avg = float(t.item()) / dist.get_world_size()
            self.writer.add_scalar("Loss/Validation", avg, self.current_epoch)
            return avg
        finally:
            self.ema.restore()

    def _val_loss(self, batch) -> float:
        """Noise loss of one validation batch (trainer.py:150-166)."""
        sim = batch["sim_full"].to(self.device)
        real = batch["real_full"].to(self.device)
        B, N, C = sim.shape
        t = _rng.source().randint(0, self.config.num_timesteps, (B,), device=self.device).long()
        noisy, actual = self.diffusion_process.q_sample(sim, t)
        pred, idx = self.model(noisy_points=noisy, timestep=t, condition_points=real,
                               cond_drop_prob=0, use_hierarchical=self.config.use_hierarchical)
        if idx is not None:
            actual = torch.gather(actual, 1, idx.unsqueeze(-1).expand(-1, -1, C))
        loss, _ = self.loss_fn(pred, actual)
        return float(loss.item())

    def save_sample_results(self, data_loader, num_samples: int = 2):
        """trainer.py:176-196."""
        self.ema.apply_shadow()
        try:
            self.model.eval()
            batch = next(iter(data_loader))
            sim = batch["sim_full"][:num_samples].to(self.device)
            real = batch["real_full"][:num_samples].to(self.device)
            with torch.no_grad():
                out = self.diffusion_process.guided_sample_loop(
                    model=self.model, source_points=sim, condition_points=real,
                    num_inference_steps=50, guidance_scale=self.config.guidance_scale)
            d = os.path.join(self.config.result_dir, self.config.experiment_name,
                             f"epoch_{self.current_epoch:04d}")
            os.makedirs(d, exist_ok=True)
            for i in range(num_samples):
                np.save(os.path.join(d, f"original_sim_{i}.npy"), sim[i].cpu().numpy())
                np.save(os.path.join(d, f"reference_real_{i}.npy"), real[i].cpu().numpy())
                np.save(os.path.join(d, f"transferred_{i}.npy"), out[i].cpu().numpy())
        finally:
            self.ema.restore()

    def train(self, train_loader, val_loader):
        """trainer.py:198-232."""
        self.current_epoch = self.checkpoint_manager.load(self.model, self.optimizer, self.ema)
        for _ in range(self.current_epoch):
            if hasattr(self.scheduler, "step"):
                self.scheduler.step()
        for epoch in range(self.current_epoch, self.config.num_epochs):
            self.current_epoch = epoch
            sampler = getattr(train_loader, "sampler", None)
            if hasattr(sampler, "set_epoch"):  # DistributedSampler: a new shuffle every epoch
                sampler.set_epoch(epoch)
            avg = self.train_one_epoch(train_loader)
            self.logger.info(f"Epoch {epoch}: train loss {avg:.6f}")
            if hasattr(self.scheduler, "step"):
                self.scheduler.step()
            if epoch % self.config.val_interval == 0:
                v = self.validate_one_epoch(val_loader)
                is_best = v < self.best_val_loss
                if is_best:
                    self.best_val_loss = v
                    self.patience_counter = 0
                else:
                    self.patience_counter += 1
                if self.rank == 0:
                    self.checkpoint_manager.save(self.model, self.optimizer, self.ema, epoch, is_best)
                if self.patience_counter >= self.max_patience:
                    break
                if epoch > 0 and epoch % (self.config.save_interval * 2) == 0 and self.rank == 0:
                    self.save_sample_results(val_loader)
        self.writer.close()
