"""PointNet++ SSG encoder on the MI355X kernels -- drop-in for the reference's
`models/pointnet2_encoder.py` (same functions, classes, parameter names and shapes).

Every compute step runs in libpcst_hip.so:
  square_distance / index_points / farthest_point_sample / query_ball_point  -> csrc/geometry.hip
  SetAbstraction grouping (gather, centring, concat)                         -> pcst_group_gather
  Conv2d 1x1 + BatchNorm2d + ReLU (+ max over nsample)                        -> csrc/sa_mlp.hip
Indices are bit-exact with the reference; features are fp32.
"""
from __future__ import annotations

from typing import List, Optional, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import _hip
from .. import rng as _rng
from . import _autograd as _ag


def square_distance(src: torch.Tensor, dst: torch.Tensor) -> torch.Tensor:
    """`square_distance` (pointnet2_encoder.py:8-15)."""
    return _hip.square_distance(src, dst)


def index_points(points: torch.Tensor, idx: torch.Tensor) -> torch.Tensor:
    """`index_points` (pointnet2_encoder.py:17-28)."""
    return _hip.index_points(points, idx)


def farthest_point_sample(xyz: torch.Tensor, npoint: int, *,
                          start_idx: Optional[torch.Tensor] = None) -> torch.Tensor:
    """`farthest_point_sample` (pointnet2_encoder.py:30-45).  The start index is drawn from the
    CPU generator exactly as the reference does (Q10); `start_idx=` overrides it."""
    B, N, _ = xyz.shape
    if start_idx is None:
        start_idx = _rng.source().randint(0, N, (B,))
    if not start_idx.is_cuda and xyz.is_cuda:
        # through pinned memory, asynchronously: a pageable host->device copy synchronises the
        # stream, which would stall the host on all the work queued before this forward
        start_idx = start_idx.pin_memory().to(xyz.device, non_blocking=True)
    return _hip.fps(xyz, npoint, start_idx.to(xyz.device))


def query_ball_point(radius: float, nsample: int, xyz: torch.Tensor,
                     new_xyz: torch.Tensor) -> torch.Tensor:
    """`query_ball_point` (pointnet2_encoder.py:47-59)."""
    return _hip.ball_query(radius, nsample, xyz, new_xyz)


class SetAbstraction(nn.Module):
    """`SetAbstraction` (pointnet2_encoder.py:61-112)."""

    def __init__(self, npoint: int, radius: float, nsample: int, in_channel: int, mlp: List[int],
                 group_all: bool = False):
        super().__init__()
        self.npoint = npoint
        self.radius = radius
        self.nsample = nsample
        self.mlp_convs = nn.ModuleList()
        self.mlp_bns = nn.ModuleList()
        last = in_channel + 3
        for out in mlp:
            self.mlp_convs.append(nn.Conv2d(last, out, 1))
            self.mlp_bns.append(nn.BatchNorm2d(out))
            last = out
        self.group_all = group_all

    def geometry(self, xyz: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
        """The layer's sampling and grouping (pointnet2_encoder.py:85-91): (FPS indices, their
        points, ball-query indices).  Positions only -- no parameter enters -- so a trainer can
        compute it ahead of the forward (DiffusionTrainer.prefetch_style_geometry)."""
        fidx = farthest_point_sample(xyz, self.npoint)
        new_xyz = index_points(xyz, fidx)
        gidx = query_ball_point(self.radius, self.nsample, xyz, new_xyz)
        return fidx, new_xyz, gidx

    def forward(self, xyz: torch.Tensor, points: Optional[torch.Tensor] = None,
                geometry: Optional[tuple] = None) -> Tuple[torch.Tensor, torch.Tensor]:
        B, N, _ = xyz.shape
        if self.group_all:
            new_xyz = torch.zeros(B, 1, 3, device=xyz.device)
            grouped = xyz if points is None else torch.cat([xyz, points], dim=-1)
            feats = self.apply_mlp(grouped.reshape(B * N, -1), pool_ns=N)  # [B, C]
            return new_xyz, feats
        fidx, new_xyz, gidx = geometry if geometry is not None else self.geometry(xyz)
        if points is not None and points.requires_grad and torch.is_grad_enabled():
            # training: the same fused gather, with its deterministic scatter backward
            new_xyz, grouped = _ag.GroupGatherFn.apply(xyz, points, fidx, gidx)
        else:
            new_xyz, grouped = _hip.group_gather(xyz, points, fidx, gidx)
        feats = self.apply_mlp(grouped.reshape(B * self.npoint * self.nsample, -1),
                               pool_ns=self.nsample)
        return new_xyz, feats.view(B, self.npoint, -1).permute(0, 2, 1)

    def apply_mlp(self, x: torch.Tensor, pool_ns: int) -> torch.Tensor:
        """(Conv2d 1x1 -> BatchNorm2d -> ReLU) x L, then max over each group of `pool_ns`
        rows.  x: [rows, C] channel-last."""
        if _ag.needs_grad(self) or (x.requires_grad and torch.is_grad_enabled()):
            return self._apply_mlp_train(x, pool_ns)
        n = len(self.mlp_convs)
        for i, (conv, bn) in enumerate(zip(self.mlp_convs, self.mlp_bns)):
            W = conv.weight.view(conv.out_channels, -1)
            pool = pool_ns if i == n - 1 else 0
            if not bn.training:
                scale = bn.weight / torch.sqrt(bn.running_var + bn.eps)
                shift = (conv.bias - bn.running_mean) * scale + bn.bias
                x = _hip.pointwise_linear(x, W.detach(), scale.detach(), shift.detach(), True, pool)
            else:
                z = _hip.pointwise_linear(x, W.detach(), None, conv.bias.detach(), False, 0)
                mean, var = _hip.channel_stats(z)
                with torch.no_grad():
                    m = bn.momentum
                    M = z.shape[0]
                    bn.running_mean.mul_(1 - m).add_(mean.float(), alpha=m)
                    bn.running_var.mul_(1 - m).add_((var * (M / max(M - 1, 1))).float(), alpha=m)
                    bn.num_batches_tracked.add_(1)
                scale = bn.weight.detach() / torch.sqrt(var.float() + bn.eps)
                shift = bn.bias.detach() - mean.float() * scale
                x = _hip.affine_act(z, scale, shift, True, pool)
        return x

    def _apply_mlp_train(self, x: torch.Tensor, pool_ns: int) -> torch.Tensor:
        """Differentiable variant: conv GEMMs on the MFMA kernel, train-mode BatchNorm + ReLU
        (+ the max over nsample on the last layer) on csrc/sa_train.hip, all with HIP
        backward (models/_autograd.py).  Eval-mode BN under autograd (not a trainer path)
        keeps the torch ops."""
        n = len(self.mlp_convs)
        for i, (conv, bn) in enumerate(zip(self.mlp_convs, self.mlp_bns)):
            z = _ag.LinearFn.apply(x, conv.weight, conv.bias, False)
            last = i == n - 1
            if bn.training:
                x = _ag.bn_relu(z, bn, pool_ns if last else 0)
                continue
            x = F.relu(F.batch_norm(z, bn.running_mean, bn.running_var, bn.weight, bn.bias,
                                    False, bn.momentum, bn.eps))
            if last:
                x = x.view(-1, pool_ns, x.shape[-1]).max(dim=1)[0]
        return x


class PointNet2Encoder(nn.Module):
    """`PointNet2Encoder` (pointnet2_encoder.py:114-131)."""

    def __init__(self, input_channels: int = 3, feature_dim: int = 512):
        super().__init__()
        self.sa1 = SetAbstraction(512, 0.2, 32, in_channel=0, mlp=[64, 64, 128])
        self.sa2 = SetAbstraction(128, 0.4, 64, in_channel=128, mlp=[128, 128, 256])
        self.sa3 = SetAbstraction(npoint=None, radius=None, nsample=None, in_channel=256,
                                  mlp=[256, 512, feature_dim], group_all=True)

    def geometry(self, xyz: torch.Tensor) -> list:
        """SA1's and SA2's sampling and grouping for `xyz`, in the forward's draw order."""
        g1 = self.sa1.geometry(xyz)
        return [g1, self.sa2.geometry(g1[1])]

    def forward(self, xyz: torch.Tensor, geometry: Optional[list] = None) -> torch.Tensor:
        B = xyz.shape[0]
        g1, g2 = geometry if geometry is not None else (None, None)
        l1_xyz, l1_points = self.sa1(xyz, None, g1)
        l2_xyz, l2_points = self.sa2(l1_xyz, l1_points.permute(0, 2, 1), g2)
        _, g = self.sa3(l2_xyz, l2_points.permute(0, 2, 1))
        return g.view(B, -1)
