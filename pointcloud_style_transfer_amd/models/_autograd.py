"""Autograd for the training path: per-point linear layers on the pointwise MFMA kernel
(csrc/sa_mlp.hip), forward and backward.

  forward   Y  = act(X W^T + b)                      pcst_pointwise_linear
  backward  dZ = dY * [Y > 0]  (ReLU)                 pcst_relu_bwd
            dX = dZ W          = linear(dZ, W^T)     pcst_pointwise_linear
            dW = dZ^T X, db = dZ^T 1                  pcst_linear_wgrad (split over row chunks)
All products are exact-f32 MFMA; the row reduction combines fixed chunks in order (no
atomics), so gradients are deterministic.  Under torch.autocast (the trainer's use_amp) the same
three products run on bf16 MFMA (pcst_gemm_nt_bf16 / pcst_linear_wgrad_bf16, csrc/train_gemm.hip).

The SetAbstraction training half (csrc/sa_train.hip):
  BNReLUFn       train-mode BatchNorm2d + ReLU (+ max over nsample with its argmax), forward
                 pcst_channel_stats / pcst_bn_train_coeffs / pcst_affine_act | pcst_bn_relu_maxpool,
                 backward pcst_bn_relu_bwd (dZ, dgamma, dbeta in one deterministic pass pair)
  GroupGatherFn  the grouped-feature gather (pcst_group_gather) and its deterministic scatter
                 backward (pcst_group_gather_bwd)
"""
from __future__ import annotations

import torch

from .. import _hip


class LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, relu):
        x2 = x.reshape(-1, x.shape[-1]).float().contiguous()
        W = weight.reshape(weight.shape[0], -1).float().contiguous()
        b = None if bias is None else bias.float()
        # under torch.autocast (the trainer's use_amp) the GEMMs run on bf16 MFMA
        ctx.bf16 = x2.is_cuda and torch.is_autocast_enabled("cuda")
        if ctx.bf16:
            y = _hip.gemm_nt_bf16(x2, W, None, b, relu)
        else:
            y = _hip.pointwise_linear(x2, W, None, b, relu, 0)
        ctx.relu = relu
        ctx.has_bias = bias is not None
        ctx.wshape = weight.shape
        ctx.xshape = x.shape
        ctx.save_for_backward(x2, W, y if relu else None)
        return y.view(*x.shape[:-1], W.shape[0])

    @staticmethod
    def backward(ctx, gy):
        x2, W, y = ctx.saved_tensors
        dz = gy.reshape(-1, W.shape[0]).float().contiguous()
        if ctx.relu:
            dz = _hip.relu_bwd(dz, y)
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            gemm = _hip.gemm_nt_bf16 if ctx.bf16 else _hip.pointwise_linear
            dx = gemm(dz, W.t().contiguous()).view(ctx.xshape)
        need_b = ctx.has_bias and ctx.needs_input_grad[2]
        if ctx.needs_input_grad[1] or need_b:
            dw, db = _hip.linear_wgrad(dz, x2, bias=need_b, bf16=ctx.bf16)
            dw = dw.view(ctx.wshape) if ctx.needs_input_grad[1] else None
        return dx, dw, db, None


class BNReLUFn(torch.autograd.Function):
    """relu(BatchNorm_train(z)) over the rows of z [M, O] (BatchNorm2d on [B, C, S, ns] with
    channel-last rows, pointnet2_encoder.py:108-110), optionally max-pooled over groups of
    `pool_ns` rows (:112).  Running statistics are updated on the device."""

    @staticmethod
    def forward(ctx, z, gamma, beta, running_mean, running_var, eps, momentum, pool_ns):
        z2 = z.reshape(-1, z.shape[-1]).float().contiguous()
        M = z2.shape[0]
        mean, var = _hip.channel_stats(z2)
        scale, shift, invstd = _hip.bn_train_coeffs(mean, var, M, gamma.detach(), beta.detach(),
                                                    eps, momentum, running_mean, running_var)
        arg = None
        if pool_ns:
            y, arg = _hip.bn_relu_maxpool(z2, scale, shift, pool_ns)
        else:
            y = _hip.affine_act(z2, scale, shift, True, 0)
        ctx.pool_ns = pool_ns
        ctx.save_for_backward(z2, scale, shift, mean, invstd, gamma, arg)
        return y

    @staticmethod
    def backward(ctx, gy):
        z2, scale, shift, mean, invstd, gamma, arg = ctx.saved_tensors
        gy = gy.float().contiguous()
        if ctx.pool_ns:
            dz, dg, db = _hip.bn_relu_bwd(z2, scale, shift, mean, invstd, gamma, dP=gy, arg=arg,
                                          ns=ctx.pool_ns)
        else:
            dz, dg, db = _hip.bn_relu_bwd(z2, scale, shift, mean, invstd, gamma, dY=gy)
        return (dz if ctx.needs_input_grad[0] else None,
                dg if ctx.needs_input_grad[1] else None,
                db if ctx.needs_input_grad[2] else None, None, None, None, None, None)


def bn_relu(z, bn, pool_ns=0):
    """Train-mode `bn` (BatchNorm2d) + ReLU (+ max-pool) on the HIP kernels."""
    momentum = bn.momentum
    if bn.track_running_stats:
        bn.num_batches_tracked.add_(1)
        if momentum is None:  # cumulative moving average
            momentum = 1.0 / float(bn.num_batches_tracked.item())
    rm = bn.running_mean if bn.track_running_stats else None
    rv = bn.running_var if bn.track_running_stats else None
    return BNReLUFn.apply(z, bn.weight, bn.bias, rm, rv, bn.eps,
                          0.0 if momentum is None else momentum, pool_ns)


class GroupGatherFn(torch.autograd.Function):
    """(new_xyz, [xyz - centroid || points] grouped by group_idx) (pointnet2_encoder.py:92-99);
    the gradient flows to `points` only (xyz is data)."""

    @staticmethod
    def forward(ctx, xyz, points, fps_idx, group_idx):
        new_xyz, grouped = _hip.group_gather(xyz, points, fps_idx, group_idx)
        ctx.save_for_backward(group_idx)
        ctx.N = points.shape[1]
        ctx.mark_non_differentiable(new_xyz)
        return new_xyz, grouped

    @staticmethod
    def backward(ctx, g_new_xyz, g_grouped):
        (group_idx,) = ctx.saved_tensors
        dp = None
        if ctx.needs_input_grad[1]:
            dp = _hip.group_gather_bwd(g_grouped, group_idx, ctx.N)
        return None, dp, None, None


def linear(x, lin, relu=False):
    """nn.Linear / Conv2d-1x1 module applied through LinearFn."""
    return LinearFn.apply(x, lin.weight, lin.bias, relu)


def needs_grad(module) -> bool:
    return torch.is_grad_enabled() and any(p.requires_grad for p in module.parameters())
