"""Autograd for the training path: per-point linear layers on the pointwise MFMA kernel
(csrc/sa_mlp.hip), forward and backward.

  forward   Y  = act(X W^T + b)                      pcst_pointwise_linear
  backward  dZ = dY * [Y > 0]  (ReLU)                 pcst_relu_bwd
            dX = dZ W          = linear(dZ, W^T)     pcst_pointwise_linear
            dW = dZ^T X, db = dZ^T 1                  pcst_linear_wgrad (split over row chunks)
All products are exact-f32 MFMA; the row reduction combines fixed chunks in order (no
atomics), so gradients are deterministic.  Under torch.autocast (the trainer's use_amp) the same
three products run on bf16 MFMA (pcst_gemm_nt_bf16 / pcst_linear_wgrad_bf16, csrc/train_gemm.hip).
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


def linear(x, lin, relu=False):
    """nn.Linear / Conv2d-1x1 module applied through LinearFn."""
    return LinearFn.apply(x, lin.weight, lin.bias, relu)


def needs_grad(module) -> bool:
    return torch.is_grad_enabled() and any(p.requires_grad for p in module.parameters())
