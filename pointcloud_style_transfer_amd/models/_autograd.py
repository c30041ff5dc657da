"""Autograd for the training path: per-point linear layers on the pointwise MFMA kernel
(csrc/sa_mlp.hip), forward and backward.

  forward   Y  = act(X W^T + b)                      pcst_pointwise_linear
  backward  dZ = dY * [Y > 0]  (ReLU)                 pcst_relu_bwd
            dX = dZ W          = linear(dZ, W^T)     pcst_pointwise_linear
            dW = dZ^T X, db = dZ^T 1                  pcst_linear_wgrad (split over row chunks)
All products are exact-f32 MFMA; the row reduction combines fixed chunks in order (no
atomics), so gradients are deterministic.  Under torch.autocast (the trainer's use_amp) the same
three products run on 16-bit MFMA in autocast's dtype -- float16 by default on CUDA, the
reference trainer's (training/trainer.py:50,78), or bfloat16 (pcst_gemm_nt_bf16 /
pcst_linear_wgrad_bf16, csrc/train_gemm.hip, f16 flag).

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


def autocast_half():
    """The 16-bit operand dtype of the CUDA autocast region this runs in (float16 unless the
    caller asked autocast for bfloat16), or None outside one."""
    if not torch.is_autocast_enabled("cuda"):
        return None
    h = torch.get_autocast_dtype("cuda")
    return h if h in (torch.float16, torch.bfloat16) else torch.float16


class LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, relu):
        x2 = x.reshape(-1, x.shape[-1]).float().contiguous()
        W = weight.reshape(weight.shape[0], -1).float().contiguous()
        b = None if bias is None else bias.float()
        # under torch.autocast (the trainer's use_amp) the GEMMs run on 16-bit MFMA
        ctx.half = autocast_half() if x2.is_cuda else None
        ctx.bf16 = ctx.half is not None
        if ctx.bf16:
            y = _hip.gemm_nt_bf16(x2, W, None, b, relu, half=ctx.half)
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
            if ctx.bf16:
                dx = _hip.gemm_nt_bf16(dz, W.t().contiguous(), half=ctx.half).view(ctx.xshape)
            else:
                dx = _hip.pointwise_linear(dz, W.t().contiguous()).view(ctx.xshape)
        need_b = ctx.has_bias and ctx.needs_input_grad[2]
        if ctx.needs_input_grad[1] or need_b:
            dw, db = _hip.linear_wgrad(dz, x2, bias=need_b, bf16=ctx.bf16,
                                       half=ctx.half or torch.bfloat16)
            dw = dw.view(ctx.wshape) if ctx.needs_input_grad[1] else None
        return dx, dw, db, None


def _h(w, half):
    return w.detach().to(half).contiguous()


def _h_t(w, half):
    return w.detach().t().to(half).contiguous()


# the fused blocks' backward reads the ReLU mask from 64 B of bits per row written by the forward
# (kernel v2) instead of h's 1 KiB per row (h itself is still kept: dW2 = dD^T h)
MASK_BITS = True
FUSED_BN_STATS = True  # BatchNorm forward: pcst_bn_train_stats instead of channel_stats + coeffs
BATCH_CAST = True   # one pcst_cast16_batch launch for a layer stack's 16-bit weight copies


def _cast_all(ts, half, transpose=False):
    """`_h` (or `_h_t`) of every tensor of `ts`: one launch when BATCH_CAST, else one each."""
    if BATCH_CAST:
        return _hip.cast16_batch(ts, half, [transpose] * len(ts))
    return [(_h_t if transpose else _h)(t, half) for t in ts]


def _draw_seed(p):
    """Dropout seed for one layer call: torch's CPU generator (torch.manual_seed governs it)."""
    return int(torch.randint(0, 2 ** 62, (1,)).item()) if p > 0 else 0


# Rows the fused residual-block kernels take: they address the [M, 512] 16-bit hidden
# activations with 32-bit byte offsets (pcst_resblock_fwd16 / _bwd16 reject M * 1024 >= 2^31);
# larger batches take the two-GEMM path (bit-identical), which has no such limit.
FUSED_BLOCK_MAX_ROWS = (2 ** 31 - 1) // 1024


def fused_block_rows_ok(M: int) -> bool:
    return M <= FUSED_BLOCK_MAX_ROWS


def _block_fwd(x, xb, w1, b1, w2, b2, p, seed):
    """x + Dropout_p(Linear2(ReLU(Linear1(x)))): -> (y fp32, y 16-bit, h 16-bit); the 16-bit
    format is that of xb / w1 / w2."""
    h = _hip.gemm_ex(xb, w1, b1, relu=True, epilogue=_hip.EP_BF16)
    y, yb = _hip.gemm_ex(h, w2, b2, epilogue=_hip.EP_RESID_DROP, aux=x, seed=seed, p=p,
                         copy_bf16=True)
    return y, yb, h


def _block_bwd(g, xb, h, w1_t, w2_t, p, seed, bias1=True, bias2=True):
    """Backward of _block_fwd from the fp32 gradient g of y: -> (gx, dW1, db1, dW2, db2)."""
    dd = _hip.dropout_grad_bf16(g, seed, p, half=xb.dtype)
    dz = _hip.gemm_ex(dd, w2_t, epilogue=_hip.EP_RELU_MASK, aux=h)
    gx = _hip.gemm_ex(dz, w1_t, epilogue=_hip.EP_ADD, aux=g)
    dw2, db2 = _hip.linear_wgrad_ex(dd, h, bias=bias2)
    dw1, db1 = _hip.linear_wgrad_ex(dz, xb, bias=bias1)
    return gx, dw1, db1, dw2, db2


class ResidualBlockFn(torch.autograd.Function):
    """x + Dropout_p(Linear2(ReLU(Linear1(x)))) -- one NoisePredictor layer
    (diffusion_model.py:48-52, applied at :57-58) -- under autocast, with 16-bit activation
    storage in autocast's dtype (written bf16 below; float16 by default) and the elementwise work
    fused into the GEMM epilogues (csrc/train_mlp.hip):

      forward   h  = bf16(relu(x W1^T + b1))                     EP_BF16
                y  = x + keep * (h W2^T + b2) / (1-p)           EP_RESID_DROP
      backward  dd = bf16(g * keep / (1-p))                     pcst_dropout_grad_bf16
                dz = bf16((dd W2) * [h > 0])                     EP_RELU_MASK
                gx = g + dz W1                                   EP_ADD
                dW2, db2 = dd^T h;  dW1, db1 = dz^T x            pcst_linear_wgrad_ex

    Every product rounds its operands to bf16 (LinearFn's autocast GEMMs do the same), so storing
    x, h, dd and dz as bf16 changes no product; the residual stream x and its gradient stay fp32.
    The dropout mask is a hash of (seed, element): one seed per call from torch's CPU generator,
    regenerated in the backward instead of stored."""

    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2, p):
        shape = x.shape
        half = autocast_half() or torch.bfloat16
        x2 = x.reshape(-1, shape[-1]).float().contiguous()
        xb = x2.to(half)
        seed = _draw_seed(p)
        y, _, h = _block_fwd(x2, xb, _h(w1, half), b1, _h(w2, half), b2, p, seed)
        ctx.save_for_backward(xb, h, w1, w2)
        ctx.seed, ctx.p, ctx.shape = seed, p, shape
        ctx.has_b = (b1 is not None, b2 is not None)
        return y.view(shape)

    @staticmethod
    def backward(ctx, gy):
        xb, h, w1, w2 = ctx.saved_tensors
        g = gy.reshape(xb.shape).float().contiguous()
        gx, dw1, db1, dw2, db2 = _block_bwd(g, xb, h, _h_t(w1, xb.dtype), _h_t(w2, xb.dtype),
                                            ctx.p, ctx.seed, *ctx.has_b)
        return gx.view(ctx.shape), dw1, db1, dw2, db2, None


def residual_block(x, layer, training):
    """`layer` = Sequential(Linear(fd, 2fd), ReLU, Linear(2fd, fd), Dropout) applied as
    x + layer(x) through ResidualBlockFn."""
    l1, l2, drop = layer[0], layer[2], layer[3]
    p = float(drop.p) if training else 0.0
    return ResidualBlockFn.apply(x, l1.weight, l1.bias, l2.weight, l2.bias, p)


# The residual stream x and its gradient in NoisePredictorFn: in autocast's 16-bit format (True,
# as the reference's autocast keeps them: every Linear output there is half precision) or fp32
# (False, the stricter round-2 layout).  16-bit halves the bytes of the residual epilogues and
# lets each Dropout backward ride on the epilogue that produces its gradient.
RESIDUAL_16BIT = True
# Each residual block's forward as one launch (pcst_resblock_fwd16: h never re-read from HBM;
# bit-identical to the EP_BF16 + EP_RESID_DROP16 pair).  tools/knobs.py may turn it off (A/B).
FUSED_BLOCK_FWD = True
# Each residual block's backward products (EP_RELU_MASK then EP_ADD16) as one launch
# (pcst_resblock_bwd16: dZ written once for dW1, never re-read; bit-identical).
FUSED_BLOCK_BWD = True


class NoisePredictorFn(torch.autograd.Function):
    """The whole per-point network of NoisePredictor.forward (diffusion_model.py:50-61) under
    autocast, forward and backward, on the fused 16-bit-storage GEMMs (autocast's dtype: float16
    by default, the reference trainer's; "bf16" below stands for it):

      h0 = relu(pts W0^T + b0)             [M,128]  bf16   (pts zero-padded to K = 8)
      h1 = relu(h0 W2^T + b2)              [M,256]  bf16
      x  = ((h1 W4^T + b4) + tf) + sf      [M,256]  fp32 + bf16 copy   (EP_COND, per cloud)
      6 x residual block                   (ResidualBlockFn's kernels)
    With RESIDUAL_16BIT (default) x and its gradient g are stored in the 16-bit format only:
    blocks run EP_BF16 + EP_RESID_DROP16 forward and EP_RELU_MASK + EP_ADD16 backward, and each
    block's Dropout backward is the dropout copy of the epilogue that produced its g.
      q0 = relu(x Wo0^T + bo0)             [M,256]  bf16
      q1 = relu(q0 Wo2^T + bo2)            [M,128]  bf16
      out = q1 Wo4^T + bo4                 [M,3]    fp32

    Inputs: pts [B,N,3], cond [B,2,256] = (time_proj(temb), style_proj(style)) -- the small
    per-cloud projections stay in autograd --, ps = the six residual blocks' dropout rates (each
    block its own, as nn.Dropout per layer does), and the network's 36 weights and biases.  Each ReLU backward
    is fused into the dX product that produces its gradient (EP_RELU_MASK on the layer's own
    bf16 output), so no [M,*] elementwise kernel runs outside the GEMMs except the per-cloud
    column sums of dL/dx for cond's gradient."""

    @staticmethod
    def forward(ctx, pts, cond, ps, *w):
        B, N, _ = pts.shape
        if len(ps) != 6:
            raise ValueError(f"NoisePredictorFn: 6 dropout rates expected, got {len(ps)}")
        M = B * N
        dev = pts.device
        xp = torch.zeros(M, 8, dtype=torch.float32, device=dev)
        xp[:, :3] = pts.reshape(M, 3)
        w0p = torch.zeros(w[0].shape[0], 8, dtype=torch.float32, device=dev)
        w0p[:, :3] = w[0].detach()
        half = autocast_half() or torch.bfloat16
        # every 2-D weight to the 16-bit format in one launch (pcst_cast16_batch)
        mats = [w0p] + [t for t in w[2:] if t.dim() == 2]
        cast = iter(_cast_all(mats, half))
        w0b = next(cast)
        wb = [next(cast) if t.dim() == 2 else t.detach() for t in w[2:]]
        wb = [w0b, w[1].detach()] + wb
        h0 = _hip.gemm_ex(xp, wb[0], wb[1], relu=True, epilogue=_hip.EP_BF16)
        h1 = _hip.gemm_ex(h0, wb[2], wb[3], relu=True, epilogue=_hip.EP_BF16)
        r16 = RESIDUAL_16BIT
        cnd = cond.detach().float().contiguous()
        if r16:
            xb = _hip.gemm_ex(h1, wb[4], wb[5], epilogue=_hip.EP_COND, aux=cnd, group_rows=N,
                              copy_bf16=True, fp32_out=False)
        else:
            x, xb = _hip.gemm_ex(h1, wb[4], wb[5], epilogue=_hip.EP_COND, aux=cnd, group_rows=N,
                                 copy_bf16=True)
        saved, seeds = [xp, h0, h1], []
        hbits = [None] * 6  # the fused blocks' ReLU masks as bits (MASK_BITS), for the backward
        for k in range(6):
            o = 6 + 4 * k
            seed = _draw_seed(ps[k])
            seeds.append(seed)
            saved.append(xb)
            if (r16 and FUSED_BLOCK_FWD and xb.shape[1] == 256 and wb[o].shape == (512, 256)
                    and fused_block_rows_ok(xb.shape[0])):
                if MASK_BITS:
                    h, xb, hbits[k] = _hip.resblock_fwd16(xb, wb[o], wb[o + 1], wb[o + 2], wb[o + 3],
                                                          seed=seed, p=ps[k], mask_bits=True)
                else:
                    h, xb = _hip.resblock_fwd16(xb, wb[o], wb[o + 1], wb[o + 2], wb[o + 3], seed=seed,
                                                p=ps[k])
            elif r16:
                h = _hip.gemm_ex(xb, wb[o], wb[o + 1], relu=True, epilogue=_hip.EP_BF16)
                xb = _hip.gemm_ex(h, wb[o + 2], wb[o + 3], epilogue=_hip.EP_RESID_DROP16, aux=xb,
                                  seed=seed, p=ps[k])
            else:
                x, xb, h = _block_fwd(x, xb, wb[o], wb[o + 1], wb[o + 2], wb[o + 3], ps[k], seed)
            saved.append(h)
        q0 = _hip.gemm_ex(xb, wb[30], wb[31], relu=True, epilogue=_hip.EP_BF16)
        q1 = _hip.gemm_ex(q0, wb[32], wb[33], relu=True, epilogue=_hip.EP_BF16)
        out = _hip.gemm_ex(q1, wb[34], wb[35], epilogue=_hip.EP_F32)
        saved += [xb, q0, q1]
        ctx.save_for_backward(*saved, *w)
        ctx.seeds, ctx.ps, ctx.BN, ctx.half, ctx.r16 = seeds, tuple(ps), (B, N), half, r16
        ctx.hbits = hbits
        return out.view(B, N, 3)

    @staticmethod
    def backward(ctx, gout):
        sv = ctx.saved_tensors
        xp, h0, h1 = sv[0], sv[1], sv[2]
        blocks = [(sv[3 + 2 * k], sv[4 + 2 * k]) for k in range(6)]
        xb, q0, q1 = sv[15], sv[16], sv[17]
        w = sv[18:]
        B, N = ctx.BN
        half = ctx.half
        M = B * N
        dev = gout.device
        grads = [None] * len(w)
        # output layer (O = 3): gradient zero-padded to 8 columns for the MFMA kernels
        g3 = torch.zeros(M, 8, dtype=torch.float32, device=dev)
        g3[:, :3] = gout.reshape(M, 3)
        dw, db = _hip.linear_wgrad_ex(g3, q1)
        grads[34], grads[35] = dw[:3].contiguous(), db[:3].contiguous()
        wo4p = torch.zeros(8, w[34].shape[1], dtype=torch.float32, device=dev)
        wo4p[:3] = w[34].detach()
        # the transposed 16-bit weights of the whole backward in one launch (pcst_cast16_batch)
        tidx = [32, 30] + [i for k in reversed(range(6)) for i in (6 + 4 * k + 2, 6 + 4 * k)] + [4, 2]
        tw = dict(zip(["o4"] + tidx, _cast_all([wo4p] + [w[i] for i in tidx], half, True)))
        dq1 = _hip.gemm_ex(g3, tw["o4"], epilogue=_hip.EP_RELU_MASK, aux=q1)
        grads[32], grads[33] = _hip.linear_wgrad_ex(dq1, q0)
        dq0 = _hip.gemm_ex(dq1, tw[32], epilogue=_hip.EP_RELU_MASK, aux=q0)
        grads[30], grads[31] = _hip.linear_wgrad_ex(dq0, xb)
        if ctx.r16:
            # g and the last block's dD from one epilogue; each block's EP_ADD16 then emits the
            # next (earlier) block's dD beside its g
            g, dd = _hip.gemm_ex(dq0, tw[30], epilogue=_hip.EP_BF16, seed=ctx.seeds[5],
                                 p=ctx.ps[5], dropout_copy=True)
            for k in reversed(range(6)):
                o = 6 + 4 * k
                xbk, hk = blocks[k]
                if (FUSED_BLOCK_BWD and dd.shape[1] == 256 and hk.shape[1] == 512
                        and fused_block_rows_ok(dd.shape[0]) and (hk.shape[0] == dd.shape[0])):
                    w2t, w1t = tw[o + 2], tw[o]
                    grads[o + 2], grads[o + 3] = _hip.linear_wgrad_ex(dd, hk)
                    dz, g, dd = _hip.resblock_bwd16(dd, w2t, w1t, hk, g,
                                                    seed=ctx.seeds[k - 1] if k else 0,
                                                    p=ctx.ps[k - 1] if k else 0.0,
                                                    dropout_copy=k > 0, hbits=ctx.hbits[k])
                    grads[o], grads[o + 1] = _hip.linear_wgrad_ex(dz, xbk)
                    continue
                dz = _hip.gemm_ex(dd, tw[o + 2], epilogue=_hip.EP_RELU_MASK, aux=hk)
                grads[o + 2], grads[o + 3] = _hip.linear_wgrad_ex(dd, hk)
                if k:
                    g, dd = _hip.gemm_ex(dz, tw[o], epilogue=_hip.EP_ADD16, aux=g,
                                         seed=ctx.seeds[k - 1], p=ctx.ps[k - 1], dropout_copy=True)
                else:
                    g = _hip.gemm_ex(dz, tw[o], epilogue=_hip.EP_ADD16, aux=g)
                grads[o], grads[o + 1] = _hip.linear_wgrad_ex(dz, xbk)
        else:
            g = _hip.gemm_ex(dq0, tw[30], epilogue=_hip.EP_F32)
            for k in reversed(range(6)):
                o = 6 + 4 * k
                xbk, hk = blocks[k]
                g, grads[o], grads[o + 1], grads[o + 2], grads[o + 3] = _block_bwd(
                    g, xbk, hk, tw[o], tw[o + 2], ctx.ps[k], ctx.seeds[k])
        # x = ((pf + tf) + sf): dL/dpf = g, dL/dtf[b] = dL/dsf[b] = sum of g over cloud b's rows
        # per-cloud row sums (pcst_group_colsum16: float accumulation, rounded to g's 16-bit
        # type as autocast's sum; replaces a hipBLASLt batched GEMV, ones [B,1,N] @ g [B,N,256])
        gsum = (_hip.group_colsum16(g, B) if g.dtype in (torch.float16, torch.bfloat16)
                else g.view(B, N, -1).sum(1).float())
        dcond = torch.stack([gsum, gsum], 1)
        grads[4], grads[5] = _hip.linear_wgrad_ex(g, h1)
        dh1 = _hip.gemm_ex(g, tw[4], epilogue=_hip.EP_RELU_MASK, aux=h1)
        grads[2], grads[3] = _hip.linear_wgrad_ex(dh1, h0)
        dh0 = _hip.gemm_ex(dh1, tw[2], epilogue=_hip.EP_RELU_MASK, aux=h0)
        dw0, grads[1] = _hip.linear_wgrad_ex(dh0, xp)
        grads[0] = dw0[:, :3].contiguous()
        return (None, dcond, None, *grads)


class BNReLUFn(torch.autograd.Function):
    """relu(BatchNorm_train(z)) over the rows of z [M, O] (BatchNorm2d on [B, C, S, ns] with
    channel-last rows, pointnet2_encoder.py:108-110), optionally max-pooled over groups of
    `pool_ns` rows (:112).  Running statistics are updated on the device."""

    @staticmethod
    def forward(ctx, z, gamma, beta, running_mean, running_var, eps, momentum, pool_ns):
        z2 = z.reshape(-1, z.shape[-1]).float().contiguous()
        M = z2.shape[0]
        if FUSED_BN_STATS:  # statistics and coefficients in two launches (the same bits)
            mean, var, scale, shift, invstd = _hip.bn_train_stats(
                z2, gamma.detach(), beta.detach(), eps, momentum, running_mean, running_var)
        else:
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
    """Train-mode `bn` (BatchNorm2d) + ReLU (+ max-pool) on the HIP kernels.  The reference's
    layers use the default momentum 0.1 (pointnet2_encoder.py:75-78); momentum=None (cumulative
    average, factor 1/num_batches_tracked) reads the counter on the host -- off the fast path.
    The counter is bumped after the forward is queued, so a failing call leaves it and the
    running statistics consistent."""
    momentum = bn.momentum
    if bn.track_running_stats and momentum is None:
        momentum = 1.0 / (float(bn.num_batches_tracked.item()) + 1.0)
    rm = bn.running_mean if bn.track_running_stats else None
    rv = bn.running_var if bn.track_running_stats else None
    y = BNReLUFn.apply(z, bn.weight, bn.bias, rm, rv, bn.eps,
                       0.0 if momentum is None else momentum, pool_ns)
    if bn.track_running_stats:
        bn.num_batches_tracked.add_(1)
    return y


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
