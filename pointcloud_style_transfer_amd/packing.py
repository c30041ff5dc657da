"""Host-side packing of NoisePredictor weights into the streaming layout of
csrc/noise_mlp.hip (done once per weight version, cached on the module).

Blob = sequence of 32 KiB parts; every layer starts on a fresh part.  A part holds
MFMA A-operand fragments, each the exact bytes one wave reads with one 16-B (bf16)
or 4-B (f32) per-lane LDS load:

  bf16 (v_mfma_f32_32x32x16_bf16), fragment (ob, s) = 1 KiB:
     lane l = (r = l & 31, h = l >> 5), element j  ->  W[32 ob + r, k]
     k = 32 (s // 2) + 16 (s % 2) + 8 (j >> 2) + 4 h + (j & 3)
  f32 (v_mfma_f32_32x32x2_f32), fragment (ob, s) = 256 B:
     lane l = (r, h)  ->  W[32 ob + r, k],  k = 32 (s // 16) + (rr & 3) + 8 (rr >> 2) + 4 h,
     rr = s % 16

The k permutation is the row order in which the previous layer's accumulator
registers arrive as this layer's B operand (the C/D map row = (reg & 3) + 8 (reg >> 2)
+ 4 (lane >> 5)), so activations never leave registers between layers.

f32 order (noise_mlp_kernel<TrF32>): point_encoder.2, point_encoder.4, 6 x 16 residual
chunks (W1 rows of the chunk, then W2 columns of the chunk for the 8 output blocks),
output_mlp.0 / .2 / .4.

bf16 order (noise_mlp_pair_kernel, "pair layout"): the same layers, but every part holds the
fragments of BOTH wave roles, role 0 in its first half and role 1 in its second:
  dense layer (NOB output blocks, NS k-steps): part q = [role 0: blocks q*k .. q*k+k-1 |
      role 1: blocks NOB/2 + q*k ..], k = 16 / NS own blocks per role and part;
  residual layer, pair of hidden chunks (it, 8 + it), it = 0..7:
      W1 part = [W1 rows of chunk it | W1 rows of chunk 8 + it]
      W2 part = [for blocks 0-3: k-steps (2it, 2it+1, 2(8+it), 2(8+it)+1) |
                 the same for blocks 4-7];
  output_mlp.4 (one block): one part, read by both roles.

bf16 16x16x32 order (noise_mlp_pair16_kernel, precision code PAIR16 = 2): the pair layout with
16-row fragments.  Fragment (rb, s) = 1 KiB:
     lane l = (r = l & 15, g = l >> 4), element j  ->  W[16 rb + r, k]
     k = 32 s + 16 (j >> 2) + 4 g + (j & 3)
(the operand of k-step s is the accumulators of row blocks 2s, 2s+1: C/D row = 4 g + i).
Parts hold the same weights as the 32x32x16 pair layout, re-cut into 16-row blocks:
  dense layer: part q = [role 0: row blocks q*k .. q*k+k-1 (each all k-steps) | role 1: ...],
      k = 16 / NKS own row blocks per role and part;
  residual W1 part = [row blocks 2it, 2it+1 | row blocks 2(8+it), 2(8+it)+1], all k-steps;
  residual W2 part = [for row blocks 0-7: k-steps (it, 8+it) | the same for row blocks 8-15];
  output_mlp.4: one part, row block 0 (rows 3..15 zero), 4 k-steps.
The residual parts are in the kernel's software-pipelined order: W1(0), then per it = 0..7
W1(it+1) (it < 7) before W2(it) -- the kernel computes the next hidden chunk before the W2
product of the current one, so the partner's chunk exchange and the ReLU/bf16 epilogue sit in
the MFMA shadow of the other part.

bf16 "solo" order (noise_mlp_solo_kernel, precision code SOLO16 = 3): the same 16x16x32 fragments
as a flat stream in consumption order, read by every wave (no roles), cut into 64 KiB superparts
(64 fragments; the kernel's DMA and barrier unit) only at the end (padded to whole superparts):
  point_encoder.2: (row block rb, k-step ks), rb-major        64 fragments
  point_encoder.4: the same                                   128
  residual layer i (512 fragments = 8 superparts), chunk c = hidden rows 32c..32c+31:
      W2(15) of layer i-1 (16 row blocks, k-step 15; zeros for i = 0), W1(0),
      then for k = 1..15: W1(k), W2(k-1)
    where W1(k) = (row block 2k + r, ks) r-major (16 fragments) and W2(k) = row blocks 0..15 at
    k-step k (16 fragments)
  W2(15) of layer 5, output_mlp.0 (128), output_mlp.2 (64), output_mlp.4 (4)
"""
from __future__ import annotations

import numpy as np
import torch

PART = 32768
BF16, F32, PAIR16, SOLO16 = 1, 0, 2, 3
SUPERPART = 65536

# bias table offsets (floats) -- must match csrc/noise_mlp.hip
OFF_W0, OFF_B0, OFF_B2, OFF_B1, OFF_BB2, OFF_O0, OFF_O2, OFF_O4, BIAS_FLOATS = (
    0, 384, 512, 768, 3840, 5376, 5632, 5760, 5792)


def _kmap(precision, nsteps):
    """k index [s, lane, j] (bf16) or [s, lane] (f32) for a K = 32*nblocks input."""
    lanes = np.arange(64)
    h = lanes >> 5
    if precision == BF16:
        s = np.arange(nsteps)[:, None, None]
        j = np.arange(8)[None, None, :]
        return (32 * (s // 2) + 16 * (s % 2) + 8 * (j >> 2) + 4 * h[None, :, None] + (j & 3))
    s = np.arange(nsteps)[:, None]
    rr = s % 16
    return 32 * (s // 16) + (rr & 3) + 8 * (rr >> 2) + 4 * h[None, :]


def _frags(W, precision):
    """W [O, K] float32 (O padded to a multiple of 32) -> [O/32, S, fragment elements]."""
    O, K = W.shape
    ks = 16 if precision == BF16 else 2
    nsteps = K // ks
    km = _kmap(precision, nsteps)
    r = np.arange(64) & 31
    nob = (O + 31) // 32
    Wp = np.zeros((nob * 32, K), np.float32)
    Wp[:O] = W
    out = []
    for ob in range(nob):
        rows = ob * 32 + r  # [64]
        if precision == BF16:
            f = Wp[rows[None, :, None], km]  # [S, 64, 8]
        else:
            f = Wp[rows[None, :], km]  # [S, 64]
        out.append(f.reshape(nsteps, -1))
    return np.stack(out)  # [nob, S, 512 or 64]


def _to_bytes(a, precision):
    t = torch.from_numpy(np.ascontiguousarray(a, np.float32))
    if precision == BF16:
        t = t.to(torch.bfloat16)
    return t.contiguous().view(torch.uint8).numpy().reshape(-1)


def _pad_part(b):
    n = (-len(b)) % PART
    return np.concatenate([b, np.zeros(n, np.uint8)]) if n else b


def pack_blob(sd, precision, pre="noise_predictor"):
    """sd: mapping name -> float32 numpy array (NoisePredictor params).  Returns uint8 array."""
    g = lambda n: np.asarray(sd[f"{pre}.{n}"], np.float32)  # noqa: E731
    if precision == BF16:
        return _pack_pair(g)
    if precision == PAIR16:
        return _pack_pair16(g)
    if precision == SOLO16:
        return _pack_solo16(g)
    parts = []

    def layer(W):
        F = _frags(W, precision)
        parts.append(_pad_part(_to_bytes(F.reshape(-1), precision)))

    layer(g("point_encoder.2.weight"))
    layer(g("point_encoder.4.weight"))
    for i in range(6):
        F1 = _frags(g(f"layers.{i}.0.weight"), precision)  # [16, 256/2, e]
        F2 = _frags(g(f"layers.{i}.2.weight"), precision)  # [8, 512/2, e]
        for c in range(16):
            parts.append(_pad_part(_to_bytes(F1[c].reshape(-1), precision)))
            parts.append(_pad_part(_to_bytes(F2[:, c * 16:(c + 1) * 16].reshape(-1), precision)))
    layer(g("output_mlp.0.weight"))
    layer(g("output_mlp.2.weight"))
    layer(g("output_mlp.4.weight"))
    return np.concatenate(parts)


def _pack_pair(g):
    """bf16 pair layout of noise_mlp_pair_kernel (module docstring)."""
    parts = []
    fpp = PART // 1024

    def emit(frags):  # list of [S, 512] fragment groups in part order
        b = _to_bytes(np.concatenate([f.reshape(-1) for f in frags]), BF16)
        assert len(b) <= PART
        parts.append(_pad_part(b))

    def dense(W):
        F = _frags(W, BF16)                  # [NOB, NS, 512]
        nob, ns = F.shape[:2]
        k = fpp // ns // 2                   # own blocks per role and part
        half = nob // 2
        for q in range(half // k):
            emit([F[q * k:(q + 1) * k], F[half + q * k:half + (q + 1) * k]])

    dense(g("point_encoder.2.weight"))
    dense(g("point_encoder.4.weight"))
    for i in range(6):
        F1 = _frags(g(f"layers.{i}.0.weight"), BF16)  # [16 chunks, 16, 512]
        F2 = _frags(g(f"layers.{i}.2.weight"), BF16)  # [8 blocks, 32, 512]
        for it in range(8):
            emit([F1[it], F1[8 + it]])
            steps = [2 * it, 2 * it + 1, 2 * (8 + it), 2 * (8 + it) + 1]
            emit([F2[0:4][:, steps], F2[4:8][:, steps]])
    dense(g("output_mlp.0.weight"))
    dense(g("output_mlp.2.weight"))
    emit([_frags(g("output_mlp.4.weight"), BF16)])
    return np.concatenate(parts)


def _kmap16(nsteps):
    """k index [s, lane, j] of the 16x16x32 fragments / operands for K = 32*nsteps."""
    g = (np.arange(64) >> 4)[None, :, None]
    s = np.arange(nsteps)[:, None, None]
    j = np.arange(8)[None, None, :]
    return 32 * s + 16 * (j >> 2) + 4 * g + (j & 3)


def _frags16(W):
    """W [O, K] float32 -> [ceil(O/16), K/32, 512] fragments of v_mfma_f32_16x16x32_bf16."""
    O, K = W.shape
    km = _kmap16(K // 32)
    r = np.arange(64) & 15
    nrb = (O + 15) // 16
    Wp = np.zeros((nrb * 16, K), np.float32)
    Wp[:O] = W
    return np.stack([Wp[(rb * 16 + r)[None, :, None], km].reshape(K // 32, -1) for rb in range(nrb)])


def _pack_pair16(g):
    """bf16 16x16x32 pair layout of noise_mlp_pair16_kernel (module docstring)."""
    parts = []
    fpp = PART // 1024

    def emit(frags):
        b = _to_bytes(np.concatenate([f.reshape(-1) for f in frags]), BF16)
        assert len(b) <= PART
        parts.append(_pad_part(b))

    def dense(W):
        F = _frags16(W)                      # [NRB, NKS, 512]
        nrb, nks = F.shape[:2]
        k = fpp // nks // 2                  # own row blocks per role and part
        half = nrb // 2
        for q in range(half // k):
            emit([F[q * k:(q + 1) * k], F[half + q * k:half + (q + 1) * k]])

    dense(g("point_encoder.2.weight"))
    dense(g("point_encoder.4.weight"))
    for i in range(6):
        F1 = _frags16(g(f"layers.{i}.0.weight"))  # [32 row blocks, 8, 512]
        F2 = _frags16(g(f"layers.{i}.2.weight"))  # [16 row blocks, 16, 512]
        w1 = lambda it: emit([F1[2 * it:2 * it + 2], F1[2 * (8 + it):2 * (8 + it) + 2]])  # noqa: E731
        w1(0)
        for it in range(8):
            if it < 7:
                w1(it + 1)
            steps = [it, 8 + it]
            emit([F2[0:8][:, steps], F2[8:16][:, steps]])
    dense(g("output_mlp.0.weight"))
    dense(g("output_mlp.2.weight"))
    emit([_frags16(g("output_mlp.4.weight"))])
    return np.concatenate(parts)


def _pack_solo16(g):
    """bf16 16x16x32 solo stream of noise_mlp_solo_kernel (module docstring)."""
    frags = []

    def dense(W):
        F = _frags16(W)                      # [NRB, NKS, 512]
        frags.extend(F.reshape(-1, 512))     # rb-major, then k-step

    dense(g("point_encoder.2.weight"))
    dense(g("point_encoder.4.weight"))
    prev = np.zeros((16, 16, 512), np.float32)     # "W2 of layer -1": zeros
    for i in range(6):
        F1 = _frags16(g(f"layers.{i}.0.weight"))  # [32 row blocks, 8, 512]
        F2 = _frags16(g(f"layers.{i}.2.weight"))  # [16 row blocks, 16, 512]
        w1 = lambda k: F1[2 * k:2 * k + 2].reshape(-1, 512)  # noqa: E731  (r, ks) r-major
        frags.extend(prev[:, 15])
        frags.extend(w1(0))
        for k in range(1, 16):
            frags.extend(w1(k))
            frags.extend(F2[:, k - 1])
        prev = F2
    frags.extend(prev[:, 15])
    dense(g("output_mlp.0.weight"))
    dense(g("output_mlp.2.weight"))
    dense(g("output_mlp.4.weight"))
    b = _to_bytes(np.stack(frags), BF16)
    n = (-len(b)) % SUPERPART
    return np.concatenate([b, np.zeros(n, np.uint8)]) if n else b


def pack_bias(sd, pre="noise_predictor"):
    g = lambda n: np.asarray(sd[f"{pre}.{n}"], np.float32)  # noqa: E731
    t = np.zeros(BIAS_FLOATS, np.float32)
    t[OFF_W0:OFF_W0 + 384] = g("point_encoder.0.weight").reshape(-1)
    t[OFF_B0:OFF_B0 + 128] = g("point_encoder.0.bias")
    t[OFF_B2:OFF_B2 + 256] = g("point_encoder.2.bias")
    for i in range(6):
        t[OFF_B1 + 512 * i:OFF_B1 + 512 * (i + 1)] = g(f"layers.{i}.0.bias")
        t[OFF_BB2 + 256 * i:OFF_BB2 + 256 * (i + 1)] = g(f"layers.{i}.2.bias")
    t[OFF_O0:OFF_O0 + 256] = g("output_mlp.0.bias")
    t[OFF_O2:OFF_O2 + 128] = g("output_mlp.2.bias")
    t[OFF_O4:OFF_O4 + 3] = g("output_mlp.4.bias")
    return t


def time_freqs(dim=128):
    """TimeEmbedding frequency table exactly as the reference builds it on the CPU
    (diffusion_model.py:18-22): exp(arange(half) * -(ln 1e4 / (half-1))) in fp32."""
    import math

    half = dim // 2
    return torch.exp(torch.arange(half) * -(math.log(10000) / (half - 1))).float()
