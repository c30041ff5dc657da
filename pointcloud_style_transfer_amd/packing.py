"""Host-side packing of NoisePredictor weights into the streaming layouts of
csrc/noise_mlp.hip (done once per weight version, cached on the module).  Every MFMA A-operand
fragment is laid out as the exact bytes one wave reads with one per-lane LDS load, in the order
the kernel consumes them.

f32 (precision code F32 = 0, noise_mlp_kernel<TrF32>, v_mfma_f32_32x32x2_f32): a sequence of
32 KiB parts, every layer starting on a fresh part.  Fragment (ob, s) = 256 B:
     lane l = (r = l & 31, h = l >> 5)  ->  W[32 ob + r, k],  k = 32 (s // 16) + (rr & 3) + 8 (rr >> 2)
     + 4 h, rr = s % 16
The k permutation is the row order in which the previous layer's accumulator registers arrive as
this layer's B operand (the C/D map row = (reg & 3) + 8 (reg >> 2) + 4 (lane >> 5)), so
activations never leave registers between layers.  Order: point_encoder.2, point_encoder.4, 6 x 16
residual chunks (W1 rows of the chunk, then W2 columns of the chunk for the 8 output blocks, each
its own part), output_mlp.0 / .2 / .4.

bf16 (precision code BF16 = 1, solo::noise_mlp_solo_kernel, v_mfma_f32_16x16x32_bf16): 16-row
fragments, (rb, s) = 1 KiB:
     lane l = (r = l & 15, g = l >> 4), element j  ->  W[16 rb + r, k],
     k = 32 s + 16 (j >> 2) + 4 g + (j & 3)
(the operand of k-step s is the accumulators of row blocks 2s, 2s+1: C/D row = 4 g + i), as a
flat stream in consumption order, read by every wave, cut into 64 KiB superparts (64 fragments;
the kernel's DMA and barrier unit) only at the end (padded to whole superparts):
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
F32, BF16 = 0, 1
SUPERPART = 65536

# bias table offsets (floats) -- must match csrc/noise_mlp.hip
OFF_W0, OFF_B0, OFF_B2, OFF_B1, OFF_BB2, OFF_O0, OFF_O2, OFF_O4, BIAS_FLOATS = (
    0, 384, 512, 768, 3840, 5376, 5632, 5760, 5792)


def _kmap(nsteps):
    """f32 k index [s, lane] for a K = 32 * (nsteps / 16) input."""
    h = np.arange(64) >> 5
    s = np.arange(nsteps)[:, None]
    rr = s % 16
    return 32 * (s // 16) + (rr & 3) + 8 * (rr >> 2) + 4 * h[None, :]


def _frags(W):
    """f32: W [O, K] (O padded to a multiple of 32) -> [O/32, K/2, 64] fragments."""
    O, K = W.shape
    nsteps = K // 2
    km = _kmap(nsteps)
    r = np.arange(64) & 31
    nob = (O + 31) // 32
    Wp = np.zeros((nob * 32, K), np.float32)
    Wp[:O] = W
    return np.stack([Wp[(ob * 32 + r)[None, :], km].reshape(nsteps, -1) for ob in range(nob)])


def _to_bytes(a, precision):
    t = torch.from_numpy(np.ascontiguousarray(a, np.float32))
    if precision == BF16:
        t = t.to(torch.bfloat16)
    return t.contiguous().view(torch.uint8).numpy().reshape(-1)


def _pad_part(b):
    n = (-len(b)) % PART
    return np.concatenate([b, np.zeros(n, np.uint8)]) if n else b


def pack_blob(sd, precision, pre="noise_predictor"):
    """sd: mapping name -> float32 numpy array (NoisePredictor params); precision F32 or BF16.
    Returns the uint8 blob of pcst_noise_mlp_blob_bytes(precision) bytes."""
    g = lambda n: np.asarray(sd[f"{pre}.{n}"], np.float32)  # noqa: E731
    if precision == BF16:
        return _pack_solo16(g)
    if precision != F32:
        raise ValueError(f"pack_blob: precision must be F32 (0) or BF16 (1), got {precision}")
    parts = []

    def layer(W):
        parts.append(_pad_part(_to_bytes(_frags(W).reshape(-1), F32)))

    layer(g("point_encoder.2.weight"))
    layer(g("point_encoder.4.weight"))
    for i in range(6):
        F1 = _frags(g(f"layers.{i}.0.weight"))  # [16, 128, 64]
        F2 = _frags(g(f"layers.{i}.2.weight"))  # [8, 256, 64]
        for c in range(16):
            parts.append(_pad_part(_to_bytes(F1[c].reshape(-1), F32)))
            parts.append(_pad_part(_to_bytes(F2[:, c * 16:(c + 1) * 16].reshape(-1), F32)))
    layer(g("output_mlp.0.weight"))
    layer(g("output_mlp.2.weight"))
    layer(g("output_mlp.4.weight"))
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


def _pack_solo16(g):
    """bf16 16x16x32 stream of noise_mlp_solo_kernel (module docstring)."""
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
