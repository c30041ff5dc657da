"""EXPERIMENT (not product code): weight layout of the quad noise-MLP kernel (tools/nm_quad.hip).
`python tools/nm_quad_pack.py` replays that kernel's read schedule over the packed blob and
checks that it recovers every weight (as bf16)."""
from __future__ import annotations

import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from pointcloud_style_transfer_amd.packing import BF16, PART, _frags, _pad_part, _to_bytes  # noqa: E402


def pack_quad(g):
    """bf16 quad layout of noise_mlp_quad_kernel (one wave per SIMD, 64 points per wave, all
    output blocks per wave):
      dense layer: fragments [block][k-step], the layer padded to whole parts;
      residual layer: 16 parts holding two 16-fragment segments each, in the kernel's
        computation order W1(0), W1(1), W2(0), W1(2), W2(1), ..., W1(15), W2(14), W2(15):
        P0 = [W1(0) | W1(1)], Pk = [W2(k-1) | W1(k+1)] (k = 1..14), P15 = [W2(14) | W2(15)],
        W1(c) = the 16 k-steps of hidden chunk c (rows 32c.. of layers.i.0),
        W2(c) = [block 0..7][k-steps 2c, 2c+1] of layers.i.2 (the columns chunk c feeds)."""
    parts = []

    def emit(frags):
        b = _to_bytes(np.concatenate([f.reshape(-1) for f in frags]), BF16)
        assert len(b) <= PART
        parts.append(_pad_part(b))

    def dense(W):
        F = _frags(W, BF16)                  # [NOB, NS, 512]
        b = _to_bytes(F.reshape(-1), BF16)
        parts.extend(np.split(_pad_part(b), max(1, len(_pad_part(b)) // PART)))

    dense(g("point_encoder.2.weight"))
    dense(g("point_encoder.4.weight"))
    for i in range(6):
        F1 = _frags(g(f"layers.{i}.0.weight"), BF16)  # [16 chunks, 16, 512]
        F2 = _frags(g(f"layers.{i}.2.weight"), BF16)  # [8 blocks, 32, 512]
        w1 = lambda c: F1[c]                          # noqa: E731
        w2 = lambda c: F2[:, 2 * c:2 * c + 2]         # noqa: E731
        emit([w1(0), w1(1)])
        for k in range(1, 15):
            emit([w2(k - 1), w1(k + 1)])
        emit([w2(14), w2(15)])
    dense(g("output_mlp.0.weight"))
    dense(g("output_mlp.2.weight"))
    dense(g("output_mlp.4.weight"))
    return np.concatenate(parts)





def check():
    """packing._pack_quad in the layout of noise_mlp_quad_kernel: replaying that kernel's read
    schedule (dense layers [block][k-step] per part; residual parts P0 = [W1(0)|W1(1)],
    Pk = [W2(k-1)|W1(k+1)], P15 = [W2(14)|W2(15)], csrc/noise_mlp.hip run_part) over the blob
    recovers every weight of every layer exactly (as bf16)."""
    import torch

    from pointcloud_style_transfer_amd import packing
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden"))
    from pointcloud_style_transfer_amd.model_spec import state_dict_shapes
    from detweights import deterministic_state

    sd = deterministic_state(state_dict_shapes())
    pre = "noise_predictor"
    g = lambda n: np.asarray(sd[f"{pre}.{n}"], np.float32)  # noqa: E731
    blob = pack_quad(g)
    vals = torch.from_numpy(blob.copy()).view(torch.bfloat16).float().numpy()
    fpe = 512
    parts = vals.reshape(-1, packing.PART // 2)
    km = packing._kmap(packing.BF16, 32)
    r = np.arange(64) & 31
    got = {}
    q = [0]

    def put(name, block, step, f):
        W = got.setdefault(name, {})
        fr = parts[q[0], f * fpe:(f + 1) * fpe].reshape(64, 8)
        for lane in range(64):
            for j in range(8):
                W[(block * 32 + r[lane], int(km[step, lane, j]))] = fr[lane, j]

    def dense(name, nob, ns):
        obpp = 32 // ns
        for ob in range(nob):
            if ob and ob % obpp == 0:
                q[0] += 1
            for s in range(ns):
                put(name, ob, s, (ob % obpp) * ns + s)
        q[0] += 1

    def w1(layer, c, base):
        for i in range(16):
            put(f"layers.{layer}.0", c, i, base + i)

    def w2(layer, c, base):
        for i in range(16):
            put(f"layers.{layer}.2", i // 2, 2 * c + i % 2, base + i)

    dense("point_encoder.2", 8, 8)
    dense("point_encoder.4", 8, 16)
    for layer in range(6):
        w1(layer, 0, 0)
        w1(layer, 1, 16)
        q[0] += 1
        for k in range(1, 15):
            w2(layer, k - 1, 0)
            w1(layer, k + 1, 16)
            q[0] += 1
        w2(layer, 14, 0)
        w2(layer, 15, 16)
        q[0] += 1
    dense("output_mlp.0", 8, 16)
    dense("output_mlp.2", 4, 16)
    dense("output_mlp.4", 1, 8)
    assert q[0] == parts.shape[0]
    for name, W in got.items():
        ref = torch.from_numpy(sd[f"{pre}.{name}.weight"]).bfloat16().float().numpy()
        O, K = ref.shape
        seen = np.full((max(O, 32), K), np.nan, np.float32)
        for (o, k), v in W.items():
            seen[o, k] = v
        np.testing.assert_array_equal(seen[:O], ref, err_msg=name)
        if O < 32:
            assert (seen[O:] == 0).all(), name


if __name__ == "__main__":
    check()
    print("quad layout replay ok")
