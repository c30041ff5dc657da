"""Noise-MLP kernel probe (GPU): the bf16 solo kernel (precision 3) against the exact-f32 kernel
and the pair16 kernel (precision 2) on deterministic weights, then per-launch time of both at the
bench launch (2 x 30000 points) and at 32 clouds (64 x 30000).  Prints one JSON line per item."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests", "golden"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from detweights import deterministic_state  # noqa: E402

from pointcloud_style_transfer_amd import _hip, packing  # noqa: E402
from pointcloud_style_transfer_amd.model_spec import state_dict_shapes  # noqa: E402


def main():
    sd = deterministic_state(state_dict_shapes())
    g = lambda n: torch.from_numpy(sd[f"noise_predictor.{n}"]).cuda()  # noqa: E731
    cp = (packing.time_freqs(128).cuda(), g("time_proj.weight").t().contiguous(),
          g("time_proj.bias"), g("style_proj.weight").t().contiguous(), g("style_proj.bias"),
          g("point_encoder.4.bias"))
    bias = torch.from_numpy(packing.pack_bias(sd)).cuda()
    blobs = {p: torch.from_numpy(packing.pack_blob(sd, p)).cuda() for p in (0, 2, 3)}
    rng = np.random.default_rng(5)
    checks = [(30000, 2), (4096, 3), (50, 11), (1, 1), (300, 1)]
    for T, C in checks:
        P = T * C - (7 if T * C > 300 else 0)
        pts = torch.from_numpy(rng.standard_normal((P, 3)).astype(np.float32)).cuda()
        t = torch.from_numpy(rng.integers(0, 1000, C)).cuda()
        style = torch.from_numpy((rng.standard_normal((C, 256)) * 0.3).astype(np.float32)).cuda()
        cond = _hip.noise_cond(t, style, *cp)
        outs = {p: _hip.noise_mlp(pts, T, cond, blobs[p], bias, p).cpu().numpy() for p in (0, 2, 3)}
        f32 = outs[0]
        scale = float(np.abs(f32).max())
        row = {"T": T, "C": C, "P": P}
        for p in (2, 3):
            d = np.abs(outs[p] - f32)
            row[f"p{p}_ok"] = float((d <= 0.05 * (np.abs(f32) + 0.1 * scale)).mean())
            row[f"p{p}_max"] = float(d.max() / scale)
            row[f"p{p}_norm"] = float(np.linalg.norm(outs[p] - f32) / np.linalg.norm(f32))
            row[f"p{p}_finite"] = bool(np.isfinite(outs[p]).all())
        row["p3_vs_p2_norm"] = float(np.linalg.norm(outs[3] - outs[2]) / np.linalg.norm(f32))
        print(json.dumps(row), flush=True)
    for C in (2, 64):
        T = 30000
        P = T * C
        pts = torch.from_numpy(rng.standard_normal((P, 3)).astype(np.float32)).cuda()
        t = torch.full((C,), 999).cuda()
        style = torch.from_numpy((rng.standard_normal((C, 256)) * 0.3).astype(np.float32)).cuda()
        cond = _hip.noise_cond(t, style, *cp)
        out = torch.empty(P, 3, device="cuda")
        for p in (2, 3, 2, 3):
            for _ in range(5):
                _hip.noise_mlp(pts, T, cond, blobs[p], bias, p, out=out)
            n = 40 if C == 2 else 6
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(n):
                _hip.noise_mlp(pts, T, cond, blobs[p], bias, p, out=out)
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / n
            fl = 3540480.0 * P
            print(json.dumps({"precision": p, "clouds": C, "points": P, "ms": round(ms, 4),
                              "tflops": round(fl / ms / 1e9, 1), "frac": round(fl / ms / 1e9 / 2500, 4)}),
                  flush=True)


if __name__ == "__main__":
    main()
