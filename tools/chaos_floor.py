"""Chaos floor of the guided sampling loop (VERDICT r2 'gate the measured mode'): the oracle
loop (numpy + C port of /root/reference/models/diffusion_model.py:224-261) run twice on the
same 120k cloud, once from x_T and once from x_T moved by one ulp per element (random
direction), same counter-keyed draws.  Whatever separates those two runs is the loop's own
amplification of a 1-ulp input change -- the floor any implementation's end-to-end distance
from the oracle is measured against.

CPU only (test infrastructure: imports oracle/).  Writes profiles/r03/chaos_floor.json.

    python tools/chaos_floor.py [--steps 10 50] [--weights det|seed0]
    python tools/chaos_floor.py --steps 1000 --base-npz tests/golden/oracle_loop120k_1000.npz \
        --out profiles/r04/chaos_floor.json
(--base-npz: the unperturbed run is the committed oracle output `x_S` of that file -- the same
oracle, inputs and draws -- so only the perturbed run is computed.)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests", "golden"))


def metrics(out, ref):
    """metrics.py:20-44 Chamfer (Euclidean, both directions, /2) + elementwise figures."""
    from scipy.spatial import cKDTree

    a, b = out[0].astype(np.float64), ref[0].astype(np.float64)
    d1 = cKDTree(b).query(a, k=1)[0]
    d2 = cKDTree(a).query(b, k=1)[0]
    d = np.abs(out.astype(np.float64) - ref.astype(np.float64))
    scale = np.abs(ref).max()
    return {"chamfer": float((d1.mean() + d2.mean()) / 2),
            "max_abs": float(d.max()), "mean_abs": float(d.mean()),
            "median_abs": float(np.median(d)),
            "p999_abs": float(np.quantile(d, 0.999)),
            "frac_within_1e-4_rel": float((d <= 1e-4 * (np.abs(ref) + 0.1 * scale)).mean()),
            "frac_within_1e-3_abs": float((d <= 1e-3).mean())}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, nargs="+", default=[10, 50])
    ap.add_argument("--weights", default="det", choices=["det", "seed0"])
    ap.add_argument("--out", default=os.path.join(REPO, "profiles", "r03", "chaos_floor.json"))
    ap.add_argument("--base-npz", default=None)
    args = ap.parse_args()
    from oracle import oracle as O
    from pointcloud_style_transfer_amd import rng
    from pointcloud_style_transfer_amd.model_spec import state_dict_shapes
    from pointcloud_style_transfer_amd.synthetic import lidar_like_cloud, standard_normal

    if args.weights == "det":
        from detweights import deterministic_state

        sd = deterministic_state(state_dict_shapes())
    else:  # bench.py's random init (torch.manual_seed(0) on the module tree)
        import torch

        from pointcloud_style_transfer_amd.config.config import Config
        from pointcloud_style_transfer_amd.models.diffusion_model import PointCloudDiffusionModel

        torch.manual_seed(0)
        m = PointCloudDiffusionModel(Config(make_dirs=False))
        sd = {k: v.detach().float().numpy() for k, v in m.state_dict().items()}
    src = lidar_like_cloud(1000, 120000)[None]
    cond = lidar_like_cloud(2000, 120000)[None]
    xT = standard_normal(3000, (1, 120000, 3))
    g = np.random.default_rng(7)
    up = g.random(xT.shape) < 0.5
    xT_p = np.where(up, np.nextafter(xT, np.float32(np.inf)),
                    np.nextafter(xT, np.float32(-np.inf))).astype(np.float32)
    res = {"what": "oracle guided loop vs itself from x_T moved by 1 ulp per element",
           "cloud": "lidar_like_cloud(1000/2000, 120000), x_T standard_normal(3000)",
           "draws": "rng.CounterRNG(6000) on both runs", "weights": args.weights,
           "guidance_scale": 7.5, "runs": {}}
    if os.path.exists(args.out):
        with open(args.out) as f:
            old = json.load(f)
        if old.get("weights") == args.weights:
            res["runs"] = old.get("runs", {})
    for S in args.steps:
        t0 = time.perf_counter()
        pert = O.guided_loop_counter(sd, src, cond, xT_p, S, rng.CounterRNG(6000))
        if args.base_npz:
            base = np.load(args.base_npz)[f"x_{S}"]
        else:
            base = O.guided_loop_counter(sd, src, cond, xT, S, rng.CounterRNG(6000))
        r = metrics(pert, base)
        r["seconds"] = round(time.perf_counter() - t0, 1)
        res["runs"][str(S)] = r
        print(S, json.dumps(r), flush=True)
        os.makedirs(os.path.dirname(args.out), exist_ok=True)
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
