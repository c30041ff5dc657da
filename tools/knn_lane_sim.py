"""Cost model of the kNN-3 lane search (knn.hip lane path) on a synthetic step cloud, on the CPU.

    python tools/knn_lane_sim.py [--rpc 3 4 6] [--cloud noise|aniso] [--rmax 3]

For the upsample of one CFG copy (120k points, 30k coarse rows by the voxel rule with a random pad)
it builds the row-major grid the build kernel would (cell size from the Gaussian peak density and
`rpc` refs per cell), finds each query's smallest cube radius R whose faces lie beyond its true
3rd-NN distance (cKDTree), and prints per-lane and per-wave (64 consecutive queries in cell order)
statistics of the passes: rows visited, refs screened, outliers (R > rmax).  A development tool:
nothing here is product code or a parity check."""
import argparse

import numpy as np
from scipy.spatial import cKDTree


def downsample(x, target, rng):
    mn = x.min(0)
    rg = x.max(0) - mn
    rg[rg < 1e-6] = 1.0
    vs = np.float32((float(np.prod(rg)) / target) ** (1 / 3) * 1.2)
    v = np.floor((x - mn) / vs).astype(np.int64)
    key = (v[:, 0] * 73856093) ^ (v[:, 1] * 19349663) ^ (v[:, 2] * 83492791)
    _, inv = np.unique(key, return_inverse=True)
    s = np.bincount(inv, weights=np.arange(len(x), dtype=np.float64))
    c = np.bincount(inv)
    reps = (s / c).astype(np.int64)
    U = len(reps)
    if U >= target:
        return reps[rng.permutation(U)[:target]]
    mask = np.ones(len(x), bool)
    mask[reps] = False
    pool = np.nonzero(mask)[0]
    return np.concatenate([reps, pool[rng.permutation(len(pool))[:target - U]]])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rpc", type=float, nargs="+", default=[2, 3, 4, 6])
    ap.add_argument("--cloud", default="noise")
    ap.add_argument("--rmax", type=int, default=3)
    ap.add_argument("--seed", type=int, default=0)
    a = ap.parse_args()
    rng = np.random.default_rng(a.seed)
    N, T = 120000, 30000
    x = rng.standard_normal((N, 3)).astype(np.float32)
    if a.cloud == "aniso":
        x *= np.array([1.0, 0.5, 0.2], np.float32)
    idx = downsample(x, T, rng)
    known = np.zeros(N, bool)
    known[idx] = True
    refs = x[idx].astype(np.float64)
    q = x[~known].astype(np.float64)
    d3 = cKDTree(refs).query(q, k=3)[0][:, 2]
    M = len(idx)
    mn, mx = x.min(0).astype(np.float64), x.max(0).astype(np.float64)
    ext = np.maximum(mx - mn, 1e-9)
    sig = x.astype(np.float64).std(0)
    rho = M / (15.7496099457 * np.prod(sig))
    for rpc in a.rpc:
        s = np.cbrt(rpc / rho)
        d = np.minimum(2048, np.maximum(1, np.ceil(ext / s))).astype(np.int64)
        cr = np.clip(np.floor((refs - mn) / s).astype(np.int64), 0, d - 1)
        cq = np.clip(np.floor((q - mn) / s).astype(np.int64), 0, d - 1)
        cnt = np.zeros(d, np.int64)
        np.add.at(cnt, (cr[:, 0], cr[:, 1], cr[:, 2]), 1)
        P = np.zeros(d + 1, np.int64)
        P[1:, 1:, 1:] = cnt.cumsum(0).cumsum(1).cumsum(2)

        def box(lo, hi):  # refs in cells [lo, hi] (inclusive, clamped), vectorised
            lo = np.clip(lo, 0, d - 1)
            hi = np.clip(hi, 0, d - 1) + 1
            t = 0
            for sx in (0, 1):
                for sy in (0, 1):
                    for sz in (0, 1):
                        sg = (-1) ** (3 - sx - sy - sz)
                        t = t + sg * P[(hi if sx else lo)[:, 0], (hi if sy else lo)[:, 1], (hi if sz else lo)[:, 2]]
            return t

        order = np.lexsort((cq[:, 0], cq[:, 1], cq[:, 2]))
        cq, qq, dd = cq[order], q[order], d3[order]
        need = np.full(len(qq), 99)
        rows = np.zeros(len(qq))
        refsc = np.zeros(len(qq))
        for R in range(1, 40):
            lo, hi = cq - R, cq + R
            face = np.full(len(qq), np.inf)
            for c in range(3):
                f_lo = np.where(lo[:, c] > 0, qq[:, c] - (mn[c] + lo[:, c] * s), np.inf)
                f_hi = np.where(hi[:, c] < d[c] - 1, (mn[c] + (hi[:, c] + 1) * s) - qq[:, c], np.inf)
                face = np.minimum(face, np.minimum(f_lo, f_hi))
            open_ = need == 99
            nrow = (np.minimum(hi[:, 1], d[1] - 1) - np.maximum(lo[:, 1], 0) + 1) * \
                   (np.minimum(hi[:, 2], d[2] - 1) - np.maximum(lo[:, 2], 0) + 1)
            rows += np.where(open_, nrow, 0)
            refsc += np.where(open_, box(lo, hi), 0)
            done = open_ & (dd < face)
            need[done] = R
            if not (need == 99).any():
                break
        W = len(qq) // 64
        wr = rows[:W * 64].reshape(W, 64)
        wf = refsc[:W * 64].reshape(W, 64)
        wn = need[:W * 64].reshape(W, 64)
        out = (need > a.rmax).sum()
        print(f"rpc {rpc}: s {s:.4f} dims {d.tolist()} cells {int(np.prod(d))} queries {len(qq)} "
              f"max refs/cell {cnt.max()}")
        print(f"  R needed: " + " ".join(f"{r}:{(need == r).mean():.4f}" for r in range(1, 8)) +
              f"  >rmax({a.rmax}): {out} ({out / len(qq):.4%})")
        print(f"  lane rows mean {rows.mean():.1f} p99 {np.percentile(rows, 99):.0f}  refs mean "
              f"{refsc.mean():.1f} p99 {np.percentile(refsc, 99):.0f}")
        wmr = np.where(wn <= a.rmax, wr, 0).max(1)
        wmf = np.where(wn <= a.rmax, wf, 0).max(1)
        print(f"  wave max rows (R<=rmax): mean {wmr.mean():.1f} max {wmr.max():.0f}; wave max refs: "
              f"mean {wmf.mean():.1f} p99 {np.percentile(wmf, 99):.0f} max {wmf.max():.0f}; "
              f"waves with an outlier {(wn > a.rmax).any(1).sum()} of {W}")


if __name__ == "__main__":
    main()
