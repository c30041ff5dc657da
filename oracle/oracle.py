"""CPU oracle: numpy + C restatement of the reference hot path.

TEST INFRASTRUCTURE ONLY.  Only `tests/`, `__graft_entry__.smoke()` and the
`cpu_baseline` leg of `bench.py` may import this module, and only as the
checker / the timed CPU baseline -- never as the thing measured or shipped.

Each function cites the reference file:line it restates.  The restatement is
pinned against golden vectors produced by the reference itself
(`tests/golden/gen_golden.py`, run in the build container): index outputs must
match bit-for-bit, float outputs within the tolerances stated in the tests.

Random draws are never made here: callers pass the draws (recorded from the
reference, or made by the test) through a `Replay`.
"""
from __future__ import annotations

import ctypes
import math
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle_pcst.so")

_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        P = ctypes.c_void_p
        I = ctypes.c_int64
        L.orc_square_distance.argtypes = [P, P, I, I, I, P]
        L.orc_fps.argtypes = [P, I, I, I, P, P]
        L.orc_ball_query.argtypes = [ctypes.c_double, I, P, P, I, I, I, P]
        L.orc_voxel_reps.argtypes = [P, I, I, P, P, P]
        L.orc_voxel_reps.restype = I
        L.orc_knn_interp.argtypes = [P, P, I, P, I, I, P, P]
        L.orc_chamfer_rowmin.argtypes = [P, I, P, I, P, P]
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def _f32(a):
    return np.ascontiguousarray(a, dtype=np.float32)


class Replay:
    """Feeds recorded random draws back in call order (kind-checked)."""

    def __init__(self, draws):
        self.draws = list(draws)
        self.pos = 0

    @classmethod
    def from_npz(cls, z, prefix):
        names = list(z[f"{prefix}_names"])
        return cls([(str(n), z[f"{prefix}_{i}"]) for i, n in enumerate(names)])

    def next(self, kind):
        name, val = self.draws[self.pos]
        if name != kind:
            raise RuntimeError(f"replay: expected {kind}, recorded {name} at draw {self.pos}")
        self.pos += 1
        return np.asarray(val)


# ------------------------------------------------------------------ pointnet2_encoder.py
def normalize_point_cloud(points, target_range=1.8):
    """`PointCloudPreprocessor.normalize_point_cloud` (data/preprocessing.py:21-38): float64
    centre/scale; the callers cast to float32."""
    c = points.mean(axis=0)
    pc = points - c
    m = np.max(np.abs(pc))
    s = 1.0 if m < 1e-6 else target_range / m
    return pc * s, {"center": c, "scale": s, "method": "isotropic", "target_range": target_range}


def denormalize_point_cloud(points, params):
    """data/preprocessing.py:40-42."""
    return (points / params["scale"]) + params["center"]


def square_distance(src, dst):
    """`square_distance` (pointnet2_encoder.py:8-15)."""
    src, dst = _f32(src), _f32(dst)
    B, S, _ = src.shape
    N = dst.shape[1]
    out = np.empty((B, S, N), np.float32)
    lib().orc_square_distance(_p(src), _p(dst), B, S, N, _p(out))
    return out


def index_points(points, idx):
    """`index_points` (pointnet2_encoder.py:17-28): gather with idx clamped to [0, N-1]."""
    B = points.shape[0]
    idx = np.clip(np.asarray(idx), 0, points.shape[1] - 1)
    bi = np.arange(B).reshape((B,) + (1,) * (idx.ndim - 1))
    return points[bi, idx]


def farthest_point_sample(xyz, npoint, start):
    """`farthest_point_sample` (pointnet2_encoder.py:30-45); `start` = the CPU randint draw."""
    xyz = _f32(xyz)
    B, N, _ = xyz.shape
    st = np.ascontiguousarray(start, dtype=np.int64)
    out = np.empty((B, npoint), np.int64)
    lib().orc_fps(_p(xyz), B, N, npoint, _p(st), _p(out))
    return out


def query_ball_point(radius, nsample, xyz, new_xyz):
    """`query_ball_point` (pointnet2_encoder.py:47-59)."""
    xyz, new_xyz = _f32(xyz), _f32(new_xyz)
    B, N, _ = xyz.shape
    S = new_xyz.shape[1]
    out = np.empty((B, S, nsample), np.int64)
    lib().orc_ball_query(float(radius), nsample, _p(xyz), _p(new_xyz), B, N, S, _p(out))
    return out


def _bn(x, sd, pre, train, eps=1e-5):
    """BatchNorm2d over channel-last x [..., C] (train: biased batch var)."""
    w, b = sd[pre + ".weight"], sd[pre + ".bias"]
    if train:
        axes = tuple(range(x.ndim - 1))
        mean = x.astype(np.float64).mean(axis=axes)
        var = x.astype(np.float64).var(axis=axes)
    else:
        mean, var = sd[pre + ".running_mean"], sd[pre + ".running_var"]
    y = (x - mean.astype(np.float32)) / np.sqrt(var.astype(np.float32) + np.float32(eps))
    return (y * w + b).astype(np.float32)


def _apply_mlp(sd, pre, x, n_layers, train):
    """`SetAbstraction.apply_mlp` (pointnet2_encoder.py:106-112), channel-last."""
    for i in range(n_layers):
        W = sd[f"{pre}.mlp_convs.{i}.weight"][:, :, 0, 0]
        x = x @ W.T + sd[f"{pre}.mlp_convs.{i}.bias"]
        x = np.maximum(_bn(x, sd, f"{pre}.mlp_bns.{i}", train), 0.0)
    return x.max(axis=-2)


SA_SPECS = {  # PointNet2Encoder.__init__ (pointnet2_encoder.py:118-121)
    "sa1": (512, 0.2, 32, False),
    "sa2": (128, 0.4, 64, False),
    "sa3": (None, None, None, True),
}


def set_abstraction(sd, pre, xyz, points, replay, train=False):
    """`SetAbstraction.forward` (pointnet2_encoder.py:78-104). Returns (new_xyz, new_points [B,C,S])."""
    npoint, radius, nsample, group_all = SA_SPECS[pre.split(".")[-1]]
    B, N, _ = xyz.shape
    if group_all:
        g = xyz[:, None] if points is None else np.concatenate([xyz, points], -1)[:, None]
        new_xyz = np.zeros((B, 1, 3), np.float32)
        f = _apply_mlp(sd, pre, g.astype(np.float32), 3, train)  # [B,1,C]
        return new_xyz, f[:, 0, :]  # squeeze(-1) of [B,C,1] (pointnet2_encoder.py:89)
    start = replay.next("randint")
    fidx = farthest_point_sample(xyz, npoint, start)
    new_xyz = index_points(xyz, fidx)
    gidx = query_ball_point(radius, nsample, xyz, new_xyz)
    gx = index_points(xyz, gidx) - new_xyz[:, :, None, :]
    g = gx if points is None else np.concatenate([gx, index_points(points, gidx)], -1)
    f = _apply_mlp(sd, pre, g.astype(np.float32), 3, train)  # [B,S,C]
    return new_xyz, f.transpose(0, 2, 1)


def pointnet2_encoder(sd, xyz, replay, train=False, pre="style_encoder.encoder"):
    """`PointNet2Encoder.forward` (pointnet2_encoder.py:123-131)."""
    l1x, l1p = set_abstraction(sd, pre + ".sa1", xyz, None, replay, train)
    l2x, l2p = set_abstraction(sd, pre + ".sa2", l1x, l1p.transpose(0, 2, 1), replay, train)
    _, l3 = set_abstraction(sd, pre + ".sa3", l2x, l2p.transpose(0, 2, 1), replay, train)
    return l3.reshape(xyz.shape[0], -1)


def _linear(sd, pre, x):
    return (x @ sd[pre + ".weight"].T + sd[pre + ".bias"]).astype(np.float32)


def style_encoder(sd, xyz, replay, train=False):
    """`StyleEncoder.forward` (diffusion_model.py:28-36); dropout inactive."""
    f = pointnet2_encoder(sd, xyz, replay, train)
    h = np.maximum(_linear(sd, "style_encoder.style_mlp.0", f), 0.0)
    return np.maximum(_linear(sd, "style_encoder.style_mlp.3", h), 0.0)


# ------------------------------------------------------------------ diffusion_model.py
def time_embedding(t, dim):
    """`TimeEmbedding.forward` (diffusion_model.py:15-26)."""
    half = dim // 2
    # The frequency table is evaluated with torch's own CPU exp: t*f reaches ~1e3 rad,
    # where one ulp of f (numpy expf vs torch's vectorised expf) moves sin by 3e-5.
    import torch

    c = math.log(10000) / (half - 1)
    freqs = torch.exp(torch.arange(half) * -c).numpy()
    e = np.asarray(t).astype(np.float32)[:, None] * freqs[None, :]
    return np.concatenate([np.sin(e), np.cos(e)], -1).astype(np.float32)


def noise_predictor(sd, x, t, style, dim_t=128, pre="noise_predictor"):
    """`NoisePredictor.forward` (diffusion_model.py:54-61); dropout inactive."""
    h = np.maximum(_linear(sd, pre + ".point_encoder.0", x), 0)
    h = np.maximum(_linear(sd, pre + ".point_encoder.2", h), 0)
    pf = _linear(sd, pre + ".point_encoder.4", h)
    tf = _linear(sd, pre + ".time_proj", time_embedding(t, dim_t))[:, None]
    sf = _linear(sd, pre + ".style_proj", style)[:, None]
    x = (pf + tf + sf).astype(np.float32)
    for i in range(6):
        hh = np.maximum(_linear(sd, f"{pre}.layers.{i}.0", x), 0)
        x = (_linear(sd, f"{pre}.layers.{i}.2", hh) + x).astype(np.float32)
    h = np.maximum(_linear(sd, pre + ".output_mlp.0", x), 0)
    h = np.maximum(_linear(sd, pre + ".output_mlp.2", h), 0)
    return _linear(sd, pre + ".output_mlp.4", h)


def voxel_downsample(points, target, replay):
    """`HierarchicalProcessor._voxel_grid_downsample_torch` (diffusion_model.py:69-122)."""
    points = _f32(points)
    B, N, _ = points.shape
    if N <= target:
        return points, np.broadcast_to(np.arange(N), (B, N))
    outs, idxs = [], []
    for b in range(B):
        pts = np.ascontiguousarray(points[b])
        reps = np.empty(N, np.int64)
        U = lib().orc_voxel_reps(_p(pts), N, target, _p(reps), None, None)
        reps = reps[:U]
        if U > target:
            final = reps[replay.next("randperm")[:target]]
        elif U < target:
            mask = np.ones(N, bool)
            mask[reps] = False
            pool = np.nonzero(mask)[0]
            if len(pool) > 0:
                perm = replay.next("randperm")
                final = np.concatenate([reps, pool[perm[:min(target - U, len(pool))]]])
            else:
                final = reps
        else:
            final = reps
        outs.append(pts[final])
        idxs.append(final)
    return np.stack(outs), np.stack(idxs)


def voxel_reps(points, target):
    """Unique-voxel representatives of ONE cloud, ascending-hash order (diffusion_model.py:78-97)."""
    pts = _f32(points)
    N = pts.shape[0]
    reps = np.empty(N, np.int64)
    hashes = np.empty(N, np.int32)
    vs = np.empty(1, np.float32)
    U = lib().orc_voxel_reps(_p(pts), N, target, _p(reps), _p(hashes), _p(vs))
    return reps[:U], hashes, float(vs[0])


def upsample_knn(coarse, orig, idx):
    """`HierarchicalProcessor.upsample_knn` (diffusion_model.py:127-153), float64 exact 3-NN."""
    coarse, orig = _f32(coarse), _f32(orig)
    B, N, _ = orig.shape
    outs = []
    for b in range(B):
        ib = np.asarray(idx[b])
        valid = ib[ib < N]
        vc = np.ascontiguousarray(coarse[b][: len(valid)])
        res = np.zeros_like(orig[b])
        res[valid] = vc
        unknown_mask = np.ones(N, bool)
        unknown_mask[valid] = False
        unknown = np.nonzero(unknown_mask)[0]
        if len(unknown) > 0 and len(valid) > 0:
            k = min(3, len(valid))
            refs = np.ascontiguousarray(orig[b][valid])
            qs = np.ascontiguousarray(orig[b][unknown])
            out = np.empty((len(unknown), 3), np.float32)
            lib().orc_knn_interp(_p(refs), _p(vc), len(valid), _p(qs), len(unknown), k,
                                 _p(out), None)
            res[unknown] = out
        outs.append(res)
    return np.stack(outs)


def beta_schedule(num_timesteps=1000, name="cosine", offset=0.0008):
    """`DiffusionProcess._get_beta_schedule` (diffusion_model.py:204-211), float32."""
    if name == "cosine":
        x = np.linspace(0, num_timesteps, num_timesteps + 1, dtype=np.float32)
        ac = np.cos(((x / np.float32(num_timesteps)) + np.float32(0.008) + np.float32(offset))
                    / np.float32(1.008) * np.float32(math.pi) * np.float32(0.5)) ** 2
        ac = (ac / ac[0]).astype(np.float32)
        return np.clip(1 - (ac[1:] / ac[:-1]), 0.0001, 0.9999).astype(np.float32)
    if name == "linear":
        return np.linspace(0.0001, 0.02, num_timesteps, dtype=np.float32)
    raise NotImplementedError(name)


class Schedule:
    """`DiffusionProcess.__init__` tables (diffusion_model.py:194-202)."""

    def __init__(self, num_timesteps=1000, name="cosine", offset=0.0008):
        self.num_timesteps = num_timesteps
        self.betas = beta_schedule(num_timesteps, name, offset)
        self.alphas_cumprod = np.cumprod((1.0 - self.betas).astype(np.float32), dtype=np.float32)
        self.sqrt_ac = np.sqrt(self.alphas_cumprod)
        self.sqrt_1mac = np.sqrt(np.float32(1.0) - self.alphas_cumprod)

    def q_sample(self, x0, t, noise):
        """`DiffusionProcess.q_sample` (diffusion_model.py:213-218)."""
        t = np.clip(np.asarray(t), 0, self.num_timesteps - 1)
        return (self.sqrt_ac[t].reshape(-1, 1, 1) * x0
                + self.sqrt_1mac[t].reshape(-1, 1, 1) * noise).astype(np.float32)


def timesteps_for(num_timesteps, steps):
    """`torch.linspace(T-1, 0, n).long()` (diffusion_model.py:235)."""
    return np.linspace(num_timesteps - 1, 0, steps, dtype=np.float32).astype(np.int64)


def guided_update(sched, x, eps_c, eps_u, source, t, t_prev, scale):
    """CFG + DDIM update of `guided_sample_loop` (diffusion_model.py:248-260)."""
    eps = eps_u + np.float32(scale) * (eps_c - eps_u)
    a_t = sched.alphas_cumprod[t]
    a_prev = sched.alphas_cumprod[t_prev] if t_prev >= 0 else np.float32(1.0)
    x0 = (x - np.sqrt(np.float32(1.0) - a_t) * eps) / (np.sqrt(a_t) + np.float32(1e-8))
    x0 = x0 + np.float32(0.1) * (source - x0)
    x0 = np.tanh(x0 / np.float32(1.8)) * np.float32(1.8)
    return (np.sqrt(a_prev) * x0 + np.sqrt(np.float32(1.0) - a_prev) * eps).astype(np.float32)


def guided_sample_loop(sd, source, cond, steps, scale, replay, global_points=30000,
                       num_timesteps=1000, sched=None):
    """`DiffusionProcess.guided_sample_loop` (diffusion_model.py:224-261)."""
    sched = sched or Schedule(num_timesteps)
    B = source.shape[0]
    cdown, _ = voxel_downsample(cond, global_points, replay)
    style = style_encoder(sd, cdown, replay)
    style_in = np.concatenate([style, np.zeros_like(style)])
    x = replay.next("randn").astype(np.float32)
    ts = timesteps_for(num_timesteps, steps)
    for i, t in enumerate(ts):
        x_in = np.concatenate([x, x])
        t_in = np.full(2 * B, t, np.int64)
        xc, xi = voxel_downsample(x_in, global_points, replay)
        nc = noise_predictor(sd, xc, t_in, style_in)
        eps_both = upsample_knn(nc, x_in, xi) if x_in.shape[1] > global_points else nc
        t_prev = ts[i + 1] if t > 0 else -1
        x = guided_update(sched, x, eps_both[:B], eps_both[B:], source, t, t_prev, scale)
    return x


def guided_step_given(sd, sched, x, source, style_in, t, t_prev, xi, scale=7.5):
    """One step of `guided_sample_loop` (diffusion_model.py:240-260) on ONE cloud x [1,N,3] with
    the CFG rows' subset indices given (xi [2,T], e.g. the product's own device-drawn subset):
    xc = x_in[b][xi[b]], eps = upsample_knn(noise_predictor(xc)), then the CFG + DDIM update.
    The subset is checked by the caller (voxel_reps); everything after it is the reference's."""
    x_in = np.concatenate([_f32(x), _f32(x)])
    xi = np.asarray(xi)
    xc = np.stack([x_in[b][xi[b]] for b in range(2)])
    eps = upsample_knn(noise_predictor(sd, xc, np.full(2, t), style_in), x_in, xi)
    return guided_update(sched, _f32(x), eps[:1], eps[1:], source, int(t), int(t_prev), scale)


def guided_loop_counter(sd, source, cond, x_T, steps, ctr, scale=7.5, global_points=30000,
                        num_timesteps=1000):
    """`guided_sample_loop` (diffusion_model.py:224-261) on ONE cloud with the draws of a
    counter-keyed generator `ctr` (`rng.CounterRNG`: the k-th draw comes from PCG64 seeded with
    (seed, k)), made in the order the product loop makes them under `rng.replay(ctr)`: the
    condition cloud's voxel permutation, the two FPS starts (SA1, SA2), then per step one
    permutation per CFG row.  x_T is passed in (the product's keyword-only `x_T=`)."""
    T = global_points
    sched = Schedule(num_timesteps)

    def down(rows):
        outs, idxs = [], []
        for b in range(rows.shape[0]):
            reps = voxel_reps(rows[b], T)[0]
            U = len(reps)   # reps may repeat an index (two voxels with the same mean index)
            n = U if U > T else (rows.shape[1] - len(np.unique(reps)) if U < T else 0)
            draws = [("randperm", ctr.generator().permutation(n))] if n else []
            p, ix = voxel_downsample(rows[b:b + 1], T, Replay(draws))
            outs.append(p[0])
            idxs.append(ix[0])
        return np.stack(outs), np.stack(idxs)

    cdown, _ = down(_f32(cond))
    starts = [("randint", ctr.generator().integers(0, cdown.shape[1], (1,), dtype=np.int64)),
              ("randint", ctr.generator().integers(0, 512, (1,), dtype=np.int64))]
    style = style_encoder(sd, cdown, Replay(starts))
    style_in = np.concatenate([style, np.zeros_like(style)])
    ts = timesteps_for(num_timesteps, steps)
    x = _f32(x_T).copy()
    for i, t in enumerate(ts):
        x_in = np.concatenate([x, x])
        xc, xi = down(x_in)
        eps = upsample_knn(noise_predictor(sd, xc, np.full(2, t), style_in), x_in, xi)
        x = guided_update(sched, x, eps[:1], eps[1:], source, int(t),
                          int(ts[i + 1]) if t > 0 else -1, scale)
    return x


# ------------------------------------------------------------------ losses.py
def chamfer_rowmin(P, Q):
    P, Q = _f32(P), _f32(Q)
    mind = np.empty(len(P), np.float32)
    arg = np.empty(len(P), np.int64)
    lib().orc_chamfer_rowmin(_p(P), len(P), _p(Q), len(Q), _p(mind), _p(arg))
    return mind, arg


def chamfer_distance(pred, target):
    """`chamfer_distance_chunked_optimized` (losses.py:8-63) -> [B] (float64 means)."""
    out = []
    for b in range(pred.shape[0]):
        m1, _ = chamfer_rowmin(pred[b], target[b])
        m2, _ = chamfer_rowmin(target[b], pred[b])
        out.append(m1.astype(np.float64).mean() + m2.astype(np.float64).mean())
    return np.array(out)


def chamfer_grad(pred, target):
    """d(sum_b chamfer_b)/d(pred, target): autograd of losses.py:24-61 written out."""
    gp = np.zeros(pred.shape, np.float64)
    gt = np.zeros(target.shape, np.float64)
    for b in range(pred.shape[0]):
        P, Q = pred[b].astype(np.float64), target[b].astype(np.float64)
        N, M = len(P), len(Q)
        m1, a1 = chamfer_rowmin(pred[b], target[b])
        live = raw_d(pred[b], target[b], a1) >= 0
        g = 2.0 * (P - Q[a1]) / N * live[:, None]
        gp[b] += g
        np.add.at(gt[b], a1, -g)
        m2, a2 = chamfer_rowmin(target[b], pred[b])
        live = raw_d(target[b], pred[b], a2) >= 0
        g = 2.0 * (Q - P[a2]) / M * live[:, None]
        gt[b] += g
        np.add.at(gp[b], a2, -g)
    return gp, gt


def raw_d(P, Q, arg):
    P, Q = _f32(P), _f32(Q)[arg]
    n1 = (P[:, 0] * P[:, 0] + P[:, 1] * P[:, 1]) + P[:, 2] * P[:, 2]
    n2 = (Q[:, 0] * Q[:, 0] + Q[:, 1] * Q[:, 1]) + Q[:, 2] * Q[:, 2]
    dot = (P.astype(np.float64) * Q).sum(-1).astype(np.float32)
    return (n1 + n2) + np.float32(-2.0) * dot


def diffusion_loss(pred_noise, actual_noise, pred_pts=None, tgt_pts=None,
                   noise_weight=1.0, chamfer_weight=0.1):
    """`DiffusionLoss.forward` (losses.py:81-104) -> (total, dict)."""
    nl = float(np.abs(pred_noise.astype(np.float64) - actual_noise).mean())
    d = {"noise_loss": nl}
    total = noise_weight * nl
    if chamfer_weight > 0 and pred_pts is not None and tgt_pts is not None:
        cl = float(chamfer_distance(pred_pts, tgt_pts).mean())
        total += chamfer_weight * cl
        d["chamfer_loss"] = cl
    d["total_loss"] = total
    return total, d


# ----------------------------------------------------------------------------- metrics
def knn_dist(P, Q, k=1):
    """Brute-force float64 Euclidean distances of the k nearest rows of Q for every row of P
    (ties to the lower index), as sklearn NearestNeighbors / cKDTree / scipy cdist compute them
    from fp32 inputs (evaluation/metrics.py:124-127,146-148; compare.py:22-34).  [B,N,k]."""
    P = np.asarray(P, np.float64)
    Q = np.asarray(Q, np.float64)
    out = np.empty(P.shape[:2] + (k,))
    for b in range(P.shape[0]):
        for s in range(0, P.shape[1], 512):
            d = P[b, s:s + 512, None, :] - Q[b, None, :, :]
            d = np.sqrt((d[..., 0] * d[..., 0] + d[..., 1] * d[..., 1]) + d[..., 2] * d[..., 2])
            o = np.argsort(d, axis=1, kind="stable")[:, :k]
            out[b, s:s + 512] = np.take_along_axis(d, o, axis=1)
    return out


def metric_chamfer(pred, target, bidirectional=True):
    """evaluation/metrics.py:20-44 (exact distances; the reference's cdist is fp32)."""
    a = knn_dist(pred, target)[..., 0].mean(1)
    if not bidirectional:
        return a
    return (a + knn_dist(target, pred)[..., 0].mean(1)) / 2


def metric_hausdorff(pred, target):
    """evaluation/metrics.py:92-107."""
    return np.maximum(knn_dist(pred, target)[..., 0].max(1), knn_dist(target, pred)[..., 0].max(1))


def metric_coverage(pred, target, threshold=0.01):
    """evaluation/metrics.py:109-135."""
    return float(np.mean((knn_dist(target, pred)[..., 0] < threshold).mean(1)))


def metric_uniformity(points, k=8):
    """evaluation/metrics.py:137-173."""
    md = knn_dist(points, points, k + 1)[..., 1:].mean(2)
    sc = [1.0 / (1.0 + s / m) if m > 0 else 0.0 for s, m in zip(md.std(1), md.mean(1))]
    return float(np.mean(sc))


def emd_greedy(pred, target):
    """evaluation/metrics.py:46-90: greedy matching in pred order, scipy cdist distances,
    strict < over ascending j; total summed in order, / N, cast to float32."""
    out = []
    for b in range(pred.shape[0]):
        p = np.asarray(pred[b], np.float64)
        q = np.asarray(target[b], np.float64)
        d = p[:, None, :] - q[None, :, :]
        D = np.sqrt((d[..., 0] * d[..., 0] + d[..., 1] * d[..., 1]) + d[..., 2] * d[..., 2])
        used = np.zeros(len(q), bool)
        total = 0.0
        for i in range(len(p)):
            row = np.where(used, np.inf, D[i])
            j = int(np.argmin(row))   # first index of the minimum
            total += float(row[j])
            used[j] = True
        out.append(total / len(p))
    return np.array(out, dtype=np.float32)


def similarity(pcd1, pcd2, threshold):
    """compare.py:6-43 -> (precision %, recall %, F1)."""
    prec = np.mean(knn_dist(pcd2[None], pcd1[None])[0, :, 0] < threshold)
    rec = np.mean(knn_dist(pcd1[None], pcd2[None])[0, :, 0] < threshold)
    f = 0.0 if prec + rec == 0 else 2 * (prec * rec) / (prec + rec)
    return prec * 100, rec * 100, f


# ----------------------------------------------------------------------------- offline preprocessing
def voxel_center_reps(points, target_size):
    """data/preprocessing.py:56-93: voxel representatives (point nearest the voxel centre,
    first index on ties) in first-appearance voxel order; float32 grid math, float64 norms."""
    points = np.asarray(points, np.float32)
    mn = points.min(axis=0)
    rng_ = points.max(axis=0) - mn
    rng_[rng_ < 1e-6] = 1.0
    vs = (rng_.prod() / target_size) ** (1 / 3) * 1.2
    if vs < 1e-6:
        vs = np.float32(1e-3)
    vox = np.floor((points - mn) / vs).astype(np.int64)
    ctr = mn.astype(np.float64) + (vox + 0.5) * np.float64(vs)
    d = points.astype(np.float64) - ctr
    dist = np.sqrt((d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1]) + d[:, 2] * d[:, 2])
    key = (vox[:, 0] << 42) | (vox[:, 1] << 21) | vox[:, 2]
    o = np.lexsort((np.arange(len(points)), dist, key))
    ks = key[o]
    head = np.ones(len(o), bool)
    head[1:] = ks[1:] != ks[:-1]
    reps = o[head]
    _, first = np.unique(key, return_index=True)   # first index per voxel, sorted by key
    return reps[np.argsort(first, kind="stable")]
