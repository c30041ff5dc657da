"""HIP kernels of the guided denoising step vs reference golden vectors and the oracle:
voxel downsample (bit-exact with replayed permutations), kNN-3 IDW upsample (bit-exact),
fused noise MLP (fp32 mode within 1e-4 rel; bf16 mode within the bf16 tolerance below),
CFG/DDIM update."""
import numpy as np
import pytest
import torch

from conftest import assert_close
from oracle import oracle as O

pytestmark = pytest.mark.gpu

# bf16 operands with fp32 accumulation through 17 chained layers: normwise relative error
# of the predicted noise vs the fp32 reference (stated tolerance of the perf path).
BF16_NORM_RTOL = 3e-2


@pytest.fixture(scope="module")
def H():
    from pointcloud_style_transfer_amd import _hip

    assert torch.cuda.is_available()
    _hip.lib()
    return _hip


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def provider_from(draws):
    it = iter(draws)

    def p(b, n):
        v = next(it)
        assert len(v) == n, (len(v), n)
        return torch.from_numpy(np.asarray(v, np.int64))
    return p


@pytest.mark.parametrize("key", ["pad", "sub"])
def test_voxel_golden(H, golden, key):
    g = golden("hierarchical.npz")
    names = list(g[f"{key}_rng_names"])
    draws = [g[f"{key}_rng_{i}"] for i in range(len(names))]
    pts, idx = H.voxel_downsample(dev(g[f"{key}_pts"]), int(g[f"{key}_target"]),
                                  perm_provider=provider_from(draws))
    np.testing.assert_array_equal(idx.cpu().numpy(), g[f"{key}_idx"])
    np.testing.assert_array_equal(pts.cpu().numpy(), g[f"{key}_down"])


def test_voxel_golden_120k(H, golden):
    from pointcloud_style_transfer_amd.synthetic import lidar_like_cloud

    g = golden("hierarchical.npz")
    pts = lidar_like_cloud(int(g["full_seed"]), 120000)[None]
    _, idx = H.voxel_downsample(dev(pts), 30000, perm_provider=provider_from([g["full_perm"]]))
    np.testing.assert_array_equal(idx.cpu().numpy(), g["full_idx"].astype(np.int64))


@pytest.mark.parametrize("N,T,B,sig", [(5000, 1000, 3, (1, 1, 0.15)), (20000, 3000, 2, (1, 1, 1e-3)),
                                        (70000, 30000, 2, (1, 1, 0.15)), (9000, 8000, 1, (1, 1, 1)),
                                        (300, 250, 2, (1, 1, 1)), (1025, 1000, 1, (1, 1, 1)),
                                        (3000, 2999, 1, (1, 1, 1))])
def test_voxel_vs_oracle_random_perm(H, N, T, B, sig):
    """Reps/pool bit-exact vs the oracle; the device-drawn subset is a valid draw."""
    rng = np.random.default_rng(N)
    pts = (rng.standard_normal((B, N, 3)) * np.array(sig)).astype(np.float32)
    U, P = H.voxel_stats(dev(pts), T)
    for b in range(B):
        reps, _, _ = O.voxel_reps(pts[b], T)
        assert int(U[b]) == len(reps)
        assert int(P[b]) == N - len(np.unique(reps))
    # replay random permutations drawn here -> bit-exact vs the oracle
    perms = []
    for b in range(B):
        n = int(U[b]) if int(U[b]) > T else (int(P[b]) if int(U[b]) < T else 0)
        if n:
            perms.append(rng.permutation(n))
    _, idx = H.voxel_downsample(dev(pts), T, perm_provider=provider_from(perms))
    _, ref = O.voxel_downsample(pts, T, O.Replay([("randperm", p) for p in perms]))
    np.testing.assert_array_equal(idx.cpu().numpy(), ref)
    # device-drawn subset (perf path): rows in ascending point-index order, bit-identical for
    # a seed; in the pad branch the reps multiset is kept whole and the rest is a duplicate-free
    # draw from the pool; in the subsample branch a sub-multiset of the reps
    pts_d, idx2 = H.voxel_downsample(dev(pts), T, seed=1234)
    idx2 = idx2.cpu().numpy()
    np.testing.assert_array_equal(pts_d.cpu().numpy(), np.stack([pts[b][idx2[b]] for b in range(B)]))
    _, idx3 = H.voxel_downsample(dev(pts), T, seed=1234)
    np.testing.assert_array_equal(idx2, idx3.cpu().numpy())  # deterministic, order included
    assert (np.diff(idx2, axis=1) >= 0).all()
    for b in range(B):
        reps, _, _ = O.voxel_reps(pts[b], T)
        U = len(reps)
        vals, cnt = np.unique(idx2[b], return_counts=True)
        rv, rc = np.unique(reps, return_counts=True)
        if U < T:
            have = dict(zip(vals.tolist(), cnt.tolist()))
            assert all(have.get(v, 0) == k for v, k in zip(rv.tolist(), rc.tolist()))
            extra = ~np.isin(vals, rv)
            assert extra.sum() == T - U and (cnt[extra] == 1).all()
        else:
            assert np.isin(idx2[b], reps).all()
            # T distinct list positions: the kept multiset is a sub-multiset of reps
            assert (cnt <= rc[np.searchsorted(rv, vals)]).all()


@pytest.mark.parametrize("N,T,B,copies,sig", [(120000, 30000, 1, 2, (1, 1, 1)),
                                               (9000, 8000, 2, 3, (1, 1, 1)),
                                               (20000, 3000, 2, 2, (1, 1, 1e-3))])
def test_voxel_copies_matches_concat(H, N, T, B, copies, sig):
    """downsample of cat([x] * copies) from the distinct clouds: per row the same kept set (and
    the same points) as the concatenated call with the same seed."""
    rng = np.random.default_rng(N + copies)
    pts = (rng.standard_normal((B, N, 3)) * np.array(sig)).astype(np.float32)
    x = dev(pts)
    p1, i1 = H.voxel_downsample(torch.cat([x] * copies), T, seed=77)
    p2, i2 = H.voxel_downsample(x, T, seed=77, copies=copies)
    i1, i2 = i1.cpu().numpy(), i2.cpu().numpy()
    assert i2.shape == (copies * B, T)
    np.testing.assert_array_equal(i1, i2)  # same rows, order included
    allp = np.concatenate([pts] * copies)
    np.testing.assert_array_equal(p2.cpu().numpy(), np.stack([allp[r][i2[r]] for r in range(copies * B)]))
    np.testing.assert_array_equal(p1.cpu().numpy(), np.stack([allp[r][i1[r]] for r in range(copies * B)]))


def _vox_fast_state(ws, B, N, copies=1):
    """(vdim [B,4], U [B]) of a device-drawn downsample's workspace (voxel.hip carve_voxel_fast:
    256-byte aligned sub-buffers in this order; white-box): the voxel box dims with the dense
    flag, and the listed-voxel count."""
    off, o, R = 0, {}, B * copies
    for name, nbytes in (("mm", B * 64 * 72), ("pmm", B * 1024 * 6 * 4), ("sel", R * 16),
                         ("reps", B * N * 8), ("rhash", B * N * 4), ("vlist", B * N * 4),
                         ("vdim", B * 16), ("phist", R * 4096 * 4), ("ties", R * 8192 * 8),
                         ("cnt4", R * 16)):
        off = (off + 255) & ~255
        o[name] = off
        off += nbytes
    vdim = ws[o["vdim"]:o["vdim"] + B * 16].view(torch.int32).view(B, 4).cpu().numpy()
    cnt4 = ws[o["cnt4"]:o["cnt4"] + R * 16].view(torch.int32).view(R, 4).cpu().numpy()
    return vdim, cnt4[:B, 0]


def _collision_cloud(rng, N):
    """A cloud whose voxel box is 197 x 17 x 3 -- outside every certified dense box -- with points
    in the voxels (190, 5, 1) and (196, 16, 2), whose xor-hashes collide (the reference merges
    them into one group)."""
    lo = np.zeros(3, np.float32)
    hi = np.array([196.5, 16.5, 2.5], np.float32)
    T = int(round(float(np.prod(hi)) * 1.728))
    vs = np.float32(float(np.float32(np.prod(hi)) / np.float32(T)) ** (1.0 / 3.0)) * np.float32(1.2)
    pts = (rng.random((N, 3)) * hi).astype(np.float32)
    pts[0], pts[1] = lo, hi
    pts[2] = (np.array([190.5, 5.5, 1.5]) * vs).astype(np.float32)
    pts[3] = (np.array([196.5, 16.5, 2.5]) * vs).astype(np.float32)
    pts[3] = np.minimum(pts[3], hi)
    return pts, T


@pytest.mark.parametrize("case", ["collision", "certified", "elongated", "lidar"])
def test_voxel_dense_and_hash_paths(H, case):
    """The device-drawn downsample's two grouping paths (voxel.hip voxel_box): a voxel box inside
    a certified collision-free box takes the dense grid (non-returning adds, no hash table), any
    other the hash table -- including a box in which two occupied voxels' hashes collide, which the
    reference (torch.unique on the hash) merges into one group.  Either way the listed-voxel count
    is the oracle's U (its groups: the reference's) and the subset is a valid draw."""
    from pointcloud_style_transfer_amd.synthetic import lidar_like_cloud

    rng = np.random.default_rng(len(case))
    N = 20000
    if case == "collision":
        pts, T = _collision_cloud(rng, N)
        want_dense = 0
    elif case == "certified":
        pts, T = rng.standard_normal((N, 3)).astype(np.float32), 5000
        want_dense = 1
    elif case == "elongated":
        pts, T = (rng.standard_normal((N, 3)) * np.array([1, 0.02, 0.02])).astype(np.float32), 8000
        want_dense = 0
    else:
        N = 120000
        pts, T = lidar_like_cloud(1000, N), 30000
        want_dense = 1
    reps, hashes, _ = O.voxel_reps(pts, T)
    if case == "collision":  # the merged pair really is in this cloud
        vs = np.float32(_)
        assert len(np.unique(hashes)) < len(np.unique(np.floor(pts / vs).astype(np.int64), axis=0))
    ws = H.voxel_copies_workspace(1, N, 1, "cuda")
    _, idx = H.voxel_downsample(dev(pts[None]), T, seed=11, ws=ws)
    vdim, U = _vox_fast_state(ws, 1, N)
    assert vdim[0, 3] == want_dense, vdim
    assert int(U[0]) == len(reps), (int(U[0]), len(reps))
    i = idx[0].cpu().numpy()
    vals, cnt = np.unique(i, return_counts=True)
    rv, rc = np.unique(reps, return_counts=True)
    if len(reps) < T:
        have = dict(zip(vals.tolist(), cnt.tolist()))
        assert all(have.get(v, 0) == k for v, k in zip(rv.tolist(), rc.tolist()))
        assert (~np.isin(vals, rv)).sum() == T - len(reps)
    else:
        assert np.isin(i, reps).all()


def test_voxel_pad_subset_is_uniform(H):
    """The device-drawn pad subset (U < T: T - U of the P non-representatives, the ones with
    the smallest counter-based random keys: csrc/voxel.hip voxf_hist/select radix select and
    the boundary bin's exact tie ranking in voxf_emit) is a uniform random subset: over 400 seeds every pool point's inclusion frequency is (T - U) / P within
    a binomial 5-sigma band, the count per seed is exact, the per-seed sets differ, and the
    frequencies of the pool's first and second halves agree (no positional bias)."""
    rng = np.random.default_rng(5)
    N, T = 6000, 3000
    pts = (rng.standard_normal((1, N, 3)) * np.array([1, 1, 0.2])).astype(np.float32)
    x = dev(pts)
    from oracle import oracle as O
    reps = O.voxel_reps(pts[0], T)[0]
    U = len(reps)
    assert U < T
    pool = np.setdiff1d(np.arange(N), reps)
    P, need = len(pool), T - U
    S = 400
    hits = np.zeros(N, np.int64)
    prev = None
    for seed in range(S):
        _, idx = H.voxel_downsample(x, T, seed=1000 + seed)
        i = idx[0].cpu().numpy()
        extra = np.setdiff1d(i, reps)
        assert len(extra) == need and len(np.unique(extra)) == need
        hits[extra] += 1
        if prev is not None:
            assert not np.array_equal(prev, extra)
        prev = extra
    f = hits[pool] / S
    p = need / P
    sd = np.sqrt(p * (1 - p) / S)
    assert np.abs(f - p).max() <= 5 * sd + 1e-12, (np.abs(f - p).max(), sd)
    h = len(pool) // 2
    assert abs(f[:h].mean() - f[h:].mean()) <= 5 * sd / np.sqrt(h)
    assert hits[reps].sum() == 0


def test_knn_golden(H, golden):
    g = golden("hierarchical.npz")
    out = H.knn3_interp(dev(g["knn_coarse"]), dev(g["knn_orig"]), dev(g["knn_idx"]), check=True)
    np.testing.assert_array_equal(out.cpu().numpy(), g["knn_out"])


def test_knn_golden_120k(H, golden):
    from pointcloud_style_transfer_amd.synthetic import lidar_like_cloud, standard_normal

    g = golden("hierarchical.npz")
    pts = lidar_like_cloud(int(g["full_seed"]), 120000)[None]
    idx = g["full_idx"].astype(np.int64)
    coarse = standard_normal(int(g["knn_full_coarse_seed"]), (1, 120000, 3))[:, idx[0]]
    out = H.knn3_interp(dev(coarse), dev(pts), dev(idx), check=True)
    np.testing.assert_array_equal(out.cpu().numpy(), g["knn_full_out"])


@pytest.mark.parametrize("N,M,B,sig", [(3000, 700, 2, (1, 1, 1)), (40000, 10000, 2, (3, 1, 0.01)),
                                        (500, 2, 1, (1, 1, 1)), (1000, 1, 1, (1, 1, 1))])
def test_knn_vs_oracle(H, N, M, B, sig):
    rng = np.random.default_rng(M)
    orig = (rng.standard_normal((B, N, 3)) * np.array(sig)).astype(np.float32)
    idx = np.stack([rng.choice(N, M, replace=False) for _ in range(B)])
    field = rng.standard_normal((B, N, 3)).astype(np.float32)
    coarse = np.stack([field[b][idx[b]] for b in range(B)])
    out = H.knn3_interp(dev(coarse), dev(orig), dev(idx), check=True).cpu().numpy()
    np.testing.assert_array_equal(out, O.upsample_knn(coarse, orig, idx))


def test_knn_outlier_pass_gaussian_vs_oracle(H):
    """A noisy-step cloud (isotropic Gaussian, the sampler's x at t = 999; 60000 rows, 15000
    coarse): its tail queries leave the query pass (sparse shells) and are answered by the
    brick-shell outlier search -- bit-exact vs the oracle's brute-force float64 3-NN."""
    rng = np.random.default_rng(999)
    N, M, B = 60000, 15000, 2
    orig = rng.standard_normal((B, N, 3)).astype(np.float32)
    idx = np.stack([rng.choice(N, M, replace=False) for _ in range(B)]).astype(np.int64)
    coarse = rng.standard_normal((B, M, 3)).astype(np.float32)
    st = []
    out = H.knn3_interp(dev(coarse), dev(orig), dev(idx), check=True, stats=st).cpu().numpy()
    assert min(st[0]["outliers"]) > 20, st
    np.testing.assert_array_equal(out, O.upsample_knn(coarse, orig, idx))


def _clustered(rng, N):
    """tight clusters, a uniform halo and far outliers (sparse shells, exhaustive fallback)"""
    centers = rng.uniform(-2, 2, (12, 3))
    pts = centers[rng.integers(0, 12, N)] + rng.standard_normal((N, 3)) * 0.02
    halo = rng.random(N) < 0.1
    pts[halo] = rng.uniform(-3, 3, (halo.sum(), 3))
    far = rng.random(N) < 0.002
    pts[far] *= 25.0
    return pts.astype(np.float32)


@pytest.mark.parametrize("case", ["clustered", "duplicates", "overfull", "planar"])
def test_knn_edge_cases(H, case):
    rng = np.random.default_rng(11)
    N, M = 20000, 5000
    if case == "clustered":
        orig = _clustered(rng, N)
        idx = rng.choice(N, M, replace=False)
    elif case == "duplicates":
        orig = rng.standard_normal((N, 3)).astype(np.float32)
        idx = rng.choice(N, M, replace=True)  # repeated rows: last coarse value wins
    elif case == "overfull":
        # thousands of refs in one cell (more than a wave's LDS stage) + exact distance ties
        orig = rng.standard_normal((N, 3)).astype(np.float32)
        orig[:6000] = np.round(orig[:6000] * 1e-3, 6)
        idx = rng.choice(N, M, replace=False)
    else:
        orig = rng.standard_normal((N, 3)).astype(np.float32)
        orig[:, 2] = 0.0
        idx = rng.choice(N, M, replace=False)
    orig, idx = orig[None], idx[None].astype(np.int64)
    coarse = rng.standard_normal((1, M, 3)).astype(np.float32)
    out = H.knn3_interp(dev(coarse), dev(orig), dev(idx), check=True).cpu().numpy()
    np.testing.assert_array_equal(out, O.upsample_knn(coarse, orig, idx))


def _noise_params(det_state, H, precision):
    from pointcloud_style_transfer_amd import packing

    blob = torch.from_numpy(packing.pack_blob(det_state, precision)).cuda()
    assert blob.numel() == H.noise_mlp_blob_bytes(precision)
    bias = dev(packing.pack_bias(det_state))
    g = lambda n: dev(det_state[f"noise_predictor.{n}"])  # noqa: E731
    freqs = packing.time_freqs(128).cuda()
    return blob, bias, (freqs, g("time_proj.weight").t().contiguous(), g("time_proj.bias"),
                        g("style_proj.weight").t().contiguous(),
                        g("style_proj.bias"), g("point_encoder.4.bias"))


@pytest.mark.parametrize("precision", [0, 1])
def test_noise_mlp_golden(H, golden, det_state, precision):
    g = golden("noise_predictor.npz")
    blob, bias, cp = _noise_params(det_state, H, precision)
    pts = g["points"]  # [2, 4096, 3]
    for t in g["ts"]:
        cond = H.noise_cond(dev(g[f"t{t}_tvec"]), dev(g["style"]), *cp)
        out = H.noise_mlp(dev(pts.reshape(-1, 3)), 4096, cond, blob, bias, precision)
        out = out.cpu().numpy().reshape(2, 4096, 3)
        ref = g[f"t{t}_out"]
        if precision == 0:
            assert_close(out, ref)
        else:
            err = np.linalg.norm(out - ref) / np.linalg.norm(ref)
            assert err < BF16_NORM_RTOL, err


@pytest.mark.parametrize("P,T", [(1, 1), (33, 33), (1000, 300), (60000, 30000)])
def test_noise_mlp_shapes_vs_oracle(H, det_state, P, T):
    blob, bias, cp = _noise_params(det_state, H, 0)
    rng = np.random.default_rng(P)
    C = (P + T - 1) // T
    pts = rng.standard_normal((P, 3)).astype(np.float32)
    t = rng.integers(0, 1000, C)
    style = rng.standard_normal((C, 256)).astype(np.float32) * 0.3
    cond = H.noise_cond(dev(t), dev(style), *cp)
    out = H.noise_mlp(dev(pts), T, cond, blob, bias, 0).cpu().numpy()
    pad = np.zeros((C * T, 3), np.float32)
    pad[:P] = pts
    ref = O.noise_predictor(det_state, pad.reshape(C, T, 3), t, style).reshape(-1, 3)[:P]
    assert_close(out, ref)


def test_cfg_ddim_step(H, golden):
    g = golden("schedule_losses.npz")
    ac = g["alphas_cumprod"]
    rng = np.random.default_rng(5)
    x, ec, eu, src = (rng.standard_normal((2, 5000, 3)).astype(np.float32) for _ in range(4))
    for t, tp in [(999, 888), (10, 0), (0, -1)]:
        a = np.float32(ac[t])
        ap = np.float32(ac[tp]) if tp >= 0 else np.float32(1.0)
        coeffs = (np.sqrt(np.float32(1) - a), np.sqrt(a) + np.float32(1e-8), np.sqrt(ap),
                  np.sqrt(np.float32(1) - ap))
        xc = torch.empty(4, 5000, 3, device="cuda")
        out = H.cfg_ddim_step(dev(x), dev(ec), dev(eu), dev(src), 7.5, coeffs, x_cat=xc)
        sched = O.Schedule()
        sched.alphas_cumprod = ac
        ref = O.guided_update(sched, x, ec, eu, src, t, tp, 7.5)
        assert_close(out.cpu().numpy(), ref, rtol=1e-5)
        np.testing.assert_array_equal(xc.cpu().numpy(), np.concatenate([out.cpu().numpy()] * 2))


def test_knn_build_query_phases_match_interp(H):
    """pcst_knn3_build on a side stream + pcst_knn3_query gives the bit-identical result of the
    one-call pcst_knn3_interp."""
    rng = np.random.default_rng(21)
    orig = dev(rng.standard_normal((2, 20000, 3)).astype(np.float32))
    idx = dev(np.stack([rng.choice(20000, 5000, replace=False) for _ in range(2)]).astype(np.int64))
    coarse = dev(rng.standard_normal((2, 5000, 3)).astype(np.float32))
    ref = H.knn3_interp(coarse, orig, idx)
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        handle = H.knn3_build(orig, idx)
    torch.cuda.current_stream().wait_stream(side)
    handle[2].record_stream(torch.cuda.current_stream())
    assert torch.equal(H.knn3_query(coarse, handle), ref)
    assert torch.equal(H.knn3_query(coarse, H.knn3_build(orig, idx)), ref)


@pytest.mark.parametrize("kind", ["gauss", "outliers", "m1"])
def test_knn_query_grid_cap_does_not_change_bits(H, kind):
    """pcst_knn3_query's grid_cap (work-groups over all clouds) only changes how many chunks each
    persistent wave takes from its row's work counters: 1, 2, 16, 64 (fewer than the 8 counter
    shards per row), 2^30 and the default (the resident grid) give the same bits, also when one
    workspace serves consecutive queries (the outlier launch re-zeroes the counters)."""
    rng = np.random.default_rng(100 + len(kind))
    orig, idx = _knn_case(kind, rng)
    coarse = dev(rng.standard_normal((2, idx.shape[1], 3)).astype(np.float32))
    h = H.knn3_build(orig, idx)
    ref = H.knn3_query(coarse, h)
    for cap in (1, 2, 16, 64, 1 << 30, 0):
        assert torch.equal(H.knn3_query(coarse, h, grid_cap=cap), ref), cap


def _knn_case(kind, rng):
    """(orig [2,N,3], idx [2,M]): a Gaussian cloud, one with far outliers (rows the query pass
    sends to the outlier pass), repeated indices (known rows written by several coarse rows) and
    the kk < 3 kernels (M = 1, 2)."""
    N, M = {"gauss": (20000, 5000), "outliers": (30000, 7500), "repeat": (8000, 3000),
            "m1": (500, 1), "m2": (500, 2)}[kind]
    orig = rng.standard_normal((2, N, 3)).astype(np.float32)
    if kind == "outliers":
        far = rng.choice(N, 300, replace=False)
        orig[:, far] *= 40.0
    if kind == "repeat":
        idx = rng.integers(0, N, (2, M))
    else:
        idx = np.stack([rng.choice(N, M, replace=False) for _ in range(2)])
    return dev(orig), dev(idx.astype(np.int64))


def _knn_carve(B, N, M):
    """Byte offsets of pcst_knn3_build's workspace arrays (knn.hip carve_knn: 256-byte aligned
    sub-buffers in this order; white-box, for the corruption test below) and the total size."""
    off = 0
    o = {}

    def take(name, nbytes):
        nonlocal off
        off = (off + 255) & ~255
        o[name] = off
        off += nbytes

    Cmax = min(max(4096, 16 * M), 1024 * 4096 - 1)
    T = -(-(Cmax + 1) // 4096)
    Cpad = T * 4096
    maxch = -(-N // 64) + 8 * (Cmax // 64) + 1
    for name, nbytes in (("stats", B * 64 * 72), ("gp", B * 8 * 4), ("refs", B * M * 16),
                         ("qorder", B * N * 4), ("crank", B * (M + N) * 8),
                         ("chunks", B * maxch * 8), ("olist", B * N * 4), ("obound", B * N * 4),
                         ("err", 16), ("qctr", B * 8 * 64 * 4), ("nchunk", 3 * ((B + 63) // 64 * 64) * 4), ("ocount", B * 4),
                         ("known", B * N * 4), ("tsum", B * T * 8), ("cnt", B * Cpad * 8)):
        take(name, nbytes)
    return o, maxch, Cpad, (off + 255) & ~255


def test_knn_query_corrupt_workspace_sets_error_bits(H):
    """The compact query's guards (knn.hip: a chunk outside [0, N] or longer than 64 rows sets
    bit 4 of the error word, a cell's or brick's ref range outside the ref array bit 8; the range
    is skipped, never read): a workspace corrupted between build and query -- chunk records with
    x > y and past N, start words of 100 cells pointing far past the refs -- yields the error bits
    and no fault; a clean build's word stays 0."""
    import ctypes

    rng = np.random.default_rng(41)
    orig, idx = _knn_case("gauss", rng)
    B, N, _ = orig.shape
    M = idx.shape[1]
    coarse = dev(rng.standard_normal((B, M, 3)).astype(np.float32))
    o, maxch, Cpad, total = _knn_carve(B, N, M)

    def err_word(ws):
        e = torch.zeros(1, dtype=torch.int32, device=ws.device)
        H._call("pcst_knn_error", H._ptr(ws), B, N, M, H._ptr(e), ctypes.c_void_p(
            torch.cuda.current_stream().cuda_stream))
        return int(e.item())

    h = H.knn3_build(orig, idx)
    ws = h[2]
    assert ws.numel() == total  # the carve above is the library's
    H.knn3_query(coarse, h)
    assert err_word(ws) == 0
    h = H.knn3_build(orig, idx, ws=ws)
    ch = ws[o["chunks"]:o["chunks"] + B * maxch * 8].view(torch.int32).view(B, maxch, 2)
    ch[0, :5, 0] = 7
    ch[0, :5, 1] = 3
    ch[1, :5, 1] = N + 100
    cnt = ws[o["cnt"]:o["cnt"] + B * Cpad * 8].view(torch.int32).view(B, Cpad, 2)
    cnt[1, 100:200, 0] = 0x7FFFFF00
    H.knn3_query(coarse, h)
    torch.cuda.synchronize()
    e = err_word(ws)
    assert e & 4 and e & 8, e


@pytest.mark.parametrize("kind", ["gauss", "outliers", "repeat"])
def test_knn_chunk_lists_tile_the_queries_long_chunks_first(H, kind):
    """The scan kernel's chunk lists (white-box, knn.hip knn_scan_kernel): per cloud the wide
    chunks (runs of two or more occupied octants) from the front of the array and the others from
    the back, their lengths in one packed word (wide << 32 | narrow) and the total beside; together
    the ranges tile the cloud's query positions [0, queries) exactly once, each 1..64 rows long."""
    rng = np.random.default_rng(7 + len(kind))
    orig, idx = _knn_case(kind, rng)
    B, N, _ = orig.shape
    M = idx.shape[1]
    o, maxch, Cpad, total = _knn_carve(B, N, M)
    h = H.knn3_build(orig, idx)
    ws = h[2]
    torch.cuda.synchronize()
    stride = (B + 63) // 64 * 64
    nch = ws[o["nchunk"]:o["nchunk"] + B * 4].view(torch.int32).cpu().numpy()
    packed = ws[o["nchunk"] + stride * 4:o["nchunk"] + stride * 4 + B * 8].view(torch.int64).cpu().numpy()
    ch = ws[o["chunks"]:o["chunks"] + B * maxch * 8].view(torch.int32).view(B, maxch, 2).cpu().numpy()
    for b in range(B):
        nw, nn = int(packed[b]) >> 32, int(packed[b]) & 0xFFFFFFFF
        assert nw + nn == nch[b] and nn > 0, (nw, nn, nch[b])
        rows = np.concatenate([ch[b, :nw], ch[b, maxch - nn:]])
        lens = rows[:, 1] - rows[:, 0]
        assert lens.min() >= 1 and lens.max() <= 64
        order = np.argsort(rows[:, 0])
        starts, ends = rows[order, 0], rows[order, 1]
        queries = N - len(np.unique(idx[b].cpu().numpy()))
        assert starts[0] == 0 and ends[-1] == queries
        assert np.array_equal(starts[1:], ends[:-1])  # contiguous, no overlap, no gap


@pytest.mark.parametrize("max_wg,floor", [(1, 0), (2, 8192), (32, 8192), (7, 0)])
def test_knn_build_workgroup_cap_is_exact(H, max_wg, floor):
    """pcst_knn3_build's max_wg only changes how many work-groups stride over the build's work
    (stats partials, element blocks, scan tiles, fill): the result is bit-identical to the
    natural grids, down to one work-group per cloud."""
    rng = np.random.default_rng(max_wg)
    orig = dev((rng.standard_normal((2, 60000, 3)) * [1, 0.5, 0.2]).astype(np.float32))
    idx = dev(np.stack([rng.choice(60000, 15000, replace=False) for _ in range(2)]).astype(np.int64))
    coarse = dev(rng.standard_normal((2, 15000, 3)).astype(np.float32))
    ref = H.knn3_interp(coarse, orig, idx)
    assert torch.equal(H.knn3_query(coarse, H.knn3_build(orig, idx, None, floor, max_wg)), ref)


def test_per_call_choices_on_concurrent_streams(H):
    """The ABI keeps no process-global switches (pcst.h conventions; tests/test_abi.py checks the
    symbol table): the kNN build's LDS floor and the Chamfer forward path are arguments, so two
    streams running the same calls with different choices at the same time cannot leak them
    into each other.  Results are bit-identical to the one-stream, default-argument calls."""
    rng = np.random.default_rng(5)
    orig = dev(rng.standard_normal((2, 40000, 3)).astype(np.float32))
    idx = dev(np.stack([rng.choice(40000, 10000, replace=False) for _ in range(2)]).astype(np.int64))
    coarse = dev(rng.standard_normal((2, 10000, 3)).astype(np.float32))
    p = dev((rng.standard_normal((4, 30000, 3)) * [1, 1, 0.2]).astype(np.float32))
    q = dev((rng.standard_normal((4, 30000, 3)) * [1, 1, 0.2]).astype(np.float32))
    ref_knn = H.knn3_interp(coarse, orig, idx)
    ref_cd = H.chamfer_fwd(p, q)
    torch.cuda.synchronize()
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    for s in (s1, s2):
        s.wait_stream(torch.cuda.current_stream())
    res = {}
    for rep in range(3):   # interleave the enqueues so the two streams' kernels overlap
        for name, s, floor, mode in (("a", s1, 8192, 2), ("b", s2, 0, 1)):
            with torch.cuda.stream(s):
                h = H.knn3_build(orig, idx, lds_floor=floor)
                res[name, rep] = (H.knn3_query(coarse, h), H.chamfer_fwd(p, q, mode))
    torch.cuda.synchronize()
    for (name, rep), (knn, cd) in res.items():
        assert torch.equal(knn, ref_knn), (name, rep)
        for x, y in zip(cd, ref_cd):
            assert torch.equal(x, y), (name, rep)


def test_device_events_order_streams(H):
    """pcst_event_* (device-scope fences, the sampling step's cross-stream dependencies): a
    consumer stream that waits on the event sees the producer stream's writes, here behind a
    long producer chain that would otherwise still be running."""
    prod, cons = torch.cuda.Stream(), torch.cuda.Stream()
    a = torch.randn(2048, 2048, device="cuda")
    out = torch.empty_like(a)
    ev = H.DeviceEvent()
    for rep in range(3):
        prod.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(prod):
            x = a.clone()
            for _ in range(20):
                x = torch.tanh(x @ a * 1e-3)
            flag = x.sum().reshape(1)
            ev.record(prod)
        ev.wait(cons)
        with torch.cuda.stream(cons):
            out.copy_(x)
            got = flag.clone()
        torch.cuda.synchronize()
        assert torch.equal(out, x) and torch.equal(got, x.sum().reshape(1)), rep
    t0, t1 = H.DeviceEvent(timing=True), H.DeviceEvent(timing=True)
    t0.record()
    torch.tanh(a @ a)
    t1.record()
    assert t0.elapsed_time(t1) > 0.0


def test_noise_mlp_wait_orders_after_the_signal(H):
    """pcst_noise_mlp_ex with a wait flag (the bf16 kernel's last work-group waits): the MLP's rows are the bits of pcst_noise_mlp, work queued after
    it on the stream sees what the signalling stream wrote before its pcst_signal_write (here a
    side stream that fills a 64 MB buffer after a delay), and the work-group counter is back to 0
    with no timeout."""
    from pointcloud_style_transfer_amd import packing
    from pointcloud_style_transfer_amd.config.config import Config
    from pointcloud_style_transfer_amd.models.diffusion_model import NoisePredictor

    torch.manual_seed(4)
    cfg = Config(make_dirs=False, precision="bf16")
    npred = NoisePredictor(cfg).cuda().eval()
    assert npred.precision_code == packing.BF16
    rng = np.random.default_rng(8)
    pts = dev(rng.standard_normal((2 * 30000, 3)).astype(np.float32))
    t = torch.tensor([999, 999], device="cuda")
    style = dev(rng.standard_normal((2, 256)).astype(np.float32))
    with torch.no_grad():
        cond = npred.cond(t, style)
        blob, bias = npred.packed()[:2]
        ref = H.noise_mlp(pts, 30000, cond, blob, bias, npred.precision_code)
        sig = H.DeviceSignal("cuda")
        side = torch.cuda.Stream()
        big = torch.zeros(16 << 20, device="cuda")
        side.wait_stream(torch.cuda.current_stream())
        for rep in range(3):
            with torch.cuda.stream(side):
                a = torch.randn(4096, 4096, device="cuda")
                for _ in range(4):
                    a = a @ a.T / 4096.0  # a delay on the side stream
                big.fill_(float(rep + 1))
                sig.signal(side)
            out = H.noise_mlp(pts, 30000, cond, blob, bias, npred.precision_code, wait=sig)
            seen = big.clone()  # ordered after the MLP, hence after the side's fill
            torch.cuda.synchronize()
            assert torch.equal(out, ref)
            assert bool((seen == float(rep + 1)).all())
            assert int(sig.flag[2].item()) == 0 and not sig.timed_out()
