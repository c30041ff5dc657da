"""The kNN-3 upsample's rows layout (pcst_knn3_rows_build / _refs / _query: the sampling step's
split of the build into a positions-only phase beside the voxel downsample and a one-launch ref
placement after it) against the compact layout (pcst_knn3_interp) and the oracle's brute-force
float64 3-NN (oracle.upsample_knn, diffusion_model.py:127-153): bit-exact on every case the
compact layout's tests cover -- Gaussian clouds, far outliers (the brick-shell pass over a
brick's whole row range, empty slots skipped), repeated indices (free slots of the cell) and a
pile-up of one index beyond its cell's rows (the overflow list), clusters, overfull cells with
exact ties, a planar cloud, kk < 3 -- and on CFG batches (copies of each cloud with their own
coarse subsets)."""
import zlib

import numpy as np
import pytest
import torch

from oracle import oracle as O

pytestmark = pytest.mark.gpu


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


@pytest.fixture(scope="module")
def H():
    from pointcloud_style_transfer_amd import _hip

    return _hip


def _cloud(kind, rng, N):
    x = rng.standard_normal((N, 3)).astype(np.float32)
    if kind == "outliers":
        x[rng.choice(N, 300, replace=False)] *= 40.0
    elif kind == "clustered":
        centers = rng.uniform(-2, 2, (12, 3))
        x = centers[rng.integers(0, 12, N)] + rng.standard_normal((N, 3)) * 0.02
        halo = rng.random(N) < 0.1
        x[halo] = rng.uniform(-3, 3, (halo.sum(), 3))
        x[rng.random(N) < 0.002] *= 25.0
        x = x.astype(np.float32)
    elif kind == "overfull":
        x[:6000] = np.round(x[:6000] * 1e-3, 6)
    elif kind == "planar":
        x[:, 2] = 0.0
    return x


@pytest.mark.parametrize("kind,N,M,C,copies", [
    ("gauss", 20000, 5000, 1, 2), ("outliers", 30000, 7500, 1, 2), ("repeat", 8000, 3000, 1, 2),
    ("clustered", 20000, 5000, 1, 1), ("overfull", 20000, 5000, 1, 1), ("planar", 20000, 5000, 1, 1),
    ("gauss", 12000, 3000, 2, 2), ("m1", 500, 1, 1, 2), ("m2", 500, 2, 1, 2),
    ("pileup", 8000, 3000, 1, 2)])
def test_knn_rows_layout_matches_compact_and_oracle(H, kind, N, M, C, copies):
    rng = np.random.default_rng(zlib.crc32(f"{kind}/{N}/{C}".encode()))
    x = np.stack([_cloud(kind, rng, N) for _ in range(C)])
    B = C * copies
    if kind == "repeat":
        idx = rng.integers(0, N, (B, M))
    else:
        idx = np.stack([rng.choice(N, M, replace=False) for _ in range(B)])
    if kind == "pileup":  # 400 refs naming one point: more than its cell has rows
        idx[:, 100:500] = idx[:, 7:8]
    idx = idx.astype(np.int64)
    coarse = rng.standard_normal((B, M, 3)).astype(np.float32)
    orig = np.concatenate([x] * copies)
    h = H.knn3_rows_build(dev(x), M, copies)
    H.knn3_rows_refs(h, dev(idx))
    got = H.knn3_rows_query(dev(coarse), h)
    st = H.knn_rows_stats(h)
    assert st["err"] == 0, st
    if kind == "pileup":
        assert min(st["overflow"]) > 0, st
    elif kind != "repeat":
        assert max(st["overflow"]) == 0, st
    ref = H.knn3_interp(dev(coarse), dev(orig), dev(idx), check=True)
    assert torch.equal(got, ref)
    np.testing.assert_array_equal(got.cpu().numpy(), O.upsample_knn(coarse, orig, idx))


def test_knn_rows_outlier_pass_gaussian(H):
    """The noisy-step cloud of test_knn_outlier_pass_gaussian_vs_oracle through the rows layout:
    its tail queries reach the brick-shell pass, whose brick ranges hold the rows without a ref."""
    rng = np.random.default_rng(999)
    N, M = 60000, 15000
    x = rng.standard_normal((1, N, 3)).astype(np.float32)
    idx = np.stack([rng.choice(N, M, replace=False) for _ in range(2)]).astype(np.int64)
    coarse = rng.standard_normal((2, M, 3)).astype(np.float32)
    h = H.knn3_rows_build(dev(x), M, 2)
    H.knn3_rows_refs(h, dev(idx))
    got = H.knn3_rows_query(dev(coarse), h).cpu().numpy()
    st = H.knn_rows_stats(h)
    assert min(st["outliers"]) > 20 and st["err"] == 0, st
    np.testing.assert_array_equal(got, O.upsample_knn(coarse, np.concatenate([x, x]), idx))


def test_knn_rows_golden_120k(H, golden):
    """The 120k golden upsample (the reference's sklearn path, tests/golden) through the rows
    layout as one CFG row."""
    from pointcloud_style_transfer_amd.synthetic import lidar_like_cloud, standard_normal

    g = golden("hierarchical.npz")
    pts = lidar_like_cloud(int(g["full_seed"]), 120000)[None]
    idx = g["full_idx"].astype(np.int64)
    coarse = standard_normal(int(g["knn_full_coarse_seed"]), (1, 120000, 3))[:, idx[0]]
    out = H.knn3_interp_rows(dev(coarse), dev(pts), dev(idx), copies=1)
    np.testing.assert_array_equal(out.cpu().numpy(), g["knn_full_out"])


def test_knn_rows_bad_index_sets_the_error_word(H):
    """An index outside [0, N) is skipped and reported (bit 1), never read or written."""
    rng = np.random.default_rng(3)
    N, M = 5000, 1000
    x = rng.standard_normal((1, N, 3)).astype(np.float32)
    idx = rng.choice(N, (1, M), replace=False).astype(np.int64)
    idx[0, 17] = N + 5
    idx[0, 18] = -1
    h = H.knn3_rows_build(dev(x), M, 1)
    H.knn3_rows_refs(h, dev(idx))
    H.knn3_rows_query(dev(rng.standard_normal((1, M, 3)).astype(np.float32)), h)
    assert H.knn_rows_stats(h)["err"] & 1


def test_knn_rows_workspace_reuse_is_stateless(H):
    """One workspace through two builds of different clouds and index sets: each query gives the
    bits of a fresh workspace (the build zeroes its counters, marks and ref slots)."""
    rng = np.random.default_rng(8)
    N, M = 16000, 4000
    ws = H.knn_rows_workspace(1, 2, N, M, "cuda")
    for it in range(2):
        x = dev(rng.standard_normal((1, N, 3)).astype(np.float32))
        idx = dev(np.stack([rng.choice(N, M, replace=it == 1) for _ in range(2)]).astype(np.int64))
        coarse = dev(rng.standard_normal((2, M, 3)).astype(np.float32))
        h = H.knn3_rows_build(x, M, 2, ws=ws)
        H.knn3_rows_refs(h, idx)
        assert torch.equal(H.knn3_rows_query(coarse, h), H.knn3_interp_rows(coarse, x, idx, copies=2))


def test_knn_rows_refs_wait_timeout_places_nothing(H):
    """A ref placement whose wait for phase A gives up writes nothing, and the query and outlier
    launches handed its error word (the handle's refs_err) leave the workspace alone and write
    eps = 0: on a fresh workspace filled with 0xFF (phase A never ran: every count, start, rank
    and slot is garbage) the calls complete without a fault and the signal reports the timeout
    (the round-5 rank kernel's timeout path left the place launch reading garbage)."""
    rng = np.random.default_rng(21)
    N, M = 16000, 4000
    x = dev(rng.standard_normal((1, N, 3)).astype(np.float32))
    idx = dev(np.stack([rng.choice(N, M, replace=False) for _ in range(2)]).astype(np.int64))
    coarse = dev(rng.standard_normal((2, M, 3)).astype(np.float32))
    ws = H.knn_rows_workspace(1, 2, N, M, "cuda")
    ws.fill_(0xFF)
    sig = H.DeviceSignal(torch.device("cuda", 0), max_polls=2000)
    sig.value = 1  # never written: phase A "never signals"
    h = H.KnnRows(x, 2, M, ws)
    H.knn3_rows_refs(h, idx, wait=sig)
    out = H.knn3_rows_query(coarse, h)
    torch.cuda.synchronize()
    assert sig.timed_out()
    with pytest.raises(H.SignalTimeout):
        sig.check()
    assert not bool(out.any())


def _spy_rows_build(monkeypatch):
    """Count the loop's rows-layout builds (the overlapped rows path really ran)."""
    from pointcloud_style_transfer_amd import _hip

    calls = []
    real = _hip.knn3_rows_build

    def spy(*a, **k):
        calls.append(1)
        return real(*a, **k)

    monkeypatch.setattr(_hip, "knn3_rows_build", spy)
    return calls


def test_guided_loop_rows_layout_bit_identical(monkeypatch):
    """The sampling loop with the step's kNN in the rows layout (the product layout at one cloud:
    phase A beside the voxel downsample, one placement launch, the MLP's last work-group waiting
    for phase A) gives the bits of the compact build and of the single-stream loop, on the bench's
    120k cloud (5 steps from t = 999); the rows path ran once per step (no fallback to the
    single-stream layout)."""
    import bench
    from pointcloud_style_transfer_amd.models import diffusion_model as dm
    from pointcloud_style_transfer_amd.synthetic import lidar_like_cloud, standard_normal

    dev0 = torch.device("cuda", 0)
    cfg, model, dp = bench.build_model("bf16", dev0)
    src = torch.from_numpy(lidar_like_cloud(1000, 120000)[None]).to(dev0)
    cond = torch.from_numpy(lidar_like_cloud(2000, 120000)[None]).to(dev0)
    xT = torch.from_numpy(standard_normal(3000, (1, 120000, 3))).to(dev0)
    assert dm.rows_layout_ok(2 * cfg.global_points)
    calls = _spy_rows_build(monkeypatch)
    outs = []
    for rows, overlap in ((True, True), (False, True), (True, False)):
        monkeypatch.setattr(dm, "ROWS_LAYOUT", rows)
        monkeypatch.setattr(dm, "OVERLAP_KNN_BUILD", overlap)
        torch.manual_seed(7)
        n0 = len(calls)
        outs.append(dp.guided_sample_loop(model, src, cond, 5, 7.5, x_T=xT))
        assert len(calls) - n0 == (5 if rows and overlap else 0), (rows, overlap)
    assert torch.equal(outs[0], outs[1])
    assert torch.equal(outs[0], outs[2])


@pytest.mark.parametrize("N,M,C", [(40000, 10000, 1), (120000, 30000, 1), (20000, 5000, 2),
                                   (120000, 30000, 3)])
def test_downsample_places_rows_refs(H, N, M, C):
    """Phase B inside the voxel emit (pcst_voxel_downsample_rows: the sampling step's layout)
    places the same refs as pcst_knn3_rows_refs on the downsample's indices: the rows query gives
    the bits of the separate placement and of the compact layout on cat([x, x]).  At 3 clouds of
    120k the emit launch has more work-groups than CUs (708): it places nothing itself and phase B
    runs as its own launch inside the same call ("Forward progress")."""
    rng = np.random.default_rng(N + C)
    x = dev(rng.standard_normal((C, N, 3)).astype(np.float32))
    coarse = dev(rng.standard_normal((2 * C, M, 3)).astype(np.float32))
    h1 = H.knn3_rows_build(x, M, 2)
    _, xi = H.voxel_downsample(x, M, seed=5, copies=2, rows=h1)
    assert h1.placed
    got = H.knn3_rows_query(coarse, h1)
    h2 = H.knn3_rows_build(x, M, 2)
    H.knn3_rows_refs(h2, xi)
    assert torch.equal(got, H.knn3_rows_query(coarse, h2))
    assert torch.equal(got, H.knn3_interp(coarse, torch.cat([x, x]), xi))
    assert H.knn_rows_stats(h1)["err"] == 0
