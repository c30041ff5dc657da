"""HIP geometry kernels vs the reference's golden vectors and the oracle (bit-exact)."""
import numpy as np
import pytest
import torch

from oracle import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def H():
    from pointcloud_style_transfer_amd import _hip

    assert torch.cuda.is_available(), "GPU tests need the HIP device"
    _hip.lib()
    return _hip


def dev(a, dtype=None):
    t = torch.from_numpy(np.ascontiguousarray(a))
    if dtype is not None:
        t = t.to(dtype)
    return t.cuda()


def test_square_distance(H, golden):
    g = golden("geometry.npz")
    out = H.square_distance(dev(g["sqd_src"]), dev(g["sqd_dst"])).cpu().numpy()
    np.testing.assert_array_equal(out, g["sqd_out"])


def test_index_points(H, golden):
    g = golden("geometry.npz")
    out = H.index_points(dev(g["ip_points"]), dev(g["ip_idx"])).cpu().numpy()
    np.testing.assert_array_equal(out, g["ip_out"])


@pytest.mark.parametrize("key", ["fps_a", "fps_b", "fps_c", "fps_tie"])
def test_fps_golden(H, golden, key):
    g = golden("geometry.npz")
    out = H.fps(dev(g[f"{key}_xyz"]), int(g[f"{key}_npoint"]), dev(g[f"{key}_start"]))
    np.testing.assert_array_equal(out.cpu().numpy(), g[f"{key}_idx"])


@pytest.mark.parametrize("N,npoint,B", [(1, 1, 1), (7, 5, 3), (513, 100, 2), (9000, 300, 2),
                                        (30720, 64, 1), (40000, 32, 2)])
def test_fps_vs_oracle_sizes(H, N, npoint, B):
    rng = np.random.default_rng(N)
    xyz = rng.standard_normal((B, N, 3)).astype(np.float32)
    start = rng.integers(0, N, B)
    out = H.fps(dev(xyz), npoint, dev(start)).cpu().numpy()
    np.testing.assert_array_equal(out, O.farthest_point_sample(xyz, npoint, start))


def _fps_one_group(H, x, npoint, start):
    """pcst_fps (no workspace): the one-work-group-per-cloud kernels (culled for 8192 < N <=
    30720, register-resident below), which pcst_fps_ws replaces by the multi-CU kernel where
    that applies."""
    out = torch.empty(x.shape[0], npoint, device=x.device, dtype=torch.int64)
    H._call("pcst_fps", H._ptr(x), x.shape[0], x.shape[1], npoint, H._ptr(start), H._ptr(out),
            H._stream())
    return out


@pytest.mark.parametrize("case", ["lidar", "duplicates", "one_bin", "lattice", "small_cluster",
                                  "empty_regions"])
def test_fps_culled_vs_oracle(H, case):
    """The spatially culled FPS (8192 < N <= 30720: Morton regions per wave, an LDS overflow
    set, skipped waves) and the multi-CU FPS (the same clouds through pcst_fps_ws: B * K <= 32
    work-groups exchanging tagged round winners) against the oracle: clouds with exact distance
    ties (duplicated points, a lattice), one dense Morton bin (the greedy fill falls back to
    index ranges), a realistic cloud at the SA1 size."""
    from pointcloud_style_transfer_amd.synthetic import lidar_like_cloud

    rng = np.random.default_rng(7)
    if case == "lidar":
        xyz = lidar_like_cloud(11, 30000)[None].astype(np.float32)
    elif case == "duplicates":
        base = rng.standard_normal((10000, 3)).astype(np.float32)
        xyz = base[rng.integers(0, 10000, 30000)][None]
    elif case == "one_bin":
        xyz = (rng.standard_normal((1, 25000, 3)) * 1e-4).astype(np.float32)
        xyz[0, :40] = rng.uniform(-5, 5, (40, 3))
    elif case == "lattice":
        g = np.arange(32, dtype=np.float32)
        xyz = np.stack(np.meshgrid(g, g, g[:29], indexing="ij"), -1).reshape(1, -1, 3)
    elif case == "empty_regions":  # 8200 points over 16 regions of 576 slots: the last ones empty
        xyz = rng.standard_normal((2, 8200, 3)).astype(np.float32)
    else:
        xyz = rng.standard_normal((2, 9000, 3)).astype(np.float32)
    B, N = xyz.shape[:2]
    start = rng.integers(0, N, B)
    ref = O.farthest_point_sample(xyz, 512, start)
    out = H.fps(dev(xyz), 512, dev(start)).cpu().numpy()
    np.testing.assert_array_equal(out, ref)
    one = _fps_one_group(H, dev(xyz), 512, dev(start)).cpu().numpy()
    np.testing.assert_array_equal(one, ref)


@pytest.mark.parametrize("N,npoint,B", [(8193, 200, 1), (16384, 300, 2), (30000, 512, 1),
                                        (32768, 128, 1), (9000, 300, 3), (20000, 1, 1),
                                        (12000, 4000, 1)])
def test_fps_multi_cu_vs_oracle(H, N, npoint, B):
    """The multi-CU FPS at its shape limits (K = ceil(N / 1024) from 9 to 32 work-groups per
    cloud, B * K up to 32, one sample, more samples than one work-group's points) against the
    oracle; the call takes that kernel (its workspace is the tagged slots)."""
    import ctypes

    sz = ctypes.c_size_t(0)
    H._call("pcst_fps_workspace_size", B, N, ctypes.byref(sz))
    K = -(-N // 1024)
    assert B * K <= 32 and sz.value == max(B * K * 2 * 8 * 8, B * N * 4 if N > 30720 else 0)
    rng = np.random.default_rng(N + B)
    xyz = rng.standard_normal((B, N, 3)).astype(np.float32)
    xyz[:, 5:9] = xyz[:, :4]  # exact ties
    start = rng.integers(0, N, B)
    out = H.fps(dev(xyz), npoint, dev(start)).cpu().numpy()
    np.testing.assert_array_equal(out, O.farthest_point_sample(xyz, npoint, start))


@pytest.mark.parametrize("key", ["bq_sa1", "bq_sa2", "bq_edge"])
def test_ball_query_golden(H, golden, key):
    g = golden("geometry.npz")
    out = H.ball_query(float(g[f"{key}_radius"]), int(g[f"{key}_nsample"]),
                       dev(g[f"{key}_xyz"]), dev(g[f"{key}_new"]))
    np.testing.assert_array_equal(out.cpu().numpy(), g[f"{key}_idx"])


@pytest.mark.parametrize("N,S,ns,r", [(100, 10, 8, 0.3), (5000, 77, 64, 0.1), (3000, 40, 512, 0.5)])
def test_ball_query_vs_oracle(H, N, S, ns, r):
    rng = np.random.default_rng(S)
    xyz = rng.uniform(-1, 1, (2, N, 3)).astype(np.float32)
    new = xyz[:, rng.integers(0, N, S)]
    out = H.ball_query(r, ns, dev(xyz), dev(new)).cpu().numpy()
    np.testing.assert_array_equal(out, O.query_ball_point(r, ns, xyz, new))


def test_group_gather(H, golden):
    g = golden("geometry.npz")
    xyz = g["fps_c_xyz"]
    fidx = g["fps_c_idx"]
    gidx = g["bq_sa2_idx"]
    feats = np.random.default_rng(0).standard_normal((2, xyz.shape[1], 5)).astype(np.float32)
    new, grouped = H.group_gather(dev(xyz), dev(feats), dev(fidx), dev(gidx))
    ref_new = O.index_points(xyz, fidx)
    np.testing.assert_array_equal(new.cpu().numpy(), ref_new)
    ref = np.concatenate([O.index_points(xyz, gidx) - ref_new[:, :, None], O.index_points(feats, gidx)], -1)
    np.testing.assert_array_equal(grouped.cpu().numpy(), ref)
