"""Pin the CPU oracle against golden vectors captured from the reference itself.

CPU-only (no GPU marker).  Index outputs bit-exact; float outputs within the
stated tolerances (numpy/OpenBLAS vs the reference's MKL sgemm differ only in
summation order).
"""
import numpy as np
import pytest

from oracle import oracle as O
from conftest import assert_close, assert_mostly_close

RTOL = 1e-4   # north_star: features/coordinates within 1e-4 rel (fp32)
ATOL = 1e-5


def test_square_distance_bitexact(golden):
    g = golden("geometry.npz")
    np.testing.assert_array_equal(O.square_distance(g["sqd_src"], g["sqd_dst"]), g["sqd_out"])


def test_index_points(golden):
    g = golden("geometry.npz")
    np.testing.assert_array_equal(O.index_points(g["ip_points"], g["ip_idx"]), g["ip_out"])


@pytest.mark.parametrize("key", ["fps_a", "fps_b", "fps_c", "fps_tie"])
def test_fps_bitexact(golden, key):
    g = golden("geometry.npz")
    out = O.farthest_point_sample(g[f"{key}_xyz"], int(g[f"{key}_npoint"]), g[f"{key}_start"])
    np.testing.assert_array_equal(out, g[f"{key}_idx"])


@pytest.mark.parametrize("key", ["bq_sa1", "bq_sa2", "bq_edge"])
def test_ball_query_bitexact(golden, key):
    g = golden("geometry.npz")
    out = O.query_ball_point(float(g[f"{key}_radius"]), int(g[f"{key}_nsample"]),
                             g[f"{key}_xyz"], g[f"{key}_new"])
    np.testing.assert_array_equal(out, g[f"{key}_idx"])


@pytest.mark.parametrize("key", ["pad", "sub", "ident"])
def test_voxel_downsample_bitexact(golden, key):
    g = golden("hierarchical.npz")
    rp = O.Replay.from_npz(g, f"{key}_rng")
    pts, idx = O.voxel_downsample(g[f"{key}_pts"], int(g[f"{key}_target"]), rp)
    np.testing.assert_array_equal(idx, g[f"{key}_idx"])
    np.testing.assert_array_equal(pts, g[f"{key}_down"])
    assert rp.pos == len(rp.draws)


def test_voxel_downsample_full_120k(golden):
    from pointcloud_style_transfer_amd.synthetic import lidar_like_cloud

    g = golden("hierarchical.npz")
    pts = lidar_like_cloud(int(g["full_seed"]), 120000)[None]
    rp = O.Replay([("randperm", g["full_perm"].astype(np.int64))])
    _, idx = O.voxel_downsample(pts, 30000, rp)
    np.testing.assert_array_equal(idx, g["full_idx"].astype(np.int64))


def test_upsample_knn(golden):
    g = golden("hierarchical.npz")
    out = O.upsample_knn(g["knn_coarse"], g["knn_orig"], g["knn_idx"])
    np.testing.assert_array_equal(out, g["knn_out"])


def test_upsample_knn_full_120k(golden):
    from pointcloud_style_transfer_amd.synthetic import lidar_like_cloud, standard_normal

    g = golden("hierarchical.npz")
    pts = lidar_like_cloud(int(g["full_seed"]), 120000)[None]
    idx = g["full_idx"].astype(np.int64)
    coarse = standard_normal(int(g["knn_full_coarse_seed"]), (1, 120000, 3))[:, idx[0]]
    out = O.upsample_knn(coarse, pts, idx)
    np.testing.assert_array_equal(out, g["knn_full_out"])


def test_schedule(golden):
    g = golden("schedule_losses.npz")
    s = O.Schedule()
    # betas = 1 - ac[t+1]/ac[t] cancels: numpy cos vs torch's vectorised cos leaves ~1 ulp of
    # ac in beta's absolute error (3e-7); the tables the sampler reads agree to 1e-4 rel.
    np.testing.assert_allclose(s.betas, g["betas"], rtol=0, atol=5e-7)
    np.testing.assert_allclose(s.alphas_cumprod, g["alphas_cumprod"], rtol=1e-4, atol=1e-9)
    np.testing.assert_allclose(O.beta_schedule(name="linear"), g["betas_linear"], rtol=1e-6)
    xt = s.q_sample(g["q_x0"], g["q_t"], g["q_noise"])
    np.testing.assert_allclose(xt, g["q_xt"], rtol=RTOL, atol=ATOL)


def test_chamfer_and_grad(golden):
    g = golden("schedule_losses.npz")
    cd = O.chamfer_distance(g["cd_pred"], g["cd_target"])
    np.testing.assert_allclose(cd, g["cd_out"], rtol=1e-5)
    gp, gt = O.chamfer_grad(g["cd_pred"], g["cd_target"])
    np.testing.assert_allclose(gp, g["cd_grad_pred"], rtol=1e-4, atol=1e-9)
    np.testing.assert_allclose(gt, g["cd_grad_target"], rtol=1e-4, atol=1e-9)
    cd2 = O.chamfer_distance(g["cd_pred"][:, :1500], g["cd_target"][:, :700])
    np.testing.assert_allclose(cd2, g["cd2_out"], rtol=1e-5)


def test_diffusion_loss(golden):
    g = golden("schedule_losses.npz")
    pn, an, pp, tp = g["dl_inputs"]
    total, d = O.diffusion_loss(pn, an, pp, tp)
    assert abs(d["noise_loss"] - float(g["dl_noise"])) < 1e-6
    assert abs(d["chamfer_loss"] - float(g["dl_chamfer"])) < 1e-5 * float(g["dl_chamfer"])
    assert abs(total - float(g["dl_total"])) < 1e-5 * float(g["dl_total"])
    t2, _ = O.diffusion_loss(pn, an)
    assert abs(t2 - float(g["dl_total_noise_only"])) < 1e-6


def test_time_embedding(golden):
    g = golden("noise_predictor.npz")
    np.testing.assert_allclose(O.time_embedding(g["temb_t"], 128), g["temb"], rtol=1e-5, atol=2e-6)


def test_noise_predictor(golden, det_state):
    g = golden("noise_predictor.npz")
    for t in g["ts"]:
        out = O.noise_predictor(det_state, g["points"], g[f"t{t}_tvec"], g["style"])
        np.testing.assert_allclose(out, g[f"t{t}_out"], rtol=RTOL, atol=ATOL)


@pytest.mark.parametrize("mode", ["eval", "train"])
def test_set_abstraction_stack(golden, det_state, mode):
    g = golden("encoder.npz")
    rp = O.Replay.from_npz(g, f"{mode}_rng")
    train = mode == "train"
    pre = "style_encoder.encoder"
    l1x, l1p = O.set_abstraction(det_state, pre + ".sa1", g["xyz"], None, rp, train)
    np.testing.assert_array_equal(l1x, g[f"{mode}_l1_xyz"])
    assert_close(l1p, g[f"{mode}_l1_points"])
    # feed the reference's own l1 outputs forward (teacher-forced per layer)
    l2x, l2p = O.set_abstraction(det_state, pre + ".sa2", g[f"{mode}_l1_xyz"],
                                 g[f"{mode}_l1_points"].transpose(0, 2, 1), rp, train)
    np.testing.assert_array_equal(l2x, g[f"{mode}_l2_xyz"])
    assert_close(l2p, g[f"{mode}_l2_points"])
    _, l3 = O.set_abstraction(det_state, pre + ".sa3", g[f"{mode}_l2_xyz"],
                              g[f"{mode}_l2_points"].transpose(0, 2, 1), rp, train)
    assert_close(l3, g[f"{mode}_l3"])


def test_style_encoder(golden, det_state):
    g = golden("encoder.npz")
    out = O.style_encoder(det_state, g["xyz"], O.Replay.from_npz(g, "style_rng"))
    np.testing.assert_allclose(out, g["style"], rtol=RTOL, atol=ATOL)
    from pointcloud_style_transfer_amd.synthetic import lidar_like_cloud

    out30 = O.style_encoder(det_state, lidar_like_cloud(43, 30000)[None],
                            O.Replay.from_npz(g, "style30_rng"))
    np.testing.assert_allclose(out30, g["style30"], rtol=RTOL, atol=ATOL)


def test_guided_loop_direct_cfg1(golden, det_state):
    g = golden("sampling.npz")
    rp = O.Replay.from_npz(g, "a_rng")
    out = O.guided_sample_loop(det_state, g["a_src"], g["a_cond"], 10, 7.5, rp)
    assert_mostly_close(out, g["a_out"])


def test_guided_loop_hierarchical(golden, det_state):
    g = golden("sampling.npz")
    rp = O.Replay.from_npz(g, "b_rng")
    out = O.guided_sample_loop(det_state, g["b_src"], g["b_cond"], 3, 7.5, rp, global_points=1024)
    assert_mostly_close(out, g["b_out"], max_abs=5e-2)
