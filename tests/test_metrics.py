"""Evaluation metrics (evaluation/metrics.py, compare.py): the oracle
against the reference's own outputs (tests/golden/metrics.npz, gen_metrics.py), and the
device kernels (pcst_knn_dist, pcst_emd_greedy) against both.

Tolerances: EMD is bit-exact (same float64 distances, same greedy order, same summation);
coverage / F-score are exact counts; chamfer / hausdorff use exact distances while the
reference's torch.cdist uses the fp32 |p|^2+|q|^2-2pq form, so they agree to 1e-4 relative."""
import numpy as np
import pytest

from oracle import oracle as O

CDIST_RTOL = 1e-4


@pytest.fixture(scope="module")
def G(golden):
    return golden("metrics.npz")


def test_oracle_metrics_vs_reference(G):
    np.testing.assert_allclose(O.metric_chamfer(G["pred"], G["target"]), G["chamfer"], rtol=CDIST_RTOL)
    np.testing.assert_allclose(O.metric_chamfer(G["pred"], G["target"], False), G["chamfer_oneway"],
                               rtol=CDIST_RTOL)
    np.testing.assert_allclose(O.metric_hausdorff(G["pred"], G["target"]), G["hausdorff"], rtol=CDIST_RTOL)
    assert O.metric_coverage(G["pred"], G["target"]) == G["coverage_001"]
    assert O.metric_coverage(G["pred"], G["target"], 0.1) == G["coverage_01"]
    np.testing.assert_allclose(O.metric_uniformity(G["pred"]), G["uniformity"], rtol=1e-12)
    np.testing.assert_allclose(O.metric_uniformity(G["target"], 4), G["uniformity_k4"], rtol=1e-12)
    assert np.array_equal(O.emd_greedy(G["emd_pred"], G["emd_target"]), G["emd"])
    np.testing.assert_allclose(O.similarity(G["cmp1"], G["cmp2"], 0.2), G["similarity"], rtol=1e-12)


@pytest.mark.gpu
def test_device_metrics_vs_reference(G):
    import torch

    from pointcloud_style_transfer_amd.evaluation import PointCloudMetrics

    m = PointCloudMetrics("cuda")
    p, t = torch.from_numpy(G["pred"]), torch.from_numpy(G["target"])
    np.testing.assert_allclose(m.chamfer_distance(p, t).cpu().numpy(), G["chamfer"], rtol=CDIST_RTOL)
    np.testing.assert_allclose(m.chamfer_distance(p, t, False).cpu().numpy(), G["chamfer_oneway"],
                               rtol=CDIST_RTOL)
    np.testing.assert_allclose(m.hausdorff_distance(p, t).cpu().numpy(), G["hausdorff"], rtol=CDIST_RTOL)
    assert m.coverage_score(p, t) == G["coverage_001"]
    assert m.coverage_score(p, t, threshold=0.1) == G["coverage_01"]
    np.testing.assert_allclose(m.uniformity_score(p), G["uniformity"], rtol=1e-12)
    np.testing.assert_allclose(m.uniformity_score(t, k=4), G["uniformity_k4"], rtol=1e-12)
    np.testing.assert_allclose(m.fidelity_score(p, t), G["fidelity"], rtol=1e-6)
    emd = m.earth_mover_distance(torch.from_numpy(G["emd_pred"]), torch.from_numpy(G["emd_target"]))
    assert np.array_equal(emd.cpu().numpy(), G["emd"])


@pytest.mark.gpu
def test_device_compare_vs_reference(G):
    from pointcloud_style_transfer_amd.compare import calculate_similarity

    np.testing.assert_allclose(calculate_similarity(G["cmp1"], G["cmp2"], 0.2), G["similarity"],
                               rtol=1e-12)


@pytest.mark.gpu
@pytest.mark.parametrize("k", [1, 3, 9, 16])
def test_knn_dist_vs_oracle(k):
    import torch

    from pointcloud_style_transfer_amd import _hip

    rng = np.random.default_rng(k)
    P = rng.standard_normal((2, 777, 3)).astype(np.float32)
    Q = rng.standard_normal((2, 3001, 3)).astype(np.float32)
    Q[0, 2000:2010] = Q[0, 5]   # duplicated refs: ties
    d = _hip.knn_dist(torch.from_numpy(P).cuda(), torch.from_numpy(Q).cuda(), k).cpu().numpy()
    np.testing.assert_allclose(d, O.knn_dist(P, Q, k), rtol=1e-6, atol=1e-7)


@pytest.mark.gpu
def test_metrics_full_size_properties():
    """120k-point clouds (no oracle at this size): chamfer of a cloud with itself is 0, with a
    shifted copy it is the shift; EMD of a cloud with itself is 0."""
    import torch

    from pointcloud_style_transfer_amd.evaluation import PointCloudMetrics
    from pointcloud_style_transfer_amd.synthetic import lidar_like_cloud

    m = PointCloudMetrics("cuda")
    x = torch.from_numpy(lidar_like_cloud(1000, 120000))[None]
    assert m.chamfer_distance(x, x).item() == 0.0
    assert m.hausdorff_distance(x, x).item() == 0.0
    assert m.coverage_score(x, x) == 1.0
    y = x[:, :4096]
    assert m.earth_mover_distance(y, y).item() == 0.0
