"""Training-path kernels: the split-K weight/bias gradient of the per-point linear layers
(pcst_linear_wgrad) against a float64 torch product of the same operands, determinism, and the
layer shapes the trainer hits (noise predictor at B=8 x 30000 coarse points, SA1/SA2 grouped
rows, odd channel counts 3/131/259)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

# exact-f32 products, float64 chunk combine: the error is the f32 summation inside a chunk
WGRAD_RTOL = 1e-5


@pytest.fixture(scope="module")
def H():
    from pointcloud_style_transfer_amd import _hip

    assert torch.cuda.is_available()
    _hip.lib()
    return _hip


@pytest.mark.parametrize("M,I,O", [(1, 3, 64), (37, 3, 64), (1000, 131, 128), (4097, 259, 256),
                                   (131072, 64, 64), (240000, 256, 512), (240000, 512, 256),
                                   (8, 256, 512)])
def test_linear_wgrad_vs_float64(H, M, I, O):
    g = torch.Generator(device="cuda").manual_seed(M + I + O)
    dz = torch.randn(M, O, device="cuda", generator=g)
    x = torch.randn(M, I, device="cuda", generator=g)
    dw, db = H.linear_wgrad(dz, x, bias=True)
    ref_w = dz.double().t() @ x.double()
    ref_b = dz.double().sum(0)
    scale = float(np.sqrt(M))  # magnitude of a sum of M unit products
    assert (dw.double() - ref_w).abs().max().item() <= WGRAD_RTOL * scale * 10
    assert (db.double() - ref_b).abs().max().item() <= WGRAD_RTOL * scale * 10
    dw2, _ = H.linear_wgrad(dz, x, bias=False)
    assert torch.equal(dw, dw2), "wgrad must be deterministic"


def test_linear_fn_backward_matches_autograd(H):
    from pointcloud_style_transfer_amd.models import _autograd as ag

    torch.manual_seed(0)
    lin = torch.nn.Linear(131, 96).cuda()
    x = torch.randn(5000, 131, device="cuda", requires_grad=True)
    y = ag.linear(x, lin, relu=True)
    gy = torch.randn_like(y)
    y.backward(gy)
    gx, gw, gb = x.grad.clone(), lin.weight.grad.clone(), lin.bias.grad.clone()
    x64 = x.detach().double().requires_grad_()
    w64 = lin.weight.detach().double().requires_grad_()
    b64 = lin.bias.detach().double().requires_grad_()
    torch.relu(x64 @ w64.t() + b64).backward(gy.double())
    for a, b in ((gx, x64.grad), (gw, w64.grad), (gb, b64.grad)):
        err = (a.double() - b).norm() / b.norm()
        assert err.item() < 1e-5
