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


def _bf(t, half=torch.bfloat16):
    return t.to(half).double()


HALVES = [torch.bfloat16, torch.float16]
HALF_IDS = ["bf16", "fp16"]


@pytest.mark.parametrize("half", HALVES, ids=HALF_IDS)
@pytest.mark.parametrize("M,K,O,relu", [(1, 3, 64, True), (1000, 3, 128, True), (4097, 131, 256, False),
                                        (60000, 256, 512, True), (60000, 512, 256, False),
                                        (300, 259, 3, False)])
def test_gemm_nt_bf16_vs_float64(H, M, K, O, relu, half):
    """16-bit-rounded operands (bfloat16, or float16 -- the reference's autocast format),
    fp32 accumulation: matches the float64 product of the same rounded operands up to fp32
    summation order."""
    g = torch.Generator(device="cuda").manual_seed(M + K + O)
    A = torch.randn(M, K, device="cuda", generator=g)
    B = torch.randn(O, K, device="cuda", generator=g)
    shift = torch.randn(O, device="cuda", generator=g)
    C = H.gemm_nt_bf16(A, B, None, shift, relu, half=half)
    ref = _bf(A, half) @ _bf(B, half).t() + shift.double()
    if relu:
        ref = ref.clamp_min(0)
    err = (C.double() - ref).norm() / ref.norm()
    assert err.item() < 1e-6, err.item()


@pytest.mark.parametrize("half", HALVES, ids=HALF_IDS)
@pytest.mark.parametrize("M,I,O", [(37, 3, 64), (4097, 259, 256), (240000, 256, 512), (8, 256, 512)])
def test_linear_wgrad_bf16_vs_float64(H, M, I, O, half):
    g = torch.Generator(device="cuda").manual_seed(M * 3 + I + O)
    dz = torch.randn(M, O, device="cuda", generator=g)
    x = torch.randn(M, I, device="cuda", generator=g)
    dw, db = H.linear_wgrad(dz, x, bias=True, bf16=True, half=half)
    ref = _bf(dz, half).t() @ _bf(x, half)
    assert ((dw.double() - ref).norm() / ref.norm()).item() < 1e-6
    ref_b = dz.double().sum(0)
    assert ((db.double() - ref_b).norm() / ref_b.norm()).item() < 1e-6
    dw2, _ = H.linear_wgrad(dz, x, bias=False, bf16=True, half=half)
    assert torch.equal(dw, dw2)


@pytest.mark.parametrize("half", HALVES, ids=HALF_IDS)
def test_linear_fn_uses_bf16_under_autocast(H, half):
    """LinearFn under autocast runs the 16-bit GEMMs in autocast's dtype: the output matches
    the float64 product of operands rounded to THAT dtype (and not the other one)."""
    from pointcloud_style_transfer_amd.models import _autograd as ag

    torch.manual_seed(1)
    lin = torch.nn.Linear(256, 512).cuda()
    x = torch.randn(3000, 256, device="cuda", requires_grad=True)
    with torch.autocast("cuda", dtype=half):
        y = ag.linear(x, lin, relu=True)
    other = torch.float16 if half == torch.bfloat16 else torch.bfloat16
    rounded = lambda h: (_bf(x.detach(), h) @ _bf(lin.weight.detach(), h).t()  # noqa: E731
                         + lin.bias.detach().double()).clamp_min(0)
    r_own, r_other = rounded(half), rounded(other)
    assert (y.double() - r_own).norm() < 1e-5 * r_own.norm()
    assert (y.double() - r_other).norm() > 1e-4 * r_own.norm()
    assert y.dtype == torch.float32
    y.sum().backward()
    x64 = x.detach().double().requires_grad_()
    w64 = lin.weight.detach().double().requires_grad_()
    y64 = torch.relu(x64 @ w64.t() + lin.bias.detach().double())
    y64.sum().backward()
    rel = lambda a, b: ((a.double() - b).norm() / b.norm()).item()  # noqa: E731
    assert 1e-7 < rel(y, y64) < 1e-2          # 16-bit operands: not the f32 path, within their error
    # backward products against float64 with the kernel's own ReLU mask (16-bit rounding flips
    # the mask of near-zero pre-activations; that is not a GEMM error)
    mask = (y.detach() > 0).double()
    assert rel(x.grad, mask @ w64.detach()) < 1e-2
    assert rel(lin.weight.grad, mask.t() @ x64.detach()) < 1e-2


def test_trainer_step_amp_close_to_fp32(H, tmp_path):
    """One DiffusionTrainer step with use_amp (bf16 GEMMs) against the same step in fp32:
    same draws, losses within the bf16 tolerance."""
    import numpy as np

    from pointcloud_style_transfer_amd.config.config import Config
    from pointcloud_style_transfer_amd.synthetic import lidar_like_cloud
    from pointcloud_style_transfer_amd.training.trainer import DiffusionTrainer

    losses = []
    for amp in (False, True):
        cfg = Config(make_dirs=False, log_dir=str(tmp_path), checkpoint_dir=str(tmp_path),
                     use_amp=amp, gradient_accumulation_steps=1, cond_drop_prob=0.0,
                     global_points=2048)
        torch.manual_seed(0)
        tr = DiffusionTrainer(cfg, device="cuda")
        tr.model.train()
        sim = torch.from_numpy(np.stack([lidar_like_cloud(1000 + i, 8192) for i in range(2)]))
        real = torch.from_numpy(np.stack([lidar_like_cloud(2000 + i, 8192) for i in range(2)]))
        torch.manual_seed(5)
        loss, _ = tr.train_step({"sim_full": sim.cuda(), "real_full": real.cuda()}, 0, 1)
        losses.append(float(loss))
    assert np.isfinite(losses).all()
    assert abs(losses[1] - losses[0]) <= 2e-2 * abs(losses[0]), losses


def test_relu_bwd_matches_torch(H):
    g = torch.Generator(device="cuda").manual_seed(3)
    for n in (1, 7, 4096, 1000003):
        dy = torch.randn(n, device="cuda", generator=g)
        y = torch.randn(n, device="cuda", generator=g).clamp_min(0)
        assert torch.equal(H.relu_bwd(dy, y), dy * (y > 0))


@pytest.mark.parametrize("M,O,ns", [(1024, 64, 0), (131072, 64, 0), (131072, 128, 32),
                                    (65536, 256, 64), (1024, 256, 128), (96, 3, 32)])
def test_bn_relu_fn_vs_torch_float64(H, M, O, ns):
    """BNReLUFn (train-mode BatchNorm + ReLU (+ max over ns rows), csrc/sa_train.hip) against
    torch's F.batch_norm(training=True) / relu / max in float64 with autograd, same upstream
    gradient: outputs and dZ / dgamma / dbeta within fp32 rounding of the float64 result, the
    running statistics updated as BatchNorm2d does, and the backward deterministic."""
    import torch.nn.functional as F

    from pointcloud_style_transfer_amd.models import _autograd as ag

    g = torch.Generator(device="cuda").manual_seed(M + O + ns)
    z = (torch.randn(M, O, device="cuda", generator=g) * 2 + 0.3).requires_grad_()
    bn = torch.nn.BatchNorm2d(O).cuda().train()
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5, generator=g)
        bn.bias.uniform_(-0.2, 0.2, generator=g)
        bn.running_mean.uniform_(-0.1, 0.1, generator=g)
    rm0, rv0 = bn.running_mean.clone(), bn.running_var.clone()
    y = ag.bn_relu(z, bn, ns)
    gy = torch.randn(y.shape, device="cuda", generator=g)
    y.backward(gy)
    z64 = z.detach().double().requires_grad_()
    w64 = bn.weight.detach().double().requires_grad_()
    b64 = bn.bias.detach().double().requires_grad_()
    rm, rv = rm0.double().clone(), rv0.double().clone()
    y64 = torch.relu(F.batch_norm(z64, rm, rv, w64, b64, True, 0.1, bn.eps))
    if ns:
        y64 = y64.view(-1, ns, O).max(dim=1)[0]
    y64.backward(gy.double())
    rel = lambda a, b: ((a.double() - b).norm() / b.norm().clamp_min(1e-300)).item()  # noqa: E731
    assert rel(y.detach(), y64.detach()) < 1e-6
    assert rel(z.grad, z64.grad) < 1e-5
    assert rel(bn.weight.grad, w64.grad) < 1e-5
    assert rel(bn.bias.grad, b64.grad) < 1e-5
    assert rel(bn.running_mean, rm) < 1e-6 and rel(bn.running_var, rv) < 1e-6
    assert int(bn.num_batches_tracked) == 1
    gz = z.grad.clone()
    z.grad = None
    ag.bn_relu(z, bn, ns).backward(gy)
    assert torch.equal(z.grad, gz), "bn_relu backward must be deterministic"


@pytest.mark.parametrize("B,N,C,S,ns", [(8, 512, 128, 128, 64), (2, 30, 5, 7, 16), (1, 1, 64, 3, 4)])
def test_group_gather_fn_backward(H, B, N, C, S, ns):
    """GroupGatherFn's scatter backward (pcst_group_gather_bwd) equals torch's advanced-index
    backward in float64 (the reference's points[batch, idx] gather, pointnet2_encoder.py:20-28,
    99), including clamped out-of-range indices (the ball query's pad value N), and is
    bit-deterministic."""
    from pointcloud_style_transfer_amd.models import _autograd as ag

    g = torch.Generator(device="cuda").manual_seed(B * N + C)
    xyz = torch.randn(B, N, 3, device="cuda", generator=g)
    pts = torch.randn(B, N, C, device="cuda", generator=g).requires_grad_()
    fidx = torch.randint(0, N, (B, S), device="cuda", generator=g)
    gidx = torch.randint(0, N + 1, (B, S, ns), device="cuda", generator=g)   # N -> clamped
    gidx[:, :, 1] = gidx[:, :, 0]   # repeated indices inside a group (the pad)
    new_xyz, grouped = ag.GroupGatherFn.apply(xyz, pts, fidx, gidx)
    gg = torch.randn(grouped.shape, device="cuda", generator=g)
    grouped.backward(gg)
    p64 = pts.detach().double().requires_grad_()
    bidx = torch.arange(B, device="cuda").view(B, 1, 1)
    p64[bidx, gidx.clamp(0, N - 1)].backward(gg[..., 3:].double())
    err = (pts.grad.double() - p64.grad).abs().max().item()
    assert err <= 1e-5 * max(1.0, p64.grad.abs().max().item())
    first = pts.grad.clone()
    pts.grad = None
    ag.GroupGatherFn.apply(xyz, pts, fidx, gidx)[1].backward(gg)
    assert torch.equal(pts.grad, first)


# ---- csrc/train_mlp.hip: bf16-storage GEMMs with fused epilogues --------------------------
def _bf16_ulp_close(a, b, ulps=1.0):
    """16-bit outputs: within `ulps` units in the last place of the reference (an ulp of x is
    at most |x| * 2^-7 for bfloat16's 8 significant bits, |x| * 2^-10 for float16's 11)."""
    rel = 2.0 ** -10 if a.dtype == torch.float16 else 2.0 ** -7
    a, b = a.double(), b.double()
    return ((a - b).abs() <= ulps * (b.abs() * rel + 1e-30) + 1e-6 * b.abs().max()).all().item()


@pytest.mark.parametrize("half", HALVES, ids=HALF_IDS)
@pytest.mark.parametrize("M,K,O", [(1, 128, 128), (1000, 256, 512), (4097, 512, 256), (300, 136, 260),
                                   (60000, 256, 512)])
@pytest.mark.parametrize("a16,b16", [(False, False), (True, False), (True, True)])
def test_gemm_ex_epilogues_vs_float64(H, M, K, O, a16, b16, half):
    g = torch.Generator(device="cuda").manual_seed(M + K + O + 7 * a16 + 3 * b16)
    A = torch.randn(M, K, device="cuda", generator=g)
    B = torch.randn(O, K, device="cuda", generator=g) * K ** -0.5
    bias = torch.randn(O, device="cuda", generator=g)
    Ain = A.to(half) if a16 else A
    Bin = B.to(half) if b16 else B
    acc = _bf(A, half) @ _bf(B, half).t()
    tol = lambda ref: 1e-6 * ref.norm().item()  # noqa: E731  fp32 summation order
    # EP_F32 / EP_BF16 with bias + relu
    C = H.gemm_ex(Ain, Bin, bias, relu=True, epilogue=H.EP_F32, half=half)
    ref = (acc + bias.double()).clamp_min(0)
    assert (C.double() - ref).norm().item() <= tol(ref)
    Cb = H.gemm_ex(Ain, Bin, bias, relu=True, epilogue=H.EP_BF16, half=half)
    assert Cb.dtype == half and _bf16_ulp_close(Cb, ref)
    # EP_F32 with the 16-bit copy (EP_COND's copy path uses the same conversion)
    C, C2 = H.gemm_ex(Ain, Bin, bias, epilogue=H.EP_F32, copy_bf16=True, half=half)
    assert C2.dtype == half and torch.equal(C2, C.to(half))
    # EP_ADD
    aux = torch.randn(M, O, device="cuda", generator=g)
    C = H.gemm_ex(Ain, Bin, epilogue=H.EP_ADD, aux=aux, half=half)
    ref = acc + aux.double()
    assert (C.double() - ref).norm().item() <= tol(ref)
    # EP_RELU_MASK: zero where the bf16 mask is <= 0 (including exact zeros)
    h = torch.randn(M, O, device="cuda", generator=g)
    h[:, ::7] = 0.0
    h = h.to(half)
    C = H.gemm_ex(Ain, Bin, epilogue=H.EP_RELU_MASK, aux=h)
    ref = acc * (h.double() > 0)
    assert C.dtype == half and _bf16_ulp_close(C, ref)
    assert torch.equal(C == 0, (h <= 0) | (C == 0))


@pytest.mark.parametrize("half", HALVES, ids=HALF_IDS)
@pytest.mark.parametrize("M,K,O", [(1, 128, 128), (4097, 512, 256), (300, 136, 260), (60000, 256, 512)])
@pytest.mark.parametrize("p", [0.0, 0.3])
def test_gemm_ex_16bit_residual_epilogues(H, M, K, O, p, half):
    """EP_RESID_DROP16 / EP_ADD16 (16-bit residual operand and output) against float64 products
    of the rounded operands; the dropout copy of EP_BF16 / EP_ADD16 equals dropout_grad_bf16 of
    the stored 16-bit output bit for bit; EP_COND's 16-bit-only output equals its copy."""
    g = torch.Generator(device="cuda").manual_seed(M + K + O + int(10 * p))
    A = torch.randn(M, K, device="cuda", generator=g).to(half)
    B = (torch.randn(O, K, device="cuda", generator=g) * K ** -0.5).to(half)
    bias = torch.randn(O, device="cuda", generator=g)
    acc = A.double() @ B.double().t()
    x16 = torch.randn(M, O, device="cuda", generator=g).to(half)
    seed = 0x0DDB_A11_5EED + M
    y = H.gemm_ex(A, B, bias, epilogue=H.EP_RESID_DROP16, aux=x16, seed=seed, p=p)
    keep = (H.dropout_grad_bf16(torch.ones(M, O, device="cuda"), seed, p, half=half) != 0).double()
    ref = x16.double() + keep * (acc + bias.double()) / (1.0 - p)
    assert y.dtype == half and _bf16_ulp_close(y, ref)
    assert torch.equal(H.gemm_ex(A, B, bias, epilogue=H.EP_RESID_DROP16, aux=x16, seed=seed, p=p), y)
    gx = H.gemm_ex(A, B, epilogue=H.EP_ADD16, aux=x16)
    assert gx.dtype == half and _bf16_ulp_close(gx, acc + x16.double())
    for ep, aux in ((H.EP_ADD16, x16), (H.EP_BF16, None)):
        c, dd = H.gemm_ex(A, B, epilogue=ep, aux=aux, seed=seed, p=p, dropout_copy=True)
        assert torch.equal(c, H.gemm_ex(A, B, epilogue=ep, aux=aux))
        assert torch.equal(dd, H.dropout_grad_bf16(c.float(), seed, p, half=half))
    if O % 4 == 0 and M % 3 == 0:
        cond = torch.randn(M // 3, 2, O, device="cuda", generator=g)
        c32, c16 = H.gemm_ex(A, B, bias, epilogue=H.EP_COND, aux=cond, group_rows=3, copy_bf16=True)
        only = H.gemm_ex(A, B, bias, epilogue=H.EP_COND, aux=cond, group_rows=3, copy_bf16=True,
                         fp32_out=False)
        assert torch.equal(only, c16)


@pytest.mark.parametrize("half", HALVES, ids=HALF_IDS)
def test_noise_predictor_16bit_residual_matches_fp32_residual(H, half, monkeypatch):
    """NoisePredictorFn with the 16-bit residual stream (default) against the fp32-stream
    layout, dropout on (the same seeds): forward and every gradient within 16-bit storage
    error of the residual stream."""
    from pointcloud_style_transfer_amd.config.config import Config
    from pointcloud_style_transfer_amd.models import _autograd as ag
    from pointcloud_style_transfer_amd.models.diffusion_model import NoisePredictor

    torch.manual_seed(0)
    npred = NoisePredictor(Config(make_dirs=False)).cuda().train()
    x = torch.randn(2, 4000, 3, device="cuda")
    t = torch.tensor([10, 500], device="cuda")
    sf = torch.randn(2, 256, device="cuda")
    outs, grads = [], []
    for r16 in (True, False):
        monkeypatch.setattr(ag, "RESIDUAL_16BIT", r16)
        npred.zero_grad()
        torch.manual_seed(5)  # the same dropout seeds
        with torch.autocast("cuda", dtype=half):
            out = npred(x, t, sf)
        out.float().pow(2).sum().backward()
        outs.append(out.detach().float())
        grads.append([p.grad.detach().clone() for p in npred.parameters()])
    rel = lambda a, b: ((a.double() - b.double()).norm() / b.double().norm()).item()  # noqa: E731
    tol = 2e-2 if half == torch.bfloat16 else 4e-3
    assert rel(outs[0], outs[1]) < tol
    for a, b in zip(grads[0], grads[1]):
        assert rel(a, b) < 2.5 * tol


@pytest.mark.parametrize("half", HALVES, ids=HALF_IDS)
@pytest.mark.parametrize("p", [0.0, 0.1, 0.5])
def test_gemm_ex_dropout_mask_fwd_bwd_consistent(H, p, half):
    """EP_RESID_DROP keeps element e iff hash(seed, e) passes; pcst_dropout_grad_bf16 must
    regenerate the same mask (read off dropout_grad of ones), the forward must equal
    x + keep * (acc + b) / (1-p), and the kept fraction must be 1-p."""
    M, K, O = 20000, 256, 256
    g = torch.Generator(device="cuda").manual_seed(11)
    h = torch.randn(M, K, device="cuda", generator=g).to(half)
    W = torch.randn(O, K, device="cuda", generator=g) * K ** -0.5
    b = torch.randn(O, device="cuda", generator=g)
    x = torch.randn(M, O, device="cuda", generator=g)
    seed = 0x1234_5678_9ABC_DEF
    y = H.gemm_ex(h, W, b, epilogue=H.EP_RESID_DROP, aux=x, seed=seed, p=p)
    keep = H.dropout_grad_bf16(torch.ones(M, O, device="cuda"), seed, p, half=half) != 0
    frac = keep.double().mean().item()
    assert abs(frac - (1 - p)) < 4 * np.sqrt(p * (1 - p) / (M * O)) + 1e-12
    v = _bf(h, half) @ _bf(W, half).t() + b.double()
    ref = x.double() + keep.double() * v * (1.0 / (1.0 - p))
    assert ((y.double() - ref).norm() / ref.norm()).item() < 1e-6
    assert torch.equal(y[~keep], x[~keep])  # dropped elements are exactly the residual
    y2 = H.gemm_ex(h, W, b, epilogue=H.EP_RESID_DROP, aux=x, seed=seed, p=p)
    assert torch.equal(y, y2)
    if p > 0:
        y3 = H.gemm_ex(h, W, b, epilogue=H.EP_RESID_DROP, aux=x, seed=seed + 1, p=p)
        assert not torch.equal(y, y3)
    gd = torch.randn(M, O, device="cuda", generator=g)
    dd = H.dropout_grad_bf16(gd, seed, p, half=half)
    assert dd.dtype == half
    assert _bf16_ulp_close(dd, gd.double() * keep.double() / (1.0 - p), 0.5)


@pytest.mark.parametrize("M,I,O", [(1, 256, 512), (100, 136, 264), (5000, 512, 256), (240000, 256, 512),
                                   (240000, 512, 256)])
@pytest.mark.parametrize("z16,x16", [(True, True), (True, False), (False, False)])
@pytest.mark.parametrize("half", HALVES, ids=HALF_IDS)
def test_linear_wgrad_ex_vs_float64(H, M, I, O, z16, x16, half):
    g = torch.Generator(device="cuda").manual_seed(M + I + 3 * O + z16 + 2 * x16)
    dz = torch.randn(M, O, device="cuda", generator=g)
    x = torch.randn(M, I, device="cuda", generator=g)
    dzi = dz.to(half) if z16 else dz
    xi = x.to(half) if x16 else x
    dw, db = H.linear_wgrad_ex(dzi, xi, bias=True, half=half)
    ref = _bf(dz, half).t() @ _bf(x, half)
    assert ((dw.double() - ref).norm() / ref.norm()).item() < 1e-6
    ref_b = dzi.double().sum(0)  # bias from the operand as stored (bf16 values or fp32)
    assert ((db.double() - ref_b).abs().max() / ref_b.abs().max()).item() < 1e-5
    dw2, db2 = H.linear_wgrad_ex(dzi, xi, bias=True, half=half)
    assert torch.equal(dw, dw2) and torch.equal(db, db2), "must be deterministic"


@pytest.mark.parametrize("p", [0.0, 0.1])
def test_residual_block_fn_vs_float64(H, p):
    """ResidualBlockFn forward and backward against a float64 restatement with the kernel's
    roundings (bf16 operands, bf16 h/dd/dz storage) and the kernel's own dropout mask."""
    from pointcloud_style_transfer_amd.models import _autograd as ag

    torch.manual_seed(3)
    layer = torch.nn.Sequential(torch.nn.Linear(256, 512), torch.nn.ReLU(), torch.nn.Linear(512, 256),
                                torch.nn.Dropout(p)).cuda()
    x = torch.randn(4, 3000, 256, device="cuda", requires_grad=True)
    torch.manual_seed(9)
    y = ag.residual_block(x, layer, training=True)
    gy = torch.randn_like(y)
    y.backward(gy)
    torch.manual_seed(9)
    seed = int(torch.randint(0, 2 ** 62, (1,)).item()) if p > 0 else 0
    M = x.numel() // 256
    keep = (H.dropout_grad_bf16(torch.ones(M, 256, device="cuda"), seed, p) != 0).double()
    s = 1.0 / (1.0 - p)
    w1, b1 = layer[0].weight.detach(), layer[0].bias.detach().double()
    w2, b2 = layer[2].weight.detach(), layer[2].bias.detach().double()
    x2 = x.detach().reshape(M, 256)
    h = (_bf(x2) @ _bf(w1).t() + b1).clamp_min(0)
    hb = h.bfloat16().double()
    y_ref = x2.double() + keep * (hb @ _bf(w2).t() + b2) * s
    rel = lambda a, b: ((a.double() - b).norm() / b.norm()).item()  # noqa: E731
    assert rel(y.detach().reshape(M, 256), y_ref) < 1e-5
    g = gy.reshape(M, 256).double()
    dd = (g * keep * s).float().bfloat16().double()
    dz = ((dd @ _bf(w2)) * (hb > 0)).float().bfloat16().double()
    gx = g + dz @ _bf(w1)
    assert rel(x.grad.reshape(M, 256), gx) < 1e-3
    assert rel(layer[2].weight.grad, dd.t() @ hb) < 1e-3
    assert rel(layer[2].bias.grad, dd.sum(0)) < 1e-3
    assert rel(layer[0].weight.grad, dz.t() @ _bf(x2)) < 1e-3
    assert rel(layer[0].bias.grad, dz.sum(0)) < 1e-3


def test_noise_predictor_fused_blocks_match_unfused(H):
    """Under autocast with dropout off, the fused residual blocks give the same forward and
    gradients as the per-linear LinearFn path within bf16 storage error."""
    from pointcloud_style_transfer_amd.config.config import Config
    from pointcloud_style_transfer_amd.models.diffusion_model import NoisePredictor

    torch.manual_seed(0)
    npred = NoisePredictor(Config(make_dirs=False)).cuda().train()
    for l in npred.layers:
        l[3].p = 0.0
    x = torch.randn(2, 4000, 3, device="cuda")
    t = torch.tensor([10, 500], device="cuda")
    sf = torch.randn(2, 256, device="cuda")
    outs, grads = [], []
    for fused in (True, False):
        npred.zero_grad()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            out = npred(x, t, sf) if fused else _unfused_forward(npred, x, t, sf)
        out.float().pow(2).sum().backward()
        outs.append(out.detach().float())
        grads.append([p.grad.detach().clone() for p in npred.parameters()])
    rel = lambda a, b: ((a.double() - b.double()).norm() / b.double().norm()).item()  # noqa: E731
    assert rel(outs[0], outs[1]) < 2e-2
    for a, b in zip(grads[0], grads[1]):
        assert rel(a, b) < 5e-2


def test_noise_predictor_row_limit_fallback_bit_identical(H, monkeypatch):
    """Batches beyond the fused residual-block kernels' row limit take the two-GEMM path
    (models/_autograd.py fused_block_rows_ok); with the limit lowered below this batch
    the forward and every gradient are the bits of the fused path (dropout on: the same draws)."""
    from pointcloud_style_transfer_amd.config.config import Config
    from pointcloud_style_transfer_amd.models import _autograd as ag
    from pointcloud_style_transfer_amd.models.diffusion_model import NoisePredictor

    torch.manual_seed(0)
    npred = NoisePredictor(Config(make_dirs=False)).cuda().train()
    x = torch.randn(2, 3000, 3, device="cuda")
    t = torch.tensor([10, 500], device="cuda")
    sf = torch.randn(2, 256, device="cuda")
    outs, grads = [], []
    for lim in (ag.FUSED_BLOCK_MAX_ROWS, 5999):   # 6000 rows: fused, then over the limit
        monkeypatch.setattr(ag, "FUSED_BLOCK_MAX_ROWS", lim)
        npred.zero_grad()
        torch.manual_seed(3)  # the dropout seeds
        with torch.autocast("cuda", dtype=torch.float16):
            out = npred(x, t, sf)
        out.float().pow(2).sum().backward()
        outs.append(out.detach().clone())
        grads.append([p.grad.detach().clone() for p in npred.parameters()])
    assert torch.equal(outs[0], outs[1])
    for a, b in zip(grads[0], grads[1]):
        assert torch.equal(a, b)


def _unfused_forward(npred, noisy_points, timestep, style_feat):
    from pointcloud_style_transfer_amd.models import _autograd as ag

    pe = npred.point_encoder
    h = ag.linear(noisy_points, pe[0], True)
    h = ag.linear(h, pe[2], True)
    pf = ag.linear(h, pe[4])
    tf = ag.linear(npred.time_embedding(timestep), npred.time_proj)
    sf = ag.linear(style_feat, npred.style_proj)
    x = pf + tf.unsqueeze(1) + sf.unsqueeze(1)
    for layer in npred.layers:
        x = ag.linear(ag.linear(x, layer[0], True), layer[2]) + x
    h = ag.linear(x, npred.output_mlp[0], True)
    h = ag.linear(h, npred.output_mlp[2], True)
    return ag.linear(h, npred.output_mlp[4])


@pytest.mark.parametrize("B,N,C", [(8, 30000, 256), (1, 1, 8), (3, 1001, 264), (2, 7, 256)])
@pytest.mark.parametrize("half", [torch.float16, torch.bfloat16])
def test_group_colsum16_vs_float64(H, B, N, C, half):
    """pcst_group_colsum16 (NoisePredictorFn's dL/dtf = dL/dsf, no hipBLASLt GEMV): each cloud's
    column sums in float, rounded to the 16-bit type.  Against the float64 sum of the same 16-bit
    values rounded the same way: within one 16-bit step of the result plus the float32
    summation bound (N * 2^-24 * sum|g| per column, which matters only where the sum cancels);
    mostly bit-equal; deterministic."""
    torch.manual_seed(B * 1000 + N + C)
    g = (torch.randn(B * N, C, device="cuda") * 0.01).to(half)
    out = H.group_colsum16(g, B)
    ref = g.double().view(B, N, C).sum(1).to(half).float()
    assert out.shape == (B, C) and out.dtype == torch.float32
    step = torch.finfo(half).eps * ref.abs().clamp_min(torch.finfo(half).tiny)
    f32_bound = N * 2.0 ** -24 * g.double().abs().view(B, N, C).sum(1).float()
    assert bool(((out - ref).abs() <= step + 2 * f32_bound).all())
    assert bool((out == ref).double().mean() >= 0.95)
    assert torch.equal(out, H.group_colsum16(g, B))


@pytest.mark.parametrize("M", [240000, 1000, 129, 1])
@pytest.mark.parametrize("p", [0.0, 0.3])
@pytest.mark.parametrize("half", [torch.float16, torch.bfloat16])
def test_resblock_fwd16_matches_two_gemms(H, M, p, half):
    """pcst_resblock_fwd16 (one residual block forward, h never re-read) gives the bits of
    gemm_ex EP_BF16 followed by EP_RESID_DROP16 with the same (seed, p): h and x' bit-equal, for
    ragged M, with and without dropout, in both 16-bit formats."""
    torch.manual_seed(M + int(p * 10))
    x = (torch.randn(M, 256, device="cuda")).to(half)
    w1 = (torch.randn(512, 256, device="cuda") * 0.06).to(half)
    w2 = (torch.randn(256, 512, device="cuda") * 0.04).to(half)
    b1 = torch.randn(512, device="cuda") * 0.1
    b2 = torch.randn(256, device="cuda") * 0.1
    seed = 123456789123
    h_ref = H.gemm_ex(x, w1, b1, relu=True, epilogue=H.EP_BF16)
    x_ref = H.gemm_ex(h_ref, w2, b2, epilogue=H.EP_RESID_DROP16, aux=x, seed=seed, p=p)
    h, xo = H.resblock_fwd16(x, w1, b1, w2, b2, seed=seed, p=p)
    assert h.dtype == half and xo.dtype == half
    assert torch.equal(h, h_ref)
    assert torch.equal(xo, x_ref)


@pytest.mark.parametrize("M", [240000, 1000, 129, 1])
@pytest.mark.parametrize("p", [0.0, 0.3])
@pytest.mark.parametrize("half", [torch.float16, torch.bfloat16])
def test_resblock_bwd16_matches_two_gemms(H, M, p, half):
    """pcst_resblock_bwd16 (one residual block's backward products, dZ never re-read) gives the
    bits of gemm_ex EP_RELU_MASK (aux h) followed by EP_ADD16 (aux g) with the previous block's
    dropout copy under the same (seed, p): dZ, g' and dD' bit-equal, for ragged M, with and
    without dropout, in both 16-bit formats; without the copy dD' is None."""
    torch.manual_seed(M + int(p * 10) + 7)
    dd = (torch.randn(M, 256, device="cuda")).to(half)
    h = torch.relu(torch.randn(M, 512, device="cuda")).to(half)
    g = (torch.randn(M, 256, device="cuda")).to(half)
    w2t = (torch.randn(512, 256, device="cuda") * 0.04).to(half)
    w1t = (torch.randn(256, 512, device="cuda") * 0.06).to(half)
    seed = 987654321987
    dz_ref = H.gemm_ex(dd, w2t, epilogue=H.EP_RELU_MASK, aux=h)
    g_ref, dd_ref = H.gemm_ex(dz_ref, w1t, epilogue=H.EP_ADD16, aux=g, seed=seed, p=p,
                              dropout_copy=True)
    dz, g2, dd2 = H.resblock_bwd16(dd, w2t, w1t, h, g, seed=seed, p=p, dropout_copy=True)
    assert dz.dtype == half and g2.dtype == half and dd2.dtype == half
    assert torch.equal(dz, dz_ref)
    assert torch.equal(g2, g_ref)
    assert torch.equal(dd2, dd_ref)
    dz3, g3, none = H.resblock_bwd16(dd, w2t, w1t, h, g)
    assert none is None and torch.equal(dz3, dz_ref)
    assert torch.equal(g3, H.gemm_ex(dz_ref, w1t, epilogue=H.EP_ADD16, aux=g))


@pytest.mark.parametrize("half", [torch.float16, torch.bfloat16])
def test_cast16_batch_matches_per_tensor_casts(H, half):
    """pcst_cast16_batch (a layer stack's 16-bit weight copies in one launch) gives the bits of
    t.to(half) and t.t().to(half) for every tensor, ragged shapes included (odd sizes, one row,
    an empty tensor), with values that round, overflow float16 and underflow to subnormals."""
    torch.manual_seed(11)
    shapes = [(512, 256), (256, 512), (8, 128), (3, 5), (1, 7), (0, 4), (259, 33), (128, 3)]
    ts = [torch.randn(r, c, device="cuda") * 10.0 ** (i - 3) for i, (r, c) in enumerate(shapes)]
    ts[1][0, :4] = torch.tensor([7e4, -7e4, 1e-8, float("inf")], device="cuda")
    flags = [i % 2 == 1 for i in range(len(ts))]
    outs = H.cast16_batch(ts, half, flags)
    for t, o, tr in zip(ts, outs, flags):
        ref = (t.t() if tr else t).to(half).contiguous()
        assert o.dtype == half and o.shape == ref.shape and o.is_contiguous()
        assert torch.equal(o.view(torch.int16), ref.view(torch.int16))
    plain = H.cast16_batch(ts[:3], half)
    assert all(torch.equal(o, t.to(half)) for o, t in zip(plain, ts[:3]))


@pytest.mark.parametrize("O", [64, 128, 3])
def test_bn_train_stats_matches_stats_then_coeffs(H, O):
    """pcst_bn_train_stats (statistics + coefficients in two launches) gives the bits of
    pcst_channel_stats followed by pcst_bn_train_coeffs: mean / var, scale / shift / invstd and
    the running-stat update, with and without running stats, vectorised and scalar channel
    counts."""
    torch.manual_seed(O)
    M = 40961
    z = torch.randn(M, O, device="cuda") * 3.0 + 0.5
    g = torch.rand(O, device="cuda") + 0.5
    b = torch.randn(O, device="cuda")
    for with_run in (True, False):
        rm1 = torch.randn(O, device="cuda") if with_run else None
        rv1 = (torch.rand(O, device="cuda") + 0.1) if with_run else None
        rm2 = rm1.clone() if with_run else None
        rv2 = rv1.clone() if with_run else None
        mean, var = H.channel_stats(z)
        ref = H.bn_train_coeffs(mean, var, M, g, b, 1e-5, 0.1, rm1, rv1)
        got = H.bn_train_stats(z, g, b, 1e-5, 0.1, rm2, rv2)
        for x, y in zip((mean, var) + tuple(ref), got):
            assert torch.equal(x, y)
        if with_run:
            assert torch.equal(rm1, rm2) and torch.equal(rv1, rv2)


@pytest.mark.parametrize("M", [240000, 1000, 129, 1])
@pytest.mark.parametrize("half", [torch.float16, torch.bfloat16])
def test_resblock_mask_bits(H, M, half):
    """resblock_fwd16(mask_bits=True) writes bit j of word w of row m = [h[m, 32w + j] > 0] of the
    h it returns (h and x' unchanged), and resblock_bwd16(hbits=) -- the mask from those bits,
    h not read -- gives the bits of the h-mask backward, ragged M included."""
    torch.manual_seed(M + 3)
    x = torch.randn(M, 256, device="cuda").to(half)
    w1 = (torch.randn(512, 256, device="cuda") * 0.06).to(half)
    w2 = (torch.randn(256, 512, device="cuda") * 0.04).to(half)
    b1 = torch.randn(512, device="cuda") * 0.1
    b2 = torch.randn(256, device="cuda") * 0.1
    h_ref, xo_ref = H.resblock_fwd16(x, w1, b1, w2, b2, seed=11, p=0.2)
    h, xo, bits = H.resblock_fwd16(x, w1, b1, w2, b2, seed=11, p=0.2, mask_bits=True)
    assert torch.equal(h, h_ref) and torch.equal(xo, xo_ref)
    pos = (h.view(torch.int16) > 0).view(M, 16, 32).to(torch.int64)
    want = (pos << torch.arange(32, device="cuda")).sum(-1)
    assert torch.equal(bits.to(torch.int64) & 0xFFFFFFFF, want & 0xFFFFFFFF)
    dd = torch.randn(M, 256, device="cuda").to(half)
    g = torch.randn(M, 256, device="cuda").to(half)
    w2t, w1t = w2.t().contiguous(), w1.t().contiguous()
    ref = H.resblock_bwd16(dd, w2t, w1t, h, g, seed=5, p=0.3, dropout_copy=True)
    got = H.resblock_bwd16(dd, w2t, w1t, None, g, seed=5, p=0.3, dropout_copy=True, hbits=bits)
    for a, b in zip(ref, got):
        assert torch.equal(a, b)
