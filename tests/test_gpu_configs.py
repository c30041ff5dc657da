"""BASELINE configs at their own sizes on one MI355X:

  configs[2]  DiffusionTrainer.train_step on 8 x 120k-point clouds under use_amp (16-bit MFMA
              GEMMs, fp16 by default as the reference, and bf16) against the same step in
              exact f32, same draws (rng.CounterRNG);
  configs[4]  the per-GPU share of the 256-cloud batch inference: 32 x 120k clouds through the
              hipGraph-captured guided step vs the eager loop; the device-drawn voxel subset of
              all 64 CFG rows (every representative kept, pad points distinct); and one
              replayed step of the 32-cloud batch against the oracle;
  configs[1]  the bf16 noise MLP per element at 60000 points (2 x 30000, the measured launch)
              and the 120k-point Chamfer-vs-oracle quality of a 10-step loop (bench.py reports
              the 50-step figure).
Reference semantics: /root/reference/training/trainer.py:70-127,
/root/reference/models/diffusion_model.py:64-153,224-261.
"""
import re

import numpy as np
import pytest
import torch

from conftest import assert_close

pytestmark = pytest.mark.gpu

PRE_BN_BIAS = re.compile(r"style_encoder\.encoder\.sa\d\.mlp_convs\.\d+\.bias$")


def _clouds(seed0, n, points):
    from pointcloud_style_transfer_amd.synthetic import lidar_like_cloud

    return torch.from_numpy(np.stack([lidar_like_cloud(seed0 + i, points) for i in range(n)]))


def _trainer_step_grads(tmp_path, sim, real, amp, lambda_chamfer, amp_dtype="float16"):
    """One DiffusionTrainer.train_step with counter-keyed draws and dropout off -> (loss, the
    gradient as the step computed it, before clipping)."""
    from pointcloud_style_transfer_amd import rng
    from pointcloud_style_transfer_amd.config.config import Config
    from pointcloud_style_transfer_amd.training import trainer as T

    cfg = Config(make_dirs=False, log_dir=str(tmp_path), checkpoint_dir=str(tmp_path),
                 use_amp=amp, gradient_accumulation_steps=1, batch_size=8,
                 lambda_chamfer=lambda_chamfer, amp_dtype=amp_dtype)
    torch.manual_seed(0)
    tr = T.DiffusionTrainer(cfg, device="cuda")
    tr.model.train()
    for m in tr.model.modules():
        if isinstance(m, torch.nn.Dropout):
            m.p = 0.0
    if not amp or amp_dtype == "bfloat16":
        tr.scaler = torch.amp.GradScaler(enabled=False)  # compare unscaled gradients
    else:
        # fp16 (the reference's autocast) needs the loss scale: the L1 gradient 1/numel sits
        # in fp16's subnormal range.  Fixed scale; unscale_ (before the snapshot) is exact
        tr.scaler = torch.amp.GradScaler(init_scale=2.0 ** 14, growth_interval=10 ** 9)
    grads = {}
    clip = torch.nn.utils.clip_grad_norm_

    def snap(params, *a, **k):
        params = list(params)
        for n, p in tr.model.named_parameters():
            grads[n] = p.grad.detach().double().clone()
        return clip(params, *a, **k)

    torch.nn.utils.clip_grad_norm_ = snap
    try:
        with rng.replay(rng.CounterRNG(4000)):
            loss, _ = tr.train_step({"sim_full": sim, "real_full": real}, 0, 1)
    finally:
        torch.nn.utils.clip_grad_norm_ = clip
    return float(loss.detach()), grads


def test_trainer_step_8x120k_amp_vs_fp32(tmp_path):
    """configs[2]: one trainer step at B = 8 x 120000 under use_amp (16-bit GEMMs: fp16, the
    default, and bf16) and in f32, same draws, dropout off: losses finite, within 2e-2
    relative, gradient norms (before clipping) within 10 %.  The gradient DIRECTION is not a bf16-vs-f32 invariant of this
    loss: L1's gradient is sign(eps_hat - eps) (bf16 rounding flips the sign of the ~0.4 % of
    elements within its error: |dg|/|g| ~ 2 sqrt(0.004) ~ 0.13) and the Chamfer term acts on
    pred_x0 = (x_t - sqrt(1-a) eps_hat)/sqrt(a), amplifying eps_hat by up to 3e3 and flipping
    nearest-neighbour assignments (measured |g16 - g32|/|g32| = 0.15 for both).  The backward
    chain itself is checked against f32 with a smooth upstream gradient below."""
    sim, real = _clouds(1000, 8, 120000).cuda(), _clouds(2000, 8, 120000).cuda()
    norm = lambda g: torch.sqrt(sum((v ** 2).sum() for v in g.values())).item()  # noqa: E731
    for lam in (0.1, 0.0):
        l32, g32 = _trainer_step_grads(tmp_path, sim, real, False, lam)
        for dt in ("float16", "bfloat16"):
            l16, g16 = _trainer_step_grads(tmp_path, sim, real, True, lam, dt)
            print(f"configs[2] lambda_chamfer {lam} {dt}: loss f32 {l32:.6f} amp {l16:.6f}; "
                  f"grad norm f32 {norm(g32):.4e} amp {norm(g16):.4e}")
            assert np.isfinite(l32) and np.isfinite(l16)
            assert abs(l16 - l32) <= 2e-2 * abs(l32), (dt, l16, l32)
            assert abs(norm(g16) - norm(g32)) <= 0.10 * norm(g32), dt


def test_model_backward_8x120k_amp_vs_fp32():
    """The training forward + backward of PointCloudDiffusionModel at configs[2]'s size
    (8 x 120k noisy + condition clouds, train-mode BN, cond drop), same draws, same smooth
    upstream gradient G on the coarse noise prediction:

    * f32 twice: bit-identical gradients (no float atomics anywhere in the backward);
    * autocast vs f32, in both 16-bit formats -- float16 (the reference's CUDA autocast,
      trainer.py:50,78, and Config.amp_dtype's default) and bfloat16: the prediction within
      2e-2 (bf16 measured 7.7e-3); the last layer's weight gradient (no ReLU behind it) within
      2e-2 (bf16 measured 7.6e-3).  Deeper layers differ by what rounding does to the ReLU
      masks: a pre-activation within the format's error of zero (~3 % of the units at K = 256
      for bf16: 2^-9 sqrt(K) of the spread; 8x fewer for fp16) flips its mask, which moves the
      gradient by ~sqrt(0.03) ~ 0.15 of its norm for bf16; measured 0.13-0.19 on the noise
      predictor, 0.36-0.59 on the SA layers (train-mode BN over the flipped units), 0.27 for
      the whole gradient.  Regression bounds above those: whole gradient <= 0.35, noise
      predictor cos >= 0.975, style encoder cos >= 0.8 (pre-BN conv biases aside:
      analytically zero gradient, rounding noise on both sides);
    * fp16 tracks the f32 step at least as closely as bf16 (3 more mantissa bits, same MFMA
      rate): prediction, last-layer gradient and whole gradient each no further from f32."""
    from pointcloud_style_transfer_amd import rng
    from pointcloud_style_transfer_amd.config.config import Config
    from pointcloud_style_transfer_amd.models.diffusion_model import PointCloudDiffusionModel

    noisy = (_clouds(1000, 8, 120000) * 0.7).cuda()
    real = _clouds(2000, 8, 120000).cuda()
    t = torch.arange(8, device="cuda") * 120 + 3
    grads, preds = [], []
    modes = [None, None, torch.float16, torch.bfloat16]
    for half in modes:
        torch.manual_seed(0)
        m = PointCloudDiffusionModel(Config(make_dirs=False)).cuda().train()
        for mod in m.modules():
            if isinstance(mod, torch.nn.Dropout):
                mod.p = 0.0
        with rng.replay(rng.CounterRNG(4100)), \
                torch.autocast("cuda", enabled=half is not None, dtype=half or torch.float16):
            pred, idx = m(noisy, t, real, cond_drop_prob=0.1)
        G = torch.randn(pred.shape, generator=torch.Generator(device="cuda").manual_seed(9),
                        device="cuda")
        pred.backward(G)
        preds.append(pred.detach())
        grads.append({n: p.grad.detach().double() for n, p in m.named_parameters()})
        del m, pred, idx
    g32, g32b = grads[0], grads[1]
    assert all(torch.equal(g32[n], g32b[n]) for n in g32), "f32 backward not deterministic"
    keep = [n for n in g32 if not PRE_BN_BIAS.search(n)]
    n32 = torch.sqrt(sum((g32[n] ** 2).sum() for n in keep)).item()
    last = "noise_predictor.output_mlp.4.weight"
    stats = {}
    for name, pred16, g16 in (("fp16", preds[2], grads[2]), ("bf16", preds[3], grads[3])):
        rel = ((pred16 - preds[0]).norm() / preds[0].norm()).item()
        nd = torch.sqrt(sum(((g16[n] - g32[n]) ** 2).sum() for n in keep)).item() / n32
        last_rel = ((g16[last] - g32[last]).norm() / g32[last].norm()).item()
        stats[name] = (rel, last_rel, nd)
        print(f"model fwd+bwd 8x120k {name}: |pred16 - pred32|/|pred32| {rel:.3e}, "
              f"last-layer dW {last_rel:.3e}, |g16 - g32| / |g32| {nd:.3e}")
        bad = []
        for n in keep:
            a, b = g16[n].flatten(), g32[n].flatten()
            cos = float((a @ b) / (a.norm() * b.norm() + 1e-300))
            floor = 0.975 if n.startswith("noise_predictor.") else 0.8
            if cos < floor:
                bad.append(f"{n}: cos {cos:.4f} < {floor}")
        assert rel <= 2e-2, (name, rel)
        assert last_rel <= 2e-2, (name, last_rel)
        assert nd <= 0.35, (name, nd)
        assert not bad, (name, bad)
    for k, what in enumerate(("prediction", "last-layer dW", "whole gradient")):
        assert stats["fp16"][k] <= stats["bf16"][k], (what, stats)


@pytest.fixture(scope="module")
def batch32():
    from pointcloud_style_transfer_amd.config.config import Config
    from pointcloud_style_transfer_amd.models.diffusion_model import (DiffusionProcess,
                                                                        PointCloudDiffusionModel)
    from pointcloud_style_transfer_amd.synthetic import standard_normal

    cfg = Config(make_dirs=False, precision="bf16")
    torch.manual_seed(0)
    model = PointCloudDiffusionModel(cfg).cuda().eval()
    dp = DiffusionProcess(cfg, device="cuda")
    src, cond = _clouds(1000, 32, 120000).cuda(), _clouds(2000, 32, 120000).cuda()
    xT = torch.from_numpy(np.stack([standard_normal(3000 + i, (120000, 3))
                                    for i in range(32)])).cuda()
    return cfg, model, dp, src, cond, xT


def test_graph_step_32x120k(batch32):
    """configs[4]: guided_sample_loop(graph=True) on 32 clouds x 120000 (64 CFG rows per step)
    vs the eager loop, same seeds; (700, 0) schedule."""
    cfg, model, dp, src, cond, xT = batch32
    dp_ts = dp._timesteps
    dp._timesteps = lambda n: [700, 0]
    outs = []
    try:
        for graph in (False, True):
            torch.manual_seed(11)
            outs.append(dp.guided_sample_loop(model, src, cond, 2, 7.5, x_T=xT, graph=graph))
    finally:
        dp._timesteps = dp_ts
    a, b = outs
    assert a.shape == (32, 120000, 3) and torch.isfinite(b).all()
    # each step is a pure function of its inputs and the seed: the kept SET is fixed by the
    # seed and the noise/kNN results do not depend on the row order of the subset
    # (tools/determinism_probe.py), so the captured graph reproduces the eager loop exactly
    assert torch.equal(a, b), (a - b).abs().max().item()


def test_device_subset_32x120k_properties(batch32):
    """The CFG batch's device-drawn subset at 32 clouds: per row, every voxel representative
    (the oracle's, diffusion_model.py:78-97) is kept with its multiplicity (two voxels whose
    mean index coincides keep that point twice, as the reference's cat(reps, pad) does), the
    T - U pad points are distinct non-representatives, the row is in ascending point-index
    order, and a second call with the same seed gives bit-identical rows."""
    from oracle import oracle as O
    from pointcloud_style_transfer_amd import _hip

    cfg, model, dp, src, cond, xT = batch32
    x = (xT * 0.5).contiguous()
    T = cfg.global_points
    pts, idx = _hip.voxel_downsample(x, T, seed=99, copies=2)
    pts2, idx2 = _hip.voxel_downsample(x, T, seed=99, copies=2)
    assert torch.equal(idx, idx2) and torch.equal(pts, pts2)
    assert idx.shape == (64, T)
    I = idx.cpu().numpy()
    xn = x.cpu().numpy()
    for row in range(64):
        c = row % 32
        r = I[row]
        assert np.all(np.diff(r) >= 0), row
        reps = O.voxel_reps(xn[c], T)[0]
        assert len(reps) < T  # the pad branch (U ~ 4.8k for these clouds)
        vals, cnts = np.unique(r, return_counts=True)
        rv, rc = np.unique(reps, return_counts=True)
        have = dict(zip(vals.tolist(), cnts.tolist()))
        assert all(have.get(v, 0) == k for v, k in zip(rv.tolist(), rc.tolist())), row
        pad = ~np.isin(vals, rv)
        assert pad.sum() == T - len(reps) and (cnts[pad] == 1).all(), row
        np.testing.assert_array_equal(pts[row].cpu().numpy(), xn[c][r])
    # the copies keep different pad subsets per row (their own keys)
    assert not torch.equal(idx[0], idx[32])


def test_replayed_step_32_clouds_vs_oracle(batch32, det_state):
    """One replayed guided step of the 32-cloud batch (the replay path: host permutations from
    rng.CounterRNG, one per CFG row, as torch.randperm is drawn per row) in fp32, checked
    against the oracle on clouds 0, 17 and 31 (rows c and 32 + c): downsample indices
    bit-exact, noise within 1e-4 rel, the kNN upsample of the same coarse noise bit-exact, the
    CFG/DDIM update within 1e-5."""
    from detweights import load_into
    from oracle import oracle as O
    from pointcloud_style_transfer_amd import _hip, rng

    cfg, model, dp, src, cond, xT = batch32
    cfg.precision = "fp32"
    try:
        load_into(model)
        sd = {k: v.detach().float().cpu().numpy() for k, v in model.state_dict().items()}
        T = cfg.global_points
        hp, npred = model.hierarchical_processor, model.noise_predictor
        g = torch.Generator(device="cpu").manual_seed(5)
        style = (torch.randn(32, 256, generator=g) * 0.3).cuda()
        style_in = torch.cat([style, torch.zeros_like(style)])
        t, t_prev = 999, 979
        t_in = torch.full((64,), t, dtype=torch.long, device="cuda")
        x = xT
        with torch.no_grad(), rng.replay(rng.CounterRNG(77)):
            xc, xi = hp.downsample_copies(x, 2)
            nc = npred(xc, t_in, style_in)
            eps = hp.upsample_knn(nc, torch.cat([x, x]), xi)
            xn = _hip.cfg_ddim_step(x, eps[:32], eps[32:], src, 7.5, dp._coeffs(t, t_prev))
        sched = O.Schedule()
        X, S = x.cpu().numpy(), src.cpu().numpy()
        for c in (0, 17, 31):
            rows = (c, 32 + c)
            x_in = np.stack([X[c], X[c]])
            cs, ids = [], []
            for k, r in enumerate(rows):
                reps = O.voxel_reps(x_in[k], T)[0]
                n = 120000 - len(np.unique(reps)) if len(reps) < T else len(reps)
                perm = np.random.default_rng([77, r]).permutation(n)
                p, ix = O.voxel_downsample(x_in[k:k + 1], T, O.Replay([("randperm", perm)]))
                cs.append(p[0])
                ids.append(ix[0])
            np.testing.assert_array_equal(xi[list(rows)].cpu().numpy(), np.stack(ids))
            st = style_in[list(rows)].cpu().numpy()
            ref_nc = O.noise_predictor(sd, np.stack(cs), np.full(2, t), st)
            got_nc = nc[list(rows)].cpu().numpy()
            assert_close(got_nc, ref_nc)
            up = O.upsample_knn(got_nc, x_in, np.stack(ids))
            np.testing.assert_array_equal(eps[list(rows)].cpu().numpy(), up)
            ref_x = O.guided_update(sched, X[c:c + 1], up[:1], up[1:], S[c:c + 1], t, t_prev, 7.5)
            assert_close(xn[c:c + 1].cpu().numpy(), ref_x, rtol=1e-5)
    finally:
        cfg.precision = "bf16"


def test_noise_mlp_bf16_per_element_60000(det_state):
    """The measured launch (bf16 noise MLP, 2 x 30000 points) against exact f32 per element:
    |bf16 - f32| <= 0.05 * (|f32| + 0.1 max|f32|) for >= 99.9 % of the elements and every
    element within 0.25 max|f32| (bf16 keeps 8 mantissa bits per operand over 14 layers)."""
    from pointcloud_style_transfer_amd import _hip, packing

    rng = np.random.default_rng(60000)
    pts = torch.from_numpy(rng.standard_normal((60000, 3)).astype(np.float32)).cuda()
    t = torch.tensor([999, 999]).cuda()
    style = torch.from_numpy((rng.standard_normal((2, 256)) * 0.3).astype(np.float32)).cuda()
    style[1] = 0
    g = lambda n: torch.from_numpy(det_state[f"noise_predictor.{n}"]).cuda()  # noqa: E731
    cp = (packing.time_freqs(128).cuda(), g("time_proj.weight").t().contiguous(),
          g("time_proj.bias"), g("style_proj.weight").t().contiguous(), g("style_proj.bias"),
          g("point_encoder.4.bias"))
    cond = _hip.noise_cond(t, style, *cp)
    bias = torch.from_numpy(packing.pack_bias(det_state)).cuda()
    outs = []
    for prec in (0, 1):   # f32, bf16 (solo 16x16x32)
        blob = torch.from_numpy(packing.pack_blob(det_state, prec)).cuda()
        outs.append(_hip.noise_mlp(pts, 30000, cond, blob, bias, prec).cpu().numpy())
    f32 = outs[0]
    scale = np.abs(f32).max()
    for prec, bf in ((1, outs[1]),):
        d = np.abs(bf - f32)
        ok = d <= 0.05 * (np.abs(f32) + 0.1 * scale)
        print(f"bf16 (code {prec}) vs f32 at 60000 pts: frac ok {ok.mean():.6f}, max "
              f"{d.max() / scale:.3e} of max|f32|, median rel {np.median(d / (np.abs(f32) + 1e-30)):.3e}")
        assert ok.mean() >= 0.999
        assert d.max() <= 0.25 * scale


def test_chamfer_vs_oracle_10_steps_120k(det_state):
    """configs[1]'s quality figure at a test-sized schedule: the HIP guided loop (fp32 noise
    MLP) against the oracle loop on one 120k cloud, 10 steps, same x_T and counter-keyed
    draws, the oracle computed live.  Per step the two agree to fp32 summation order (1e-4
    rel, the teacher-forced tests); the loop amplifies that.  The 10-step chaos floor (oracle
    vs itself from x_T moved by 1 ulp, CHAOS_FLOOR_10, profiles/r03/chaos_floor.json) is
    large -- the first update divides by sqrt(a_999) = 3.1e-4, and a voxel size moved by one
    ulp re-draws the subset -- so the bounds are fractions of it: Chamfer (metrics.py:20-44)
    and the 99.9th percentile within 0.25x the floor, the maximum within 0.005x (round 2
    measured Chamfer 1.5e-4 = 0.13x and max 2.4e-3 = 0.003x)."""
    from detweights import load_into
    from oracle import oracle as O
    from pointcloud_style_transfer_amd import rng
    from pointcloud_style_transfer_amd.config.config import Config
    from pointcloud_style_transfer_amd.evaluation.metrics import PointCloudMetrics
    from pointcloud_style_transfer_amd.models.diffusion_model import (DiffusionProcess,
                                                                        PointCloudDiffusionModel)
    from pointcloud_style_transfer_amd.synthetic import standard_normal

    cfg = Config(make_dirs=False, precision="fp32")
    model = PointCloudDiffusionModel(cfg)
    load_into(model)
    model = model.cuda().eval()
    dp = DiffusionProcess(cfg, device="cuda")
    src, cond = _clouds(1000, 1, 120000).numpy(), _clouds(2000, 1, 120000).numpy()
    xT = standard_normal(3000, (1, 120000, 3))
    S, T = 10, cfg.global_points
    with rng.replay(rng.CounterRNG(6000)):
        out = dp.guided_sample_loop(model, torch.from_numpy(src).cuda(),
                                    torch.from_numpy(cond).cuda(), S, 7.5,
                                    x_T=torch.from_numpy(xT).cuda())
    sd = {k: v.detach().float().cpu().numpy() for k, v in model.state_dict().items()}
    ctr = rng.CounterRNG(6000)

    def down(rows):
        outs, idxs = [], []
        for b in range(rows.shape[0]):
            reps = O.voxel_reps(rows[b], T)[0]
            n = len(reps) if len(reps) > T else rows.shape[1] - len(np.unique(reps))
            p, ix = O.voxel_downsample(rows[b:b + 1], T,
                                       O.Replay([("randperm", ctr.generator().permutation(n))]))
            outs.append(p[0])
            idxs.append(ix[0])
        return np.stack(outs), np.stack(idxs)

    cd, _ = down(cond)
    starts = [("randint", ctr.generator().integers(0, cd.shape[1], (1,), dtype=np.int64)),
              ("randint", ctr.generator().integers(0, 512, (1,), dtype=np.int64))]
    style = O.style_encoder(sd, cd, O.Replay(starts))
    style_in = np.concatenate([style, np.zeros_like(style)])
    sched = O.Schedule()
    ts = O.timesteps_for(1000, S)
    x = xT.copy()
    for i, t in enumerate(ts):
        x_in = np.concatenate([x, x])
        xc, xi = down(x_in)
        eps = O.upsample_knn(O.noise_predictor(sd, xc, np.full(2, t), style_in), x_in, xi)
        x = O.guided_update(sched, x, eps[:1], eps[1:], src, int(t),
                            int(ts[i + 1]) if t > 0 else -1, 7.5)
    ref = torch.from_numpy(x).cuda()
    ch = float(PointCloudMetrics().chamfer_distance(out, ref)[0])
    d = (out - ref).abs()
    within = (d <= 1e-4 * (ref.abs() + 0.1 * ref.abs().max())).float().mean().item()
    w3 = (d <= 1e-3).float().mean().item()
    print(f"10-step 120k fp32: chamfer_vs_ref {ch:.3e}, within 1e-4 rel {within:.6f}, "
          f"within 1e-3 abs {w3:.6f}, median abs {d.median().item():.3e}, "
          f"max abs {d.max().item():.3e}")
    p999 = float(torch.quantile(d.flatten().double(), 0.999))
    print(f"  vs the 10-step floor: chamfer {ch / CHAOS_FLOOR_10['chamfer']:.3f} x, p999 "
          f"{p999 / CHAOS_FLOOR_10['p999_abs']:.3f} x, max "
          f"{d.max().item() / CHAOS_FLOOR_10['max_abs']:.4f} x")
    assert ch <= 0.25 * CHAOS_FLOOR_10["chamfer"]
    assert p999 <= 0.25 * CHAOS_FLOOR_10["p999_abs"]
    assert d.max().item() <= 0.005 * CHAOS_FLOOR_10["max_abs"]
    assert w3 >= 0.99


# The loop's own chaos floor (tools/chaos_floor.py -> profiles/r04/chaos_floor.json): the oracle
# loop against itself from x_T moved by one ulp per element, same cloud / weights / draws as
# below, 50-step schedule.  tests/test_host.py checks these constants against the JSON.
CHAOS_FLOOR_50 = {"chamfer": 1.0649e-4, "p999_abs": 9.448e-4, "max_abs": 9.332e-3}
CHAOS_FLOOR_10 = {"chamfer": 1.1634e-3, "p999_abs": 1.8010e-2, "max_abs": 7.4255e-1}
# the same for BASELINE configs[1]'s full 1000-step schedule (profiles/r04/chaos_floor.json)
CHAOS_FLOOR_1000 = {"chamfer": 6.9574e-06, "p999_abs": 3.0011e-05, "max_abs": 7.2047e-05}


@pytest.mark.parametrize("precision,mult", [("fp32", 1.0), ("bf16", 1.5)])
def test_loop_vs_oracle_50_steps_120k(det_state, golden, precision, mult):
    """BASELINE configs[1]'s quality gate ("Chamfer vs ref"), for the mode bench.py measures
    (bf16 noise MLP) and the parity mode (fp32): the HIP guided loop on the 120k lidar-like
    cloud, 50 steps, guidance 7.5, the same x_T and counter-keyed draws as the committed oracle
    output (tests/golden/gen_oracle_loop.py).  Bounds are a stated multiple of the chaos floor
    -- what a 1-ulp change of x_T does to the oracle itself over the same loop: fp32 within
    1x the floor, bf16 within 1.5x, for the metrics.py:20-44 Chamfer, the 99.9th percentile
    and the maximum of |hip - oracle|.  Measured (round 3): fp32 0.39 / 0.18 / 0.05 x the
    floor, bf16 0.95 / 0.35 / 0.94 x; the loop is deterministic (replayed draws), so these
    figures repeat run to run."""
    from detweights import load_into
    from pointcloud_style_transfer_amd import rng
    from pointcloud_style_transfer_amd.config.config import Config
    from pointcloud_style_transfer_amd.evaluation.metrics import PointCloudMetrics
    from pointcloud_style_transfer_amd.models.diffusion_model import (DiffusionProcess,
                                                                        PointCloudDiffusionModel)
    from pointcloud_style_transfer_amd.synthetic import standard_normal

    ref = torch.from_numpy(golden("oracle_loop120k.npz")["x_50"]).cuda()
    cfg = Config(make_dirs=False, precision=precision)
    model = PointCloudDiffusionModel(cfg)
    load_into(model)
    model = model.cuda().eval()
    dp = DiffusionProcess(cfg, device="cuda")
    src, cond = _clouds(1000, 1, 120000).cuda(), _clouds(2000, 1, 120000).cuda()
    xT = torch.from_numpy(standard_normal(3000, (1, 120000, 3))).cuda()
    with rng.replay(rng.CounterRNG(6000)):
        out = dp.guided_sample_loop(model, src, cond, 50, 7.5, x_T=xT)
    ch = float(PointCloudMetrics().chamfer_distance(out, ref)[0])
    d = (out - ref).abs().flatten().double()
    p999 = float(torch.quantile(d, 0.999))
    mx = float(d.max())
    print(f"50-step 120k {precision}: chamfer_vs_oracle {ch:.3e} ({ch / CHAOS_FLOOR_50['chamfer']:.2f}"
          f" x floor), p999 {p999:.3e} ({p999 / CHAOS_FLOOR_50['p999_abs']:.2f} x), max {mx:.3e} "
          f"({mx / CHAOS_FLOOR_50['max_abs']:.2f} x), within 1e-3 abs {(d <= 1e-3).double().mean():.6f}")
    assert ch <= mult * CHAOS_FLOOR_50["chamfer"]
    assert p999 <= mult * CHAOS_FLOOR_50["p999_abs"]
    assert mx <= mult * CHAOS_FLOOR_50["max_abs"]


# (chamfer, p99.9, max) multiples of the 1000-step chaos floor, per precision
GATE_1000 = {"fp32": (1.0, 1.0, 1.0), "bf16": (3.0, 1.5, 1.5)}


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_loop_vs_oracle_1000_steps_120k(det_state, golden, precision):
    """BASELINE configs[1] as written -- the full 1000-step schedule (every t from 999 to 0,
    /root/reference/models/diffusion_model.py:224-261), 120k lidar-like cloud, guidance 7.5 --
    against the committed 1000-step oracle output (tests/golden/gen_oracle_loop.py 1000) on the
    same x_T and counter-keyed draws, for the parity mode (fp32) and the mode bench.py measures
    (bf16 noise MLP).  Bounds are multiples of the loop's own 1000-step chaos floor (the oracle
    against itself from x_T moved by one ulp, tools/chaos_floor.py -> profiles/r04/chaos_floor.json)
    for the metrics.py:20-44 Chamfer, the 99.9th percentile and the maximum of |hip - oracle|
    (GATE_1000): fp32 within 1x on all three; bf16 within 3x on Chamfer and 1.5x on the tails.
    The bf16 Chamfer multiple is wider because the floor is one ulp of x_T, while bf16 rounds
    the MLP's inputs every step: the error is spread thinly over every point rather than
    concentrated (its max stays under the floor's).  Every element of both modes must also sit
    within 1e-4 absolute of the oracle.  Measured (round 4, profiles/r04/loop1000.jsonl): fp32
    0.88 / 0.89 / 0.97 x the floor, bf16 2.30 / 1.29 / 0.95 x, max |diff| 7.0e-5 and 6.9e-5; the
    loop is deterministic (replayed draws), so these figures repeat run to run."""
    from detweights import load_into
    from pointcloud_style_transfer_amd import rng
    from pointcloud_style_transfer_amd.config.config import Config
    from pointcloud_style_transfer_amd.evaluation.metrics import PointCloudMetrics
    from pointcloud_style_transfer_amd.models.diffusion_model import (DiffusionProcess,
                                                                        PointCloudDiffusionModel)
    from pointcloud_style_transfer_amd.synthetic import standard_normal

    if CHAOS_FLOOR_1000 is None:
        pytest.skip("1000-step chaos floor not measured yet")
    ref = torch.from_numpy(golden("oracle_loop120k_1000.npz")["x_1000"]).cuda()
    cfg = Config(make_dirs=False, precision=precision)
    model = PointCloudDiffusionModel(cfg)
    load_into(model)
    model = model.cuda().eval()
    dp = DiffusionProcess(cfg, device="cuda")
    src, cond = _clouds(1000, 1, 120000).cuda(), _clouds(2000, 1, 120000).cuda()
    xT = torch.from_numpy(standard_normal(3000, (1, 120000, 3))).cuda()
    with rng.replay(rng.CounterRNG(6000)):
        out = dp.guided_sample_loop(model, src, cond, 1000, 7.5, x_T=xT)
    ch = float(PointCloudMetrics().chamfer_distance(out, ref)[0])
    d = (out - ref).abs().flatten().double()
    p999 = float(torch.quantile(d, 0.999))
    mx = float(d.max())
    fl = CHAOS_FLOOR_1000
    print(f"1000-step 120k {precision}: chamfer_vs_oracle {ch:.3e} ({ch / fl['chamfer']:.2f} x floor), "
          f"p999 {p999:.3e} ({p999 / fl['p999_abs']:.2f} x), max {mx:.3e} ({mx / fl['max_abs']:.2f} x), "
          f"within 1e-3 abs {(d <= 1e-3).double().mean():.6f}")
    m_ch, m_p999, m_max = GATE_1000[precision]
    assert ch <= m_ch * fl["chamfer"]
    assert p999 <= m_p999 * fl["p999_abs"]
    assert mx <= m_max * fl["max_abs"]
    assert mx <= 1e-4


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_timed_path_teacher_forced_vs_oracle_120k(det_state, precision):
    """The bench's timed path end to end: the guided loop with its DEVICE-drawn
    voxel subsets (no replay: the prepared downsample, the pool histogram made by the previous
    update, the rows-layout kNN on the side stream), the 1000-step schedule, 120k cloud, with the
    fp32 (parity) noise MLP and with the bf16 one -- the mode bench.py times.
    For each of the first 6 steps the loop's own (x, subset) are recorded; (a) each CFG row's
    subset is a valid draw of the reference's downsample (diffusion_model.py:90-120): U > T -> T
    of the representatives (as a multiset), U < T -> every representative plus T - U distinct
    non-representatives, computed by the oracle's voxel_reps on the same x; (b) the oracle's step
    (exact f32 noise MLP, exact kNN-3 IDW, CFG + DDIM update) from that x and subset gives the
    loop's next x within the MLP's per-element bound carried through the CFG combination:
    eps_u + 7.5 (eps_c - eps_u) scales the two rows' error difference by up to 16x, so a factor 20
    on the MLP's bound.  fp32: the noise MLP agrees to 1e-4 rel per element -> 2e-3 rel for
    >= 99.9 % of the elements and every element within 2e-5 absolute (x is ~|eps| ~ 1e-2 here;
    round 5 measured max 6e-6).  bf16: the MLP's measured-launch bound
    (test_noise_mlp_bf16_per_element_60000: >= 99.9 % within 0.05 rel, every element within
    0.25 max|f32|) -> >= 99.9 % within 1.0 rel and every element within 5 max|x'|."""
    from collections import Counter

    from conftest import assert_mostly_close
    from detweights import load_into
    from oracle import oracle as O
    from pointcloud_style_transfer_amd.config.config import Config
    from pointcloud_style_transfer_amd.models.diffusion_model import (DiffusionProcess,
                                                                        PointCloudDiffusionModel)
    from pointcloud_style_transfer_amd.synthetic import standard_normal

    cfg = Config(make_dirs=False, precision=precision)
    model = PointCloudDiffusionModel(cfg)
    load_into(model)
    model = model.cuda().eval()
    dp = DiffusionProcess(cfg, device="cuda")
    src = _clouds(1000, 1, 120000)
    cond = _clouds(2000, 1, 120000)
    xT = torch.from_numpy(standard_normal(3000, (1, 120000, 3)))
    K, T = 6, cfg.global_points
    rtol, max_abs_of = (2e-3, lambda scale: 2e-5) if precision == "fp32" else (1.0, lambda scale: 5.0 * scale)
    hp = model.hierarchical_processor
    rec, styles = [], []
    real_down = hp.downsample_copies

    def recording(x, *a, **k):
        xc, xi = real_down(x, *a, **k)
        if len(rec) <= K:  # stream-ordered copies of the step's input and subset
            rec.append((x.clone(), xi.clone()))
        return xc, xi

    hook = model.style_encoder.register_forward_hook(lambda m, i, o: styles.append(o.detach().clone()))
    hp.downsample_copies = recording
    try:
        with torch.no_grad():
            dp.guided_sample_loop(model, src.cuda(), cond.cuda(), 1000, 7.5, x_T=xT.cuda())
    finally:
        del hp.downsample_copies
        hook.remove()
    torch.cuda.synchronize()
    assert len(rec) == K + 1 and len(styles) == 1
    sd = {k: v.detach().float().cpu().numpy() for k, v in model.state_dict().items()}
    style = styles[0].cpu().numpy()
    style_in = np.concatenate([style, np.zeros_like(style)])
    sched = O.Schedule()
    ts = O.timesteps_for(1000, 1000)
    for i in range(K):
        x = rec[i][0].cpu().numpy()
        xi = rec[i][1].cpu().numpy()
        reps = Counter(O.voxel_reps(x[0], T)[0].tolist())
        U = sum(reps.values())
        for b in range(2):
            got = Counter(xi[b].tolist())
            assert sum(got.values()) == T
            if U > T:
                assert not (got - reps), (i, b, "an index outside the representatives")
            else:
                assert not (reps - got), (i, b, "a representative missing")
                extra = got - reps
                assert all(c == 1 for c in extra.values()) and sum(extra.values()) == T - U
                assert not (set(extra) & set(reps)), (i, b)
        nxt = O.guided_step_given(sd, sched, x, src.numpy(), style_in, int(ts[i]), int(ts[i + 1]),
                                  xi, 7.5)
        hip = rec[i + 1][0].cpu().numpy()
        d = np.abs(hip - nxt)
        rel = lambda r: np.mean(d <= r * (np.abs(nxt) + 0.1 * np.abs(nxt).max()))  # noqa: E731
        print(f"{precision} step {i} t={int(ts[i])}: U={U}, max|x| {np.abs(nxt).max():.3e}, max abs "
              f"{d.max():.3e}, within 1e-4 / 1e-3 / 2e-3 / 5e-2 rel {rel(1e-4):.6f} / {rel(1e-3):.6f} / "
              f"{rel(2e-3):.6f} / {rel(5e-2):.6f}")
        assert_mostly_close(hip, nxt, rtol=rtol, frac=0.999,
                            max_abs=max_abs_of(float(np.abs(nxt).max())))
