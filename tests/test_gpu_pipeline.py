"""The reference's two callers of the hot path, end to end on the GPU, against fixtures the
reference itself produced (tests/golden/gen_golden.py):

  * one `DiffusionTrainer.train_one_epoch` step (trainer.py:70-127) at B=2 x 4096 points,
    hierarchical 4096 -> 1024, Chamfer + L1, use_amp=False, dropout off, reference draws
    replayed -- loss, every parameter gradient, the AdamW update and the EMA update;
  * BASELINE config 1: `scripts/inference.py` on a 2048 x 3 cloud, 10 steps, from a
    reference-format checkpoint (EMA weights, BN buffers left at init: quirk Q9).
"""
import os

import numpy as np
import pytest
import torch

from conftest import assert_mostly_close

pytestmark = pytest.mark.gpu


def test_trainer_step(golden, tmp_path, monkeypatch):
    from detweights import load_into
    from pointcloud_style_transfer_amd import rng
    from pointcloud_style_transfer_amd.config.config import Config
    from pointcloud_style_transfer_amd.training.trainer import DiffusionTrainer
    from pointcloud_style_transfer_amd.utils.ema import ExponentialMovingAverage

    monkeypatch.chdir(tmp_path)
    g = golden("trainer_step.npz")
    cfg = Config(total_points=4096, global_points=1024, use_amp=False,
                 gradient_accumulation_steps=1, experiment_name="golden", precision="fp32")
    tr = DiffusionTrainer(cfg, device="cuda")
    load_into(tr.model)
    tr.optimizer = torch.optim.AdamW(tr.model.parameters(), lr=cfg.learning_rate,
                                     weight_decay=cfg.weight_decay, betas=(0.9, 0.95))
    tr.ema = ExponentialMovingAverage(tr.model.parameters(), decay=cfg.ema_decay)
    for mod in tr.model.modules():
        if isinstance(mod, torch.nn.Dropout):
            mod.p = 0.0
    grads = {}
    o_step = tr.optimizer.step

    def step(*a, **k):
        for n, p in tr.model.named_parameters():
            grads[n] = p.grad.detach().double().cpu()
        return o_step(*a, **k)

    tr.optimizer.step = step
    loader = [{"sim_full": torch.from_numpy(g["sim"]), "real_full": torch.from_numpy(g["real"])}]
    rp = rng.ReplayRNG.from_npz(g, "rng")
    with rng.replay(rp):
        avg = tr.train_one_epoch(loader)
    assert rp.exhausted
    np.testing.assert_allclose(avg, float(g["avg_loss"]), rtol=1e-4)
    names = [str(n) for n in g["param_names"]]
    assert names == list(grads)
    # Gradients against the reference's own fp32 accuracy.  tests/golden/trainer_sketch.npz
    # holds, for this exact step, 32 random projections of each gradient as the reference
    # computes it in fp32 and in fp64 (same draws), and the exact normwise error of its fp32
    # gradient vs fp64 (~1-2e-3: the Chamfer term's |p|^2+|q|^2-2pq cancels).  Ours must be
    # within 4x that error of the fp64 gradient (the 32-projection estimate is good to
    # ~+-15%).  Conv biases in front of a train-mode BatchNorm have an analytically zero
    # gradient (fp64: ~1e-15); both fp32 sides hold rounding noise there, so those must only
    # be negligible next to their conv weight's.
    import re

    from gen_sketch import gradient_sketch

    sk = golden("trainer_sketch.npz")
    assert [str(n) for n in sk["param_names"]] == names
    pre_bn = re.compile(r"style_encoder\.encoder\.sa\d\.mlp_convs\.\d+\.bias$")
    bad = []
    for i, n in enumerate(names):
        gabs = grads[n].abs().sum().item()
        if pre_bn.search(n):
            wabs = grads[n[:-4] + "weight"].abs().sum().item()
            if gabs > 1e-3 * wabs:
                bad.append(f"{n}: pre-BN bias sum|g| {gabs:.3e} vs weight {wabs:.3e}")
            continue
        s_ours = gradient_sketch(grads[n].numpy(), i)
        err = np.linalg.norm(s_ours - sk["sk64"][i]) / np.linalg.norm(sk["sk64"][i])
        if err > 4 * sk["rel32"][i] + 1e-6:
            bad.append(f"{n}: |ours - fp64| ~ {err:.2e} vs reference fp32 {sk['rel32'][i]:.2e}")
    assert not bad, "\n".join(bad)
    # AdamW + EMA: parameter sums after the step.  Adam's first step moves every element by
    # ~lr * sign(g), so an element whose gradient is at rounding level can flip by 2 lr:
    # allow that for 1% of the elements (all of them for the pre-BN biases).
    sd = tr.model.state_dict()
    ema = {n: p.double().sum().item() for n, p in zip(names, tr.ema.shadow_params)}
    for i, n in enumerate(names):
        flips = sd[n].numel() if pre_bn.search(n) else 1 + 0.01 * sd[n].numel()
        tol = 2 * cfg.learning_rate * flips
        got = sd[n].double().sum().item()
        assert abs(got - g["param_after_sum"][i]) <= tol + 1e-5 * abs(g["param_after_sum"][i]), n
        e_tol = (1 - cfg.ema_decay) * tol + 1e-5 * abs(g["ema_after_sum"][i]) + 1e-6
        assert abs(ema[n] - g["ema_after_sum"][i]) <= e_tol, n


def test_inference_cfg1(golden, tmp_path, monkeypatch):
    """BASELINE configs[0]: scripts/inference.py --num_steps 10 on 2048 x 3 clouds."""
    from detweights import load_into
    from pointcloud_style_transfer_amd import rng
    from pointcloud_style_transfer_amd.config.config import Config
    from pointcloud_style_transfer_amd.models.diffusion_model import PointCloudDiffusionModel
    from pointcloud_style_transfer_amd.scripts import inference as inf
    from pointcloud_style_transfer_amd.utils.checkpoint import CheckpointManager
    from pointcloud_style_transfer_amd.utils.ema import ExponentialMovingAverage

    monkeypatch.chdir(tmp_path)
    g = golden("inference_cfg1.npz")
    cfg = Config(experiment_name="cfg1", precision="fp32")
    m = PointCloudDiffusionModel(cfg)
    load_into(m)
    opt = torch.optim.AdamW(m.parameters(), lr=1e-4)
    ema = ExponentialMovingAverage(m.parameters(), decay=0.999)
    CheckpointManager(cfg.checkpoint_dir, cfg.experiment_name).save(m, opt, ema, epoch=0)
    np.save("src.npy", g["src"])
    np.save("ref.npy", g["ref"])
    ck = os.path.join(cfg.checkpoint_dir, "cfg1", "ckpt_epoch_0000.pth")
    rp = rng.ReplayRNG.from_npz(g, "rng")
    with rng.replay(rp):
        inf.main(["--checkpoint", ck, "--source", "src.npy", "--reference", "ref.npy",
                  "--output", "out/out.npy", "--num_steps", "10"])
    assert rp.exhausted
    out = np.load("out/out.npy")
    # outputs are denormalised (x25 / +3): the 10-step criterion scaled by the cloud's extent
    assert_mostly_close(out, g["out"], max_abs=1e-3 * 25)


@pytest.mark.parametrize("B", [1, 2])
def test_guided_sample_graph_matches_eager(B):
    """BASELINE configs[4]'s hipGraph-captured denoise step: guided_sample_loop(graph=True)
    replays one captured step per timestep with the per-step scalars in device buffers; same
    draws and kernels as the eager loop.  The device-drawn voxel subset is the same SET every
    run (its row order follows atomics), and the noise MLP and the kNN-3 upsample do not depend
    on that order (tools/determinism_probe.py: noise by index and upsample bit-identical across
    reorderings), so graph and eager agree bit for bit."""
    import torch

    from pointcloud_style_transfer_amd.config.config import Config
    from pointcloud_style_transfer_amd.models.diffusion_model import (DiffusionProcess,
                                                                        PointCloudDiffusionModel)
    from pointcloud_style_transfer_amd.synthetic import lidar_like_cloud

    cfg = Config(make_dirs=False, precision="bf16", global_points=2048)
    torch.manual_seed(0)
    model = PointCloudDiffusionModel(cfg).cuda().eval()
    dp = DiffusionProcess(cfg, device="cuda")
    src = torch.from_numpy(np.stack([lidar_like_cloud(1000 + i, 8192) for i in range(B)])).cuda()
    cond = torch.from_numpy(np.stack([lidar_like_cloud(2000 + i, 8192) for i in range(B)])).cuda()
    dp._timesteps = lambda n: [500, 0]
    outs = []
    for graph in (False, True):
        torch.manual_seed(7)
        outs.append(dp.guided_sample_loop(model, src, cond, num_inference_steps=2, graph=graph))
    assert torch.equal(outs[0], outs[1]), (outs[1] - outs[0]).abs().max().item()


def test_inference_entry_point_bf16(golden, tmp_path, monkeypatch):
    """`scripts/inference.py --precision bf16` reaches the measured mode: the noise MLP runs
    the bf16 solo kernel (precision code 1, `packing.BF16`) on every step, and the result stays within the
    bf16 mode's distance of the fp32 run (same draws)."""
    from detweights import load_into
    from pointcloud_style_transfer_amd import _hip, packing, rng
    from pointcloud_style_transfer_amd.config.config import Config
    from pointcloud_style_transfer_amd.models.diffusion_model import PointCloudDiffusionModel
    from pointcloud_style_transfer_amd.scripts import inference as inf
    from pointcloud_style_transfer_amd.utils.checkpoint import CheckpointManager
    from pointcloud_style_transfer_amd.utils.ema import ExponentialMovingAverage

    monkeypatch.chdir(tmp_path)
    g = golden("inference_cfg1.npz")
    cfg = Config(experiment_name="cfg1")   # precision left at its default (fp32)
    m = PointCloudDiffusionModel(cfg)
    load_into(m)
    CheckpointManager(cfg.checkpoint_dir, cfg.experiment_name).save(
        m, torch.optim.AdamW(m.parameters(), lr=1e-4),
        ExponentialMovingAverage(m.parameters(), decay=0.999), epoch=0)
    np.save("src.npy", g["src"])
    np.save("ref.npy", g["ref"])
    ck = os.path.join(cfg.checkpoint_dir, "cfg1", "ckpt_epoch_0000.pth")
    codes = []
    orig = _hip.noise_mlp

    def spy(*a, **k):
        codes.append(a[5] if len(a) > 5 else k.get("precision"))
        return orig(*a, **k)

    monkeypatch.setattr(_hip, "noise_mlp", spy)
    outs = {}
    for prec in ("fp32", "bf16"):
        codes.clear()
        with rng.replay(rng.ReplayRNG.from_npz(g, "rng")):
            inf.main(["--checkpoint", ck, "--source", "src.npy", "--reference", "ref.npy",
                      "--output", f"out/{prec}.npy", "--num_steps", "10", "--precision", prec])
        assert len(codes) == 10, codes
        assert set(codes) == {packing.F32 if prec == "fp32" else packing.BF16}, codes
        outs[prec] = np.load(f"out/{prec}.npy")
    # 2048-point clouds (no hierarchy), 10 steps, outputs denormalised (x25): bf16 moves the
    # trajectory by well under the cloud's point spacing
    d = np.abs(outs["bf16"] - outs["fp32"])
    print(f"entry point bf16 vs fp32: mean {d.mean():.3e}, p99 {np.quantile(d, 0.99):.3e}, "
          f"max {d.max():.3e} (cloud extent {np.ptp(outs['fp32'], 0)})")
    assert d.mean() <= 2e-2 and np.quantile(d, 0.99) <= 0.25, (d.mean(), d.max())


def test_trainer_resumes_reference_checkpoint_under_amp(tmp_path, monkeypatch):
    """DiffusionTrainer.train() loads the latest checkpoint into its fused
    AdamW; a checkpoint whose optimizer state came from a non-fused AdamW (the reference's)
    must resume and take a use_amp step with the GradScaler enabled (found_inf handed to the
    fused kernel on the device)."""
    from pointcloud_style_transfer_amd.config.config import Config
    from pointcloud_style_transfer_amd.synthetic import lidar_like_cloud
    from pointcloud_style_transfer_amd.training.trainer import DiffusionTrainer
    from pointcloud_style_transfer_amd.utils.ema import ExponentialMovingAverage

    monkeypatch.chdir(tmp_path)
    cfg = Config(total_points=8192, global_points=2048, use_amp=True,
                 gradient_accumulation_steps=1, experiment_name="resume")
    torch.manual_seed(0)
    tr = DiffusionTrainer(cfg, device="cuda")
    ref_opt = torch.optim.AdamW(tr.model.parameters(), lr=cfg.learning_rate,
                                weight_decay=cfg.weight_decay, betas=(0.9, 0.95))
    for p in tr.model.parameters():
        p.grad = torch.randn_like(p) * 1e-3
    ref_opt.step()
    tr.checkpoint_manager.save(tr.model, ref_opt, ExponentialMovingAverage(tr.model.parameters()),
                               epoch=3)
    assert tr.checkpoint_manager.load(tr.model, tr.optimizer, tr.ema) == 4
    assert all(g["fused"] for g in tr.optimizer.param_groups)
    assert tr.scaler.is_enabled()
    sim = torch.from_numpy(np.stack([lidar_like_cloud(1000 + i, 8192) for i in range(2)]))
    real = torch.from_numpy(np.stack([lidar_like_cloud(2000 + i, 8192) for i in range(2)]))
    tr.model.train()
    tr.optimizer.zero_grad()
    before = [p.detach().clone() for p in tr.model.parameters()]
    loss, _ = tr.train_step({"sim_full": sim, "real_full": real}, 0, 1)
    torch.cuda.synchronize()
    assert np.isfinite(float(loss))
    moved = sum(not torch.equal(b, p.detach()) for b, p in zip(before, tr.model.parameters()))
    assert moved > 70, moved


def test_train_one_epoch_pipelined_readback_matches_per_step(tmp_path, monkeypatch):
    """train_one_epoch reads step k's loss after queueing step k + 1 (train_step(host_sync=False))
    and hands each step the next batch (style-geometry prefetch): the epoch average and the final
    weights equal those of a loop that makes the same train_step calls but reads every step's
    floats right away (the reference's order, trainer.py:70-127)."""
    from pointcloud_style_transfer_amd.config.config import Config
    from pointcloud_style_transfer_amd.synthetic import lidar_like_cloud
    from pointcloud_style_transfer_amd.training.trainer import DiffusionTrainer

    monkeypatch.chdir(tmp_path)
    batches = [{"sim_full": torch.from_numpy(np.stack([lidar_like_cloud(10 * i + j, 4096)
                                                       for j in range(2)])),
                "real_full": torch.from_numpy(np.stack([lidar_like_cloud(500 + 10 * i + j, 4096)
                                                        for j in range(2)]))}
               for i in range(3)]

    def fresh():
        torch.manual_seed(0)
        cfg = Config(total_points=4096, global_points=1024, use_amp=True,
                     gradient_accumulation_steps=1, experiment_name="pipe", precision="fp32")
        return DiffusionTrainer(cfg, device="cuda")

    a = fresh()
    torch.manual_seed(1)
    avg_a = a.train_one_epoch(batches)
    b = fresh()
    torch.manual_seed(1)
    b.model.train()
    b.optimizer.zero_grad()
    total = 0.0
    for i, batch in enumerate(batches):
        nxt = batches[i + 1] if i + 1 < len(batches) else None
        loss, d = b.train_step(batch, i, len(batches), next_batch=nxt)
        total += loss.item()
        assert set(d) >= {"total_loss", "noise_loss"} and all(isinstance(v, float) for v in d.values())
    assert avg_a == total / len(batches)
    for (n, pa), (_, pb) in zip(a.model.named_parameters(), b.model.named_parameters()):
        assert torch.equal(pa, pb), n


@pytest.mark.parametrize("train", [False, True])
def test_style_geometry_prefetch_equals_inline(train):
    """forward(style_geometry=style_geometry(cond)) -- the trainer's prefetched style branch --
    gives the forward's own result: same downsample, FPS and ball-query draws in the same order,
    so with the generators reset the prediction and indices are bit-identical."""
    from pointcloud_style_transfer_amd.config.config import Config
    from pointcloud_style_transfer_amd.models.diffusion_model import PointCloudDiffusionModel
    from pointcloud_style_transfer_amd.synthetic import lidar_like_cloud

    torch.manual_seed(0)
    cfg = Config(total_points=8192, global_points=2048, make_dirs=False, precision="fp32")
    m = PointCloudDiffusionModel(cfg).cuda().train(train)
    for mod in m.modules():
        if isinstance(mod, torch.nn.Dropout):
            mod.p = 0.0
    noisy = torch.from_numpy(np.stack([lidar_like_cloud(7 + j, 8192) for j in range(2)])).cuda()
    real = torch.from_numpy(np.stack([lidar_like_cloud(70 + j, 8192) for j in range(2)])).cuda()
    t = torch.tensor([10, 500], device="cuda")
    outs = []
    for pre in (False, True):
        torch.manual_seed(123)
        torch.cuda.manual_seed(123)
        with torch.no_grad():
            geo = m.style_geometry(real) if pre else None
            outs.append(m(noisy, t, real, 0.0, True, style_geometry=geo))
    assert torch.equal(outs[0][1], outs[1][1])
    assert torch.equal(outs[0][0], outs[1][0])

