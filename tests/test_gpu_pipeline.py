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
