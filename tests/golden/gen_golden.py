"""Generate golden input/output vectors by running the REFERENCE implementation.

Runs only in the survey/build container, where `/root/reference` exists; the
reference itself never travels.  Usage (from any scratch directory, because
`Config.__post_init__` mkdirs in the CWD, `config/config.py:64-67`):

    cd /tmp/gg && PYTHONDONTWRITEBYTECODE=1 python /root/repo/tests/golden/gen_golden.py

Every random draw the reference makes (torch.randint / randperm / randn / rand /
randn_like) is recorded in call order and stored next to the outputs, so the
tests can replay it.  Weights come from `detweights.deterministic_state`.
Outputs land in `tests/golden/*.npz` (+ `checkpoint_manifest.json`).
"""
from __future__ import annotations

import io
import json
import os
import pickletools
import sys
import types
import zipfile

import numpy as np

REF = os.environ.get("PCST_REFERENCE", "/root/reference")
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REF)
sys.path.insert(0, HERE)
sys.path.insert(0, REPO)

# Harness-only stubs for modules that are not on the math path.
sys.modules.setdefault("open3d", types.ModuleType("open3d"))
_tb = types.ModuleType("torch.utils.tensorboard")


class _NullWriter:
    def __init__(self, *a, **k):
        pass

    def add_scalar(self, *a, **k):
        pass

    def close(self):
        pass


_tb.SummaryWriter = _NullWriter
sys.modules["torch.utils.tensorboard"] = _tb

import torch  # noqa: E402

torch.set_num_threads(8)

from config.config import Config  # noqa: E402
from models import pointnet2_encoder as ref_pn  # noqa: E402
from models import diffusion_model as ref_dm  # noqa: E402
from models import losses as ref_losses  # noqa: E402

from detweights import load_into  # noqa: E402
from pointcloud_style_transfer_amd.synthetic import (  # noqa: E402
    lidar_like_cloud, standard_normal)


class RNGRecorder:
    """Record every torch RNG draw the reference makes, in call order."""

    NAMES = ("randperm", "randn", "randint", "rand", "randn_like")

    def __init__(self):
        self.log = []

    def __enter__(self):
        self.orig = {n: getattr(torch, n) for n in self.NAMES}
        for n, f in self.orig.items():
            setattr(torch, n, self._wrap(n, f))
        return self

    def _wrap(self, name, fn):
        def g(*a, **k):
            out = fn(*a, **k)
            self.log.append((name, out.detach().clone()))
            return out
        return g

    def __exit__(self, *exc):
        for n, f in self.orig.items():
            setattr(torch, n, f)

    def pack(self, prefix="rng"):
        d = {f"{prefix}_names": np.array([n for n, _ in self.log])}
        for i, (_, t) in enumerate(self.log):
            d[f"{prefix}_{i}"] = t.numpy()
        return d


def save(name, **arrays):
    path = os.path.join(HERE, name)
    np.savez_compressed(path, **arrays)
    print(f"wrote {path}: {os.path.getsize(path) / 1024:.1f} KiB")


def t32(a):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32))


# ---------------------------------------------------------------------------
def gen_geometry():
    out = {}
    # square_distance (pointnet2_encoder.py:8-15)
    src = standard_normal(11, (2, 64, 3))
    dst = standard_normal(12, (2, 1000, 3))
    out["sqd_src"], out["sqd_dst"] = src, dst
    out["sqd_out"] = ref_pn.square_distance(t32(src), t32(dst)).numpy()

    # FPS (pointnet2_encoder.py:30-45): start index from the CPU generator.
    cases = {
        "fps_a": (standard_normal(21, (2, 2048, 3)), 512),
        "fps_b": (lidar_like_cloud(22, 30000)[None], 512),
        "fps_c": (lidar_like_cloud(23, 512)[None].repeat(2, 0), 128),
    }
    # tie case: 256 distinct points, each present 4 times, shuffled; npoint > 256
    base = standard_normal(24, (256, 3))
    perm = np.random.Generator(np.random.PCG64(25)).permutation(1024)
    out["fps_tie_xyz"] = base[np.arange(1024) % 256][perm][None]
    cases["fps_tie"] = (out["fps_tie_xyz"], 300)
    for key, (xyz, npoint) in cases.items():
        with RNGRecorder() as rec:
            idx = ref_pn.farthest_point_sample(t32(xyz), npoint)
        out[f"{key}_xyz"] = xyz
        out[f"{key}_npoint"] = np.int64(npoint)
        out[f"{key}_start"] = rec.log[0][1].numpy()
        out[f"{key}_idx"] = idx.numpy()

    # index_points (pointnet2_encoder.py:17-28), incl. clamping of idx == N
    pts = standard_normal(31, (2, 100, 5))
    gi = np.random.Generator(np.random.PCG64(32)).integers(0, 101, (2, 7, 4))
    out["ip_points"], out["ip_idx"] = pts, gi
    out["ip_out"] = ref_pn.index_points(t32(pts), torch.from_numpy(gi)).numpy()

    # ball query (pointnet2_encoder.py:47-59)
    xyz_b = out["fps_b_xyz"]
    new_b = ref_pn.index_points(t32(xyz_b), torch.from_numpy(out["fps_b_idx"])).numpy()
    bq = {
        "bq_sa1": (0.2, 32, xyz_b, new_b),
        "bq_sa2": (0.4, 64, out["fps_c_xyz"],
                   ref_pn.index_points(t32(out["fps_c_xyz"]),
                                       torch.from_numpy(out["fps_c_idx"])).numpy()),
    }
    # radius-boundary lattice + far centroids (no neighbours -> pad value N)
    g = np.arange(-5, 6, dtype=np.float64) * 0.1
    lat = np.stack(np.meshgrid(g, g, g, indexing="ij"), -1).reshape(-1, 3).astype(np.float32)
    cen = np.concatenate([lat[::97], np.array([[9.0, 9.0, 9.0], [-7.0, 0.0, 3.0]], np.float32)])
    bq["bq_edge"] = (0.2, 40, lat[None], cen[None])
    for key, (r, ns, xyz, new) in bq.items():
        out[f"{key}_radius"] = np.float64(r)
        out[f"{key}_nsample"] = np.int64(ns)
        out[f"{key}_xyz"] = xyz
        out[f"{key}_new"] = new
        out[f"{key}_idx"] = ref_pn.query_ball_point(r, ns, t32(xyz), t32(new)).numpy()
    save("geometry.npz", **out)


# ---------------------------------------------------------------------------
def make_model(cfg):
    m = ref_dm.PointCloudDiffusionModel(cfg)
    load_into(m)
    return m


def gen_encoder():
    cfg = Config()
    m = make_model(cfg)
    out = {}
    enc = m.style_encoder.encoder
    xyz = np.stack([lidar_like_cloud(41, 2048), lidar_like_cloud(42, 2048)])
    out["xyz"] = xyz
    for mode in ("eval", "train"):
        m.train(mode == "train")
        with torch.no_grad(), RNGRecorder() as rec:
            l1_xyz, l1_pts = enc.sa1(t32(xyz), None)
            l2_xyz, l2_pts = enc.sa2(l1_xyz, l1_pts.permute(0, 2, 1))
            _, l3 = enc.sa3(l2_xyz, l2_pts.permute(0, 2, 1))
        out.update({f"{mode}_l1_xyz": l1_xyz.numpy(), f"{mode}_l1_points": l1_pts.numpy(),
                    f"{mode}_l2_xyz": l2_xyz.numpy(), f"{mode}_l2_points": l2_pts.numpy(),
                    f"{mode}_l3": l3.numpy()})
        out.update(rec.pack(f"{mode}_rng"))
    # full StyleEncoder in eval mode (dropout inactive); re-load the weights because the
    # train-mode pass above updated the BN running statistics.
    load_into(m)
    m.eval()
    with torch.no_grad(), RNGRecorder() as rec:
        style = m.style_encoder(t32(xyz))
    out["style"] = style.numpy()
    out.update(rec.pack("style_rng"))
    # a 30000-point cond cloud (the SA1 shape of the 120k pipeline)
    xyz30 = lidar_like_cloud(43, 30000)[None]
    with torch.no_grad(), RNGRecorder() as rec:
        style30 = m.style_encoder(t32(xyz30))
    out["style30"] = style30.numpy()
    out.update(rec.pack("style30_rng"))
    save("encoder.npz", **out)


def gen_noise_predictor():
    cfg = Config()
    m = make_model(cfg).eval()
    out = {}
    pts = standard_normal(51, (2, 4096, 3))
    style = (standard_normal(52, (2, 256)) * 0.5).astype(np.float32)
    out["points"], out["style"] = pts, style
    ts = [0, 1, 499, 998, 999]
    out["ts"] = np.array(ts, np.int64)
    with torch.no_grad():
        for t in ts:
            tt = torch.tensor([t, max(t - 7, 0)], dtype=torch.long)
            out[f"t{t}_tvec"] = tt.numpy()
            out[f"t{t}_out"] = m.noise_predictor(t32(pts), tt, t32(style)).numpy()
        emb = m.noise_predictor.time_embedding(torch.arange(0, 1000, 37, dtype=torch.long))
        out["temb_t"] = np.arange(0, 1000, 37, dtype=np.int64)
        out["temb"] = emb.numpy()
    save("noise_predictor.npz", **out)


# ---------------------------------------------------------------------------
def gen_hierarchical():
    out = {}
    hp = ref_dm.HierarchicalProcessor(total_points=4096, global_points=1024)
    # pad branch (U < target): anisotropic cloud
    cases = {
        "pad": (np.stack([lidar_like_cloud(61, 4096), lidar_like_cloud(62, 4096)]), 1024),
        # subsample branch (U > target): nearly flat cloud
        "sub": (lidar_like_cloud(63, 4096, sigma=(1.0, 1.0, 1e-3))[None], 1024),
        # exact-size (N <= target -> identity)
        "ident": (lidar_like_cloud(64, 1000)[None], 1024),
    }
    for key, (pts, target) in cases.items():
        hp.global_points = target
        with RNGRecorder() as rec:
            dpts, didx = hp.downsample(t32(pts))
        out[f"{key}_pts"] = pts
        out[f"{key}_target"] = np.int64(target)
        out[f"{key}_down"] = dpts.numpy()
        out[f"{key}_idx"] = didx.numpy()
        out.update(rec.pack(f"{key}_rng"))
    # full-size 120k -> 30k (input regenerated from seed 65 in the tests)
    hp.global_points = 30000
    pts120 = lidar_like_cloud(65, 120000)[None]
    with RNGRecorder() as rec:
        _, idx120 = hp.downsample(t32(pts120))
    out["full_seed"] = np.int64(65)
    out["full_idx"] = idx120.numpy().astype(np.int32)
    out["full_perm"] = rec.log[0][1].numpy().astype(np.int32)
    out["full_names"] = np.array([n for n, _ in rec.log])

    # upsample_knn (diffusion_model.py:127-153)
    hp.global_points = 1024
    orig = cases["pad"][0]
    idx = out["pad_idx"]
    # coarse values are a per-point field gathered at idx: duplicate coarse
    # indices (frequent: mean-index representatives collide) then carry equal
    # values, as they do in the sampler, so KD-tree tie order cannot matter.
    field = standard_normal(66, (2, 4096, 3))
    coarse = np.stack([field[b][idx[b]] for b in range(2)])
    out["knn_coarse"], out["knn_orig"], out["knn_idx"] = coarse, orig, idx
    out["knn_out"] = hp.upsample_knn(t32(coarse), t32(orig), torch.from_numpy(idx)).numpy()
    # full-size upsample: 120k orig, 30k coarse values
    coarse120 = standard_normal(67, (1, 120000, 3))[:, idx120[0].numpy()]
    up = hp.upsample_knn(t32(coarse120), t32(pts120), idx120)
    out["knn_full_coarse_seed"] = np.int64(67)
    out["knn_full_out"] = up.numpy()
    save("hierarchical.npz", **out)


# ---------------------------------------------------------------------------
def gen_schedule_and_losses():
    out = {}
    cfg = Config()
    dp = ref_dm.DiffusionProcess(cfg, device="cpu")
    out["betas"] = dp.betas.numpy()
    out["alphas_cumprod"] = dp.alphas_cumprod.numpy()
    out["sqrt_ac"] = dp.sqrt_alphas_cumprod.numpy()
    out["sqrt_1mac"] = dp.sqrt_one_minus_alphas_cumprod.numpy()
    cfg_lin = Config(beta_schedule="linear")
    out["betas_linear"] = ref_dm.DiffusionProcess(cfg_lin, device="cpu").betas.numpy()
    x0 = standard_normal(71, (2, 500, 3))
    noise = standard_normal(72, (2, 500, 3))
    t = torch.tensor([3, 998])
    xt, _ = dp.q_sample(t32(x0), t, t32(noise))
    out["q_x0"], out["q_noise"], out["q_t"], out["q_xt"] = x0, noise, t.numpy(), xt.numpy()

    # Chamfer (losses.py:8-63) value + gradients
    pred = standard_normal(73, (2, 3000, 3))
    tgt = standard_normal(74, (2, 2500, 3))
    p = t32(pred).requires_grad_(True)
    q = t32(tgt).requires_grad_(True)
    cd = ref_losses.chamfer_distance_chunked_optimized(p, q)
    cd.sum().backward()
    out["cd_pred"], out["cd_target"] = pred, tgt
    out["cd_out"] = cd.detach().numpy()
    out["cd_grad_pred"] = p.grad.numpy()
    out["cd_grad_target"] = q.grad.numpy()
    # chunk boundary case: N not a multiple of 1024, small chunk
    cd2 = ref_losses.chamfer_distance_chunked_optimized(t32(pred[:, :1500]), t32(tgt[:, :700]),
                                                        chunk_size=256)
    out["cd2_out"] = cd2.numpy()

    # DiffusionLoss (losses.py:66-104)
    lf = ref_losses.DiffusionLoss(1.0, 0.1)
    pn = standard_normal(75, (2, 1000, 3))
    an = standard_normal(76, (2, 1000, 3))
    pp = standard_normal(77, (2, 1000, 3))
    tp = standard_normal(78, (2, 1000, 3))
    loss, d = lf(t32(pn), t32(an), t32(pp), t32(tp))
    out["dl_inputs"] = np.stack([pn, an, pp, tp])
    out["dl_total"] = np.float32(loss.item())
    out["dl_noise"] = np.float64(d["noise_loss"])
    out["dl_chamfer"] = np.float64(d["chamfer_loss"])
    loss_n, _ = lf(t32(pn), t32(an))
    out["dl_total_noise_only"] = np.float32(loss_n.item())
    save("schedule_losses.npz", **out)


# ---------------------------------------------------------------------------
def record_steps(m):
    """Patch the model's hierarchical processor / noise predictor to capture per-step tensors."""
    hp = m.hierarchical_processor
    cap = {"down_in": [], "down_idx": [], "np_in": [], "np_t": [], "np_style": [],
           "np_out": [], "up_out": []}
    o_down, o_up, o_np = hp.downsample, hp.upsample_knn, m.noise_predictor.forward

    def down(points):
        r = o_down(points)
        cap["down_in"].append(points.clone())
        cap["down_idx"].append(r[1].clone())
        return r

    def up(c, o, i):
        r = o_up(c, o, i)
        cap["up_out"].append(r.clone())
        return r

    def npf(x, t, s):
        r = o_np(x, t, s)
        cap["np_in"].append(x.clone())
        cap["np_t"].append(t.clone())
        cap["np_style"].append(s.clone())
        cap["np_out"].append(r.clone())
        return r

    hp.downsample, hp.upsample_knn, m.noise_predictor.forward = down, up, npf
    return cap


def gen_sampling():
    out = {}
    # (a) cfg-1 shape: 2048 points, default Config (global 30000 -> direct path), 10 steps
    cfg = Config()
    m = make_model(cfg).eval()
    dp = ref_dm.DiffusionProcess(cfg, device="cpu")
    src = lidar_like_cloud(1000, 2048)[None]
    cond = lidar_like_cloud(2000, 2048)[None]
    with RNGRecorder() as rec:
        x = dp.guided_sample_loop(m, t32(src), t32(cond), num_inference_steps=10, guidance_scale=7.5)
    out.update({"a_src": src, "a_cond": cond, "a_out": x.numpy()})
    out.update(rec.pack("a_rng"))

    # (b) hierarchical path at reduced size: N=4096, global 1024, 3 steps, per-step capture
    cfg_b = Config(total_points=4096, global_points=1024)
    mb = make_model(cfg_b).eval()
    dpb = ref_dm.DiffusionProcess(cfg_b, device="cpu")
    src_b = lidar_like_cloud(1001, 4096)[None]
    cond_b = lidar_like_cloud(2001, 4096)[None]
    cap = record_steps(mb)
    with RNGRecorder() as rec:
        xb = dpb.guided_sample_loop(mb, t32(src_b), t32(cond_b), num_inference_steps=3,
                                    guidance_scale=7.5)
    out.update({"b_src": src_b, "b_cond": cond_b, "b_out": xb.numpy()})
    out.update(rec.pack("b_rng"))
    for k, v in cap.items():
        out[f"b_cap_{k}_n"] = np.int64(len(v))
        for i, t in enumerate(v):
            out[f"b_cap_{k}_{i}"] = t.numpy()

    # (c) ddim_sample_loop, direct path, 4 steps
    with RNGRecorder() as rec:
        xc = dp.ddim_sample_loop(m, (1, 2048, 3), t32(cond), num_inference_steps=4)
    out["c_out"] = xc.numpy()
    out.update(rec.pack("c_rng"))

    # (d) full model.forward in train mode with cond dropout (hierarchical)
    mb.train()
    for mod in mb.modules():
        if isinstance(mod, torch.nn.Dropout):
            mod.p = 0.0
    mb.hierarchical_processor.downsample = ref_dm.HierarchicalProcessor.downsample.__get__(
        mb.hierarchical_processor)
    mb.noise_predictor.forward = ref_dm.NoisePredictor.forward.__get__(mb.noise_predictor)
    noisy = standard_normal(81, (2, 4096, 3))
    condd = np.stack([lidar_like_cloud(82, 4096), lidar_like_cloud(83, 4096)])
    with torch.no_grad(), RNGRecorder() as rec:
        pred, idx = mb(t32(noisy), torch.tensor([10, 900]), t32(condd), cond_drop_prob=0.5)
    out.update({"d_noisy": noisy, "d_cond": condd, "d_t": np.array([10, 900]),
                "d_pred": pred.numpy(), "d_idx": idx.numpy()})
    out.update(rec.pack("d_rng"))
    save("sampling.npz", **out)


# ---------------------------------------------------------------------------
def gen_trainer_and_checkpoint():
    from training.trainer import DiffusionTrainer
    from utils.checkpoint import CheckpointManager

    out = {}
    cfg = Config(total_points=4096, global_points=1024, use_amp=False,
                 gradient_accumulation_steps=1, experiment_name="golden")
    tr = DiffusionTrainer(cfg, device="cpu")
    load_into(tr.model)
    # re-init optimizer/EMA on the deterministic weights
    tr.optimizer = torch.optim.AdamW(tr.model.parameters(), lr=cfg.learning_rate,
                                     weight_decay=cfg.weight_decay, betas=(0.9, 0.95))
    from utils.ema import ExponentialMovingAverage
    tr.ema = ExponentialMovingAverage(tr.model.parameters(), decay=cfg.ema_decay)
    for mod in tr.model.modules():
        if isinstance(mod, torch.nn.Dropout):
            mod.p = 0.0
    sim = np.stack([lidar_like_cloud(91, 4096), lidar_like_cloud(92, 4096)])
    real = np.stack([lidar_like_cloud(93, 4096), lidar_like_cloud(94, 4096)])
    grads = {}
    o_step = tr.optimizer.step

    def step(*a, **k):
        for n, p in tr.model.named_parameters():
            grads[n] = p.grad.detach().clone()
        return o_step(*a, **k)

    tr.optimizer.step = step
    loader = [{"sim_full": t32(sim), "real_full": t32(real)}]
    with RNGRecorder() as rec:
        avg = tr.train_one_epoch(loader)
    out.update({"sim": sim, "real": real, "avg_loss": np.float64(avg)})
    out.update(rec.pack("rng"))
    names = list(grads)
    out["param_names"] = np.array(names)
    out["grad_sum"] = np.array([grads[n].double().sum().item() for n in names])
    out["grad_abs"] = np.array([grads[n].double().abs().sum().item() for n in names])
    out["grad_head"] = np.stack([np.pad(grads[n].flatten()[:8].numpy(), (0, 8 - min(8, grads[n].numel())))
                                 for n in names])
    sd = tr.model.state_dict()
    out["param_after_sum"] = np.array([sd[n].double().sum().item() for n in names])
    out["ema_after_sum"] = np.array([p.double().sum().item() for p in tr.ema.shadow_params])
    save("trainer_step.npz", **out)

    # reference-format checkpoint: describe its structure (too large to commit as-is)
    cm = CheckpointManager(cfg.checkpoint_dir, cfg.experiment_name)
    cm.save(tr.model, tr.optimizer, tr.ema, epoch=3, is_best=True)
    path = os.path.join(cfg.checkpoint_dir, cfg.experiment_name, "ckpt_epoch_0003.pth")
    ck = torch.load(path, map_location="cpu", weights_only=False)
    globals_seen = set()
    with zipfile.ZipFile(path) as zf:
        pkl = [n for n in zf.namelist() if n.endswith("data.pkl")][0]
        for op, arg, _ in pickletools.genops(io.BytesIO(zf.read(pkl))):
            if op.name in ("GLOBAL", "STACK_GLOBAL") and arg:
                globals_seen.add(str(arg).replace(" ", "."))
    manifest = {
        "files": sorted(os.listdir(os.path.join(cfg.checkpoint_dir, cfg.experiment_name))),
        "top_keys": sorted(ck.keys()),
        "epoch": ck["epoch"],
        "config_class": f"{type(ck['config']).__module__}.{type(ck['config']).__qualname__}",
        "config_fields": {k: v for k, v in vars(ck["config"]).items()},
        "model_state_dict": [[k, list(v.shape), str(v.dtype)] for k, v in ck["model_state_dict"].items()],
        "optimizer_keys": sorted(ck["optimizer_state_dict"].keys()),
        "optimizer_param_groups": [{k: v for k, v in g.items() if k != "params"}
                                   for g in ck["optimizer_state_dict"]["param_groups"]],
        "optimizer_n_state": len(ck["optimizer_state_dict"]["state"]),
        "optimizer_state_keys": sorted(ck["optimizer_state_dict"]["state"][0].keys()),
        "ema_keys": sorted(ck["ema_state_dict"].keys()),
        "ema_decay": ck["ema_state_dict"]["decay"],
        "ema_shapes": [list(p.shape) for p in ck["ema_state_dict"]["shadow_params"]],
        "pickle_globals": sorted(g for g in globals_seen if "(" not in g),
    }
    with open(os.path.join(HERE, "checkpoint_manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1, default=str)
    print("wrote checkpoint_manifest.json")


from gen_sketch import gradient_sketch  # noqa: E402


def gen_trainer_sketch():
    """The trainer step of trainer_step.npz in fp32 and in fp64 (weights, data and every
    random draw identical: both replay that fixture's recorded draws), stored as
    32-projection sketches of each parameter gradient plus the exact normwise distance of
    the fp32 gradient from the fp64 one -- the reference's own fp32 error, which is the
    yardstick for ours."""
    from training.trainer import DiffusionTrainer
    from utils.ema import ExponentialMovingAverage

    def run(dtype):
        torch.set_default_dtype(dtype)
        try:
            cfg = Config(total_points=4096, global_points=1024, use_amp=False,
                         gradient_accumulation_steps=1, experiment_name="golden_sketch")
            tr = DiffusionTrainer(cfg, device="cpu")
            load_into(tr.model)
            tr.model.to(dtype)
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
                    grads[n] = p.grad.detach().double().clone()
                return o_step(*a, **k)

            tr.optimizer.step = step
            sim = np.stack([lidar_like_cloud(91, 4096), lidar_like_cloud(92, 4096)])
            real = np.stack([lidar_like_cloud(93, 4096), lidar_like_cloud(94, 4096)])
            tr.train_one_epoch([{"sim_full": torch.from_numpy(sim).to(dtype),
                                 "real_full": torch.from_numpy(real).to(dtype)}])
            return grads
        finally:
            torch.set_default_dtype(torch.float32)

    # both runs replay the draws recorded for trainer_step.npz, so the fp32 run IS that step
    z = np.load(os.path.join(HERE, "trainer_step.npz"))
    draws = [(str(n), torch.from_numpy(z[f"rng_{i}"])) for i, n in enumerate(z["rng_names"])]
    orig = {n: getattr(torch, n) for n in RNGRecorder.NAMES}
    pos = [0]

    def replay(name, dtype):
        def f(*a, **k):
            n, v = draws[pos[0]]
            pos[0] += 1
            assert n == name, (n, name)
            return v.to(dtype) if v.is_floating_point() else v.clone()
        return f

    grads = {}
    for dtype in (torch.float32, torch.float64):
        pos[0] = 0
        for n in RNGRecorder.NAMES:
            setattr(torch, n, replay(n, dtype))
        try:
            grads[dtype] = run(dtype)
        finally:
            for n, f in orig.items():
                setattr(torch, n, f)
        assert pos[0] == len(draws)
    g32, g64 = grads[torch.float32], grads[torch.float64]
    ref = z["grad_abs"]
    for i, n in enumerate(g32):  # the fp32 run reproduces trainer_step.npz
        if n.endswith(".bias") and "mlp_convs" in n:
            continue  # pre-BN conv biases: rounding noise only
        assert abs(g32[n].abs().sum().item() - ref[i]) <= 1e-5 * ref[i], n
    names = list(g32)
    out = {"param_names": np.array(names),
           "sk32": np.stack([gradient_sketch(g32[n].numpy(), i) for i, n in enumerate(names)]),
           "sk64": np.stack([gradient_sketch(g64[n].numpy(), i) for i, n in enumerate(names)]),
           "rel32": np.array([(g32[n] - g64[n]).norm().item() / max(g64[n].norm().item(), 1e-300)
                              for n in names]),
           "norm64": np.array([g64[n].norm().item() for n in names])}
    save("trainer_sketch.npz", **out)


def gen_ddim_hierarchical():
    """ddim_sample_loop's hierarchical branch (diffusion_model.py:278-280): N=4096 > global
    1024, 3 steps, eval mode; model.forward re-encodes the style every step."""
    cfg = Config(total_points=4096, global_points=1024)
    m = make_model(cfg).eval()
    dp = ref_dm.DiffusionProcess(cfg, device="cpu")
    cond = lidar_like_cloud(2003, 4096)[None]
    with RNGRecorder() as rec:
        x = dp.ddim_sample_loop(m, (1, 4096, 3), t32(cond), num_inference_steps=3)
    out = {"cond": cond, "out": x.numpy()}
    out.update(rec.pack("rng"))
    save("ddim_hier.npz", **out)


def gen_inference_cfg1():
    """BASELINE config 1: scripts/inference.py on CPU, 2048x3 .npy, 10 steps."""
    from utils.checkpoint import CheckpointManager
    from utils.ema import ExponentialMovingAverage
    import scripts.inference as inf

    cfg = Config(experiment_name="cfg1")
    m = make_model(cfg)
    opt = torch.optim.AdamW(m.parameters(), lr=1e-4)
    ema = ExponentialMovingAverage(m.parameters(), decay=0.999)
    CheckpointManager(cfg.checkpoint_dir, cfg.experiment_name).save(m, opt, ema, epoch=0)
    src = lidar_like_cloud(1002, 2048) * np.float32(25.0) + np.float32(3.0)
    ref = lidar_like_cloud(2002, 2048) * np.float32(40.0) - np.float32(1.0)
    os.makedirs("cfg1", exist_ok=True)
    np.save("cfg1/src.npy", src)
    np.save("cfg1/ref.npy", ref)
    sys.argv = ["inference.py", "--checkpoint", "checkpoints/cfg1/ckpt_epoch_0000.pth",
                "--source", "cfg1/src.npy", "--reference", "cfg1/ref.npy",
                "--output", "cfg1/out/out.npy", "--device", "cpu", "--num_steps", "10"]
    with RNGRecorder() as rec:
        inf.main()
    res = np.load("cfg1/out/out.npy")
    out = {"src": src, "ref": ref, "out": res}
    out.update(rec.pack("rng"))
    save("inference_cfg1.npz", **out)


if __name__ == "__main__":
    which = sys.argv[1:] or ["geometry", "encoder", "noise", "hier", "sched", "sampling",
                             "trainer", "cfg1", "trainer_sketch"]
    fns = {"geometry": gen_geometry, "encoder": gen_encoder, "noise": gen_noise_predictor,
           "hier": gen_hierarchical, "sched": gen_schedule_and_losses, "sampling": gen_sampling,
           "trainer": gen_trainer_and_checkpoint, "cfg1": gen_inference_cfg1,
           "trainer_sketch": gen_trainer_sketch, "ddim_hier": gen_ddim_hierarchical}
    for w in which:
        torch.manual_seed(0)
        fns[w]()
