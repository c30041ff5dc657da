"""Host-side logic around the hot path (CPU only): checkpoint format and safe loading, EMA,
the LR schedule, the inference normaliser.  Pinned by the reference's checkpoint manifest
(tests/golden/checkpoint_manifest.json, written from a checkpoint the reference saved) and by
the formulas cited from the reference sources."""
import io
import json
import math
import os
import pickletools
import zipfile

import numpy as np
import pytest
import torch

from conftest import GOLDEN


@pytest.fixture()
def tiny_model(tmp_path, monkeypatch):
    from detweights import load_into
    from pointcloud_style_transfer_amd.config.config import Config
    from pointcloud_style_transfer_amd.models.diffusion_model import PointCloudDiffusionModel

    monkeypatch.chdir(tmp_path)
    cfg = Config(total_points=4096, global_points=1024, use_amp=False,
                 gradient_accumulation_steps=1, experiment_name="golden")
    m = PointCloudDiffusionModel(cfg)
    load_into(m)
    return cfg, m


def _pickle_globals(path):
    seen = set()
    with zipfile.ZipFile(path) as zf:
        pkl = [n for n in zf.namelist() if n.endswith("data.pkl")][0]
        for op, arg, _ in pickletools.genops(io.BytesIO(zf.read(pkl))):
            if op.name in ("GLOBAL", "STACK_GLOBAL") and arg:
                seen.add(str(arg).replace(" ", "."))
    return sorted(g for g in seen if "(" not in g)


def test_checkpoint_matches_reference_format(tiny_model):
    from pointcloud_style_transfer_amd.utils.checkpoint import CheckpointManager, safe_load
    from pointcloud_style_transfer_amd.utils.ema import ExponentialMovingAverage
    from pointcloud_style_transfer_amd.config.config import Config

    with open(os.path.join(GOLDEN, "checkpoint_manifest.json")) as f:
        man = json.load(f)
    cfg, m = tiny_model
    opt = torch.optim.AdamW(m.parameters(), lr=cfg.learning_rate, weight_decay=cfg.weight_decay,
                            betas=(0.9, 0.95))
    # one optimizer step so the AdamW state exists, as in the reference's checkpoint
    for p in m.parameters():
        p.grad = torch.ones_like(p) * 1e-3
    opt.step()
    ema = ExponentialMovingAverage(m.parameters(), decay=cfg.ema_decay)
    cm = CheckpointManager(cfg.checkpoint_dir, cfg.experiment_name)
    cm.save(m, opt, ema, epoch=3, is_best=True)
    d = os.path.join(cfg.checkpoint_dir, cfg.experiment_name)
    assert sorted(os.listdir(d)) == man["files"]
    path = os.path.join(d, "ckpt_epoch_0003.pth")
    # the same pickle globals as the reference's file -- Config under config.config
    assert _pickle_globals(path) == man["pickle_globals"]
    ck = safe_load(path)
    assert sorted(ck.keys()) == man["top_keys"]
    assert ck["epoch"] == man["epoch"]
    assert isinstance(ck["config"], Config)
    for k, v in man["config_fields"].items():
        assert getattr(ck["config"], k) == v, k
    assert [[k, list(v.shape), str(v.dtype)] for k, v in ck["model_state_dict"].items()] \
        == man["model_state_dict"]
    assert sorted(ck["optimizer_state_dict"].keys()) == man["optimizer_keys"]
    assert len(ck["optimizer_state_dict"]["state"]) == man["optimizer_n_state"]
    assert sorted(ck["optimizer_state_dict"]["state"][0].keys()) == man["optimizer_state_keys"]
    assert sorted(ck["ema_state_dict"].keys()) == man["ema_keys"]
    assert ck["ema_state_dict"]["decay"] == man["ema_decay"]
    assert [list(p.shape) for p in ck["ema_state_dict"]["shadow_params"]] == man["ema_shapes"]
    # resume: CheckpointManager.load returns epoch + 1 and restores the weights
    from pointcloud_style_transfer_amd.models.diffusion_model import PointCloudDiffusionModel

    m2 = PointCloudDiffusionModel(cfg)
    opt2 = torch.optim.AdamW(m2.parameters(), lr=cfg.learning_rate)
    ema2 = ExponentialMovingAverage(m2.parameters(), decay=0.5)
    assert cm.load(m2, opt2, ema2) == 4
    for (k, a), b in zip(m.state_dict().items(), m2.state_dict().values()):
        assert torch.equal(a, b), k
    assert ema2.decay == cfg.ema_decay


def test_safe_load_refuses_arbitrary_globals(tmp_path):
    from pointcloud_style_transfer_amd.utils.checkpoint import safe_load

    class Evil:
        def __reduce__(self):
            return (os.system, ("true",))

    p = tmp_path / "evil.pth"
    torch.save({"x": Evil()}, p)
    with pytest.raises(Exception):
        safe_load(str(p))


def test_ema_matches_reference_formula():
    from pointcloud_style_transfer_amd.utils.ema import ExponentialMovingAverage

    torch.manual_seed(0)
    ps = [torch.nn.Parameter(torch.randn(5, 3)), torch.nn.Parameter(torch.randn(7)),
          torch.nn.Parameter(torch.randn(2), requires_grad=False)]
    ema = ExponentialMovingAverage(ps, decay=0.9)
    assert len(ema.shadow_params) == 2
    want = [p.detach().clone() for p in ps[:2]]
    for _ in range(3):
        with torch.no_grad():
            for p in ps:
                p.add_(0.5)
        ema.update()
        want = [0.9 * w + 0.1 * p.detach() for w, p in zip(want, ps[:2])]  # ema.py:39-53
    for w, s in zip(want, ema.shadow_params):
        torch.testing.assert_close(s, w, rtol=1e-6, atol=1e-6)
    before = [p.detach().clone() for p in ps]
    ema.apply_shadow()
    for p, s in zip(ps[:2], ema.shadow_params):
        assert torch.equal(p.data, s)
    ema.restore()
    for p, b in zip(ps, before):
        assert torch.equal(p.data, b)
    st = ema.state_dict()
    assert set(st) == {"decay", "shadow_params"} and st["decay"] == 0.9


def test_cosine_with_warmup_schedule():
    from pointcloud_style_transfer_amd.training.trainer import CosineWithWarmupLR

    p = torch.nn.Parameter(torch.zeros(1))
    opt = torch.optim.AdamW([p], lr=1e-4)
    s = CosineWithWarmupLR(opt, warmup_epochs=20, total_epochs=200, min_lr_ratio=0.01)
    lrs = []
    for _ in range(200):
        s.step()
        lrs.append(opt.param_groups[0]["lr"])
    # trainer.py:20-34
    assert lrs[0] == pytest.approx(1e-4 / 20)
    assert lrs[19] == pytest.approx(1e-4)
    e = 100
    prog = (e - 20) / 180
    assert lrs[e - 1] == pytest.approx(1e-4 * (0.01 + 0.5 * 0.99 * (1 + math.cos(math.pi * prog))))
    assert lrs[-1] == pytest.approx(1e-6)


def test_normalizer_matches_oracle():
    from oracle import oracle as O
    from pointcloud_style_transfer_amd.data.preprocessing import PointCloudPreprocessor

    rng = np.random.default_rng(7)
    pts = (rng.standard_normal((5000, 3)) * [30, 20, 2] + [100, -50, 3]).astype(np.float64)
    pp = PointCloudPreprocessor()
    n, prm = pp.normalize_point_cloud(pts)
    n2, prm2 = O.normalize_point_cloud(pts)
    np.testing.assert_array_equal(n, n2)
    assert n.dtype == np.float64 and np.abs(n).max() <= 1.8 + 1e-9  # callers cast to f32
    back = pp.denormalize_point_cloud(n, prm)
    np.testing.assert_array_equal(back, O.denormalize_point_cloud(n2, prm2))
    np.testing.assert_allclose(back, pts, rtol=1e-5, atol=1e-4)


def test_inference_requires_gpu():
    """No CPU fallback: the entry point refuses to run without the HIP device."""
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from pointcloud_style_transfer_amd.scripts.inference import DiffusionInference

    with pytest.raises(RuntimeError, match="HIP"):
        DiffusionInference("nonexistent.pth", "cuda")


@pytest.mark.parametrize("device", ["cpu", "meta"])
def test_inference_rejects_non_hip_device(device):
    """`--device cpu` raises (the reference falls back to the CPU at inference.py:65; this build
    has no CPU path) -- on any machine, with or without a GPU."""
    from pointcloud_style_transfer_amd.scripts.inference import DiffusionInference

    with pytest.raises(RuntimeError, match="HIP path only"):
        DiffusionInference("nonexistent.pth", device)


def test_ema_swap_bumps_parameter_versions():
    """apply_shadow / restore must be visible to caches keyed on the parameter's version
    (NoisePredictor.packed): a p.data.copy_ would not bump it."""
    from pointcloud_style_transfer_amd.utils.ema import ExponentialMovingAverage

    lin = torch.nn.Linear(4, 3)
    ema = ExponentialMovingAverage(lin.parameters(), decay=0.5)
    with torch.no_grad():
        lin.weight.add_(1.0)
    ema.update()
    v0 = lin.weight._version
    w_raw = lin.weight.detach().clone()
    ema.apply_shadow()
    assert lin.weight._version > v0
    assert not torch.equal(lin.weight, w_raw)
    v1 = lin.weight._version
    ema.restore()
    assert lin.weight._version > v1
    assert torch.equal(lin.weight, w_raw)


def test_noise_predictor_pack_follows_ema_swap():
    """The packed weight stream is rebuilt after apply_shadow and after restore (the pack key
    is (data_ptr, _version) of every parameter)."""
    from pointcloud_style_transfer_amd.config.config import Config
    from pointcloud_style_transfer_amd.models.diffusion_model import NoisePredictor
    from pointcloud_style_transfer_amd.utils.ema import ExponentialMovingAverage

    npred = NoisePredictor(Config(make_dirs=False))
    ema = ExponentialMovingAverage(npred.parameters(), decay=0.5)
    key = lambda: tuple((p.data_ptr(), p._version) for p in npred.parameters())  # noqa: E731
    k0 = key()
    with torch.no_grad():
        for p in npred.parameters():
            p.mul_(0.5)
    ema.update()
    k1 = key()
    ema.apply_shadow()
    k2 = key()
    ema.restore()
    k3 = key()
    assert len({k0, k1, k2, k3}) == 4


def test_hip_wrappers_run_on_the_tensors_device(monkeypatch):
    """Every public ctypes wrapper is device-guarded, and the guard makes the tensors' device
    current when the caller's current device differs (a model on cuda:1 without
    torch.cuda.set_device must not launch on cuda:0)."""
    import inspect
    import types

    from pointcloud_style_transfer_amd import _hip

    calling = [n for n, f in vars(_hip).items() if inspect.isfunction(f) and not n.startswith("_")
               and "_call(" in inspect.getsource(f)]
    assert calling and all(getattr(getattr(_hip, n), "device_guarded", False) for n in calling), \
        [n for n in calling if not getattr(getattr(_hip, n), "device_guarded", False)]

    entered = []

    class FakeDev:
        def __init__(self, idx):
            self.idx = idx

        def __enter__(self):
            entered.append(self.idx)

        def __exit__(self, *a):
            return False

    monkeypatch.setattr(_hip.torch.cuda, "current_device", lambda: 0)
    monkeypatch.setattr(_hip.torch.cuda, "device", FakeDev)
    seen = []
    f = _hip._on_tensor_device(lambda *a, **k: seen.append(a) or "ok")
    t1 = types.SimpleNamespace(is_cuda=True, device=types.SimpleNamespace(index=1))
    t0 = types.SimpleNamespace(is_cuda=True, device=types.SimpleNamespace(index=0))
    assert f(3.0, t1) == "ok" and entered == [1]
    assert f(t0) == "ok" and entered == [1]          # already current: no switch
    assert f((t1, None)) == "ok" and entered == [1, 1]  # tuple handle (knn3_query)
    assert f(torch.zeros(2)) == "ok" and entered == [1, 1]  # CPU tensor: no switch


def test_bf16_packing_follows_the_solo_kernel_read_schedule():
    """packing.pack_blob(BF16), the stream of noise_mlp_solo_kernel: replaying that kernel's
    consumption order (csrc/noise_mlp.hip solo::: h2 rb-major, x, per layer W2(15) of the previous
    layer then W1(0), then W1(k), W2(k-1) for k = 1..15, the tail W2(15), out0, out1, out2)
    recovers every weight of every layer exactly (as bf16), the layer-0 W2 slot is zero, and the
    blob is 55 superparts of 64 fragments (the kernel's DMA unit)."""
    import torch

    from pointcloud_style_transfer_amd import packing
    from pointcloud_style_transfer_amd.model_spec import state_dict_shapes
    from detweights import deterministic_state

    sd = deterministic_state(state_dict_shapes())
    pre = "noise_predictor"
    blob = packing.pack_blob(sd, packing.BF16)
    assert len(blob) == 55 * packing.SUPERPART
    vals = torch.from_numpy(blob.copy()).view(torch.bfloat16).float().numpy()
    frags = vals.reshape(-1, 512)
    km = packing._kmap16(16)                    # [S, 64, 8]
    r = np.arange(64) & 15
    pos = [0]
    got = {}

    def take(name, rb, step):
        fr = frags[pos[0]].reshape(64, 8)
        pos[0] += 1
        if name is None:
            assert (fr == 0).all()
            return
        W = got.setdefault(name, {})
        for lane in range(64):
            for j in range(8):
                W[(rb * 16 + r[lane], int(km[step, lane, j]))] = fr[lane, j]

    def dense(name, nrb, nks):
        for rb in range(nrb):
            for ks in range(nks):
                take(name, rb, ks)

    dense("point_encoder.2", 16, 4)
    dense("point_encoder.4", 16, 8)
    for layer in range(6):
        for rb in range(16):
            take(f"layers.{layer - 1}.2" if layer else None, rb, 15)
        for k in range(16):
            for rr in range(2):
                for ks in range(8):
                    take(f"layers.{layer}.0", 2 * k + rr, ks)
            if k:
                for rb in range(16):
                    take(f"layers.{layer}.2", rb, k - 1)
    for rb in range(16):
        take("layers.5.2", rb, 15)
    dense("output_mlp.0", 16, 8)
    dense("output_mlp.2", 8, 8)
    dense("output_mlp.4", 1, 4)
    assert pos[0] == 212 + 192 + 6 * 512
    assert (frags[pos[0]:] == 0).all()
    for name, W in got.items():
        ref = torch.from_numpy(sd[f"{pre}.{name}.weight"]).bfloat16().float().numpy()
        O, K = ref.shape
        seen = np.full((max(O, 16), K), np.nan, np.float32)
        for (o, k), v in W.items():
            seen[o, k] = v
        np.testing.assert_array_equal(seen[:O], ref, err_msg=name)
        if O < 16:
            assert (seen[O:] == 0).all(), name


def test_solo16_kernel_schedule_emulated_matches_the_network():
    """tests/solo_emulator.py replays noise_mlp_solo_kernel's dataflow lane by lane over the packed
    BF16 blob (fragment order, v_mfma_f32_16x16x32_bf16 layouts, bias placement, the hidden-chunk
    software pipeline, bf16 operand rounding) for one wave's 32 points; it must equal the exact-f32
    network (oracle.noise_predictor) within the bf16 mode's normwise bound (3e-2, as the GPU
    tests) -- a schedule or layout error gives O(1) differences."""
    import solo_emulator as SE
    from pointcloud_style_transfer_amd import packing
    from pointcloud_style_transfer_amd.model_spec import state_dict_shapes
    from detweights import deterministic_state
    import oracle.oracle as O

    sd = deterministic_state(state_dict_shapes())
    blob = packing.pack_blob(sd, packing.BF16)
    bias = packing.pack_bias(sd)
    rng = np.random.default_rng(11)
    pts = rng.standard_normal((1, 32, 3)).astype(np.float32)
    t = np.array([731])
    style = (rng.standard_normal((1, 256)) * 0.3).astype(np.float32)
    ref = O.noise_predictor(sd, pts, t, style).reshape(-1, 3)
    pre = "noise_predictor"
    cond = (sd[pre + ".point_encoder.4.bias"] + O._linear(sd, pre + ".time_proj", O.time_embedding(t, 128))
            + O._linear(sd, pre + ".style_proj", style)).astype(np.float32)
    out = SE.run_wave(blob, bias, pts[0], np.repeat(cond, 32, axis=0))
    err = np.linalg.norm(out - ref) / np.linalg.norm(ref)
    assert err < 3e-2, err


def test_chaos_floor_constants_match_profile():
    """The end-to-end gates of tests/test_gpu_configs.py quote the chaos floor measured by
    tools/chaos_floor.py (profiles/r04/chaos_floor.json: 10, 50 and 1000 steps); keep the two in
    step."""
    import json

    import test_gpu_configs as G

    from conftest import REPO

    rec = json.load(open(os.path.join(REPO, "profiles", "r04", "chaos_floor.json")))
    assert rec["weights"] == "det"
    for steps, consts in (("50", G.CHAOS_FLOOR_50), ("10", G.CHAOS_FLOOR_10),
                          ("1000", G.CHAOS_FLOOR_1000)):
        for k, v in consts.items():
            assert abs(rec["runs"][steps][k] - v) <= 1e-3 * v, (steps, k)


def test_fused_adamw_resumes_a_non_fused_checkpoint():
    """the trainer's AdamW is fused, and load_state_dict takes the saved
    param groups -- a checkpoint written by the reference (non-fused AdamW) carries fused=None.
    The trainer's pre-hook (trainer.keep_fused) keeps the groups fused and loads `step` as
    float32 (torch's rule for fused state), so GradScaler's found_inf protocol still applies.
    CPU fused AdamW exercises the same torch code path as the device one."""
    import torch.optim as optim

    from pointcloud_style_transfer_amd.training.trainer import keep_fused

    p = [torch.nn.Parameter(torch.randn(8, 4)), torch.nn.Parameter(torch.randn(4))]
    ref_opt = optim.AdamW(p, lr=1e-3, betas=(0.9, 0.95))   # the reference's optimizer
    for q in p:
        q.grad = torch.randn_like(q)
    ref_opt.step()
    saved = ref_opt.state_dict()
    assert saved["param_groups"][0].get("fused") is None
    opt = optim.AdamW(p, lr=1e-3, betas=(0.9, 0.95), fused=True)
    opt.register_load_state_dict_pre_hook(keep_fused)
    opt.load_state_dict(saved)
    g = opt.param_groups[0]
    assert g["fused"] is True and g["foreach"] is None
    assert opt.state[p[0]]["step"].dtype == torch.float32
    # the amp-scaling protocol GradScaler uses with a fused optimizer
    opt.grad_scale, opt.found_inf = torch.ones(()), torch.zeros(())
    before = p[0].detach().clone()
    opt.step()
    assert float(opt.state[p[0]]["step"]) == 2.0
    assert not torch.equal(before, p[0].detach())


def test_fused_block_row_limit_matches_the_kernels():
    """The fused residual-block dispatch (models/_autograd.py) sends M rows to pcst_resblock_*16
    only while M * 1024 < 2^31, the kernels' own bound; larger M takes the two-GEMM path."""
    from pointcloud_style_transfer_amd.models import _autograd as A

    lim = (2 ** 31 - 1) // 1024
    assert A.fused_block_rows_ok(lim) and lim * 1024 < 2 ** 31
    assert not A.fused_block_rows_ok(lim + 1) and (lim + 1) * 1024 >= 2 ** 31
    assert A.fused_block_rows_ok(8 * 30000)          # the trainer's batch
    assert not A.fused_block_rows_ok(70 * 30000)     # 70 clouds: the unfused path


def test_generator_rng_randn_like_keeps_the_dtype():
    """rng.GeneratorRNG.randn_like keeps x's dtype, as TorchRNG.randn_like (torch.randn_like)
    does, so q_sample's noise has the same dtype whichever source the thread installed."""
    from pointcloud_style_transfer_amd import rng

    for dt in (torch.float32, torch.float64, torch.float16):
        x = torch.zeros(3, 4, dtype=dt)
        assert rng.GeneratorRNG(1).randn_like(x).dtype == dt
        assert rng.TorchRNG().randn_like(x).dtype == dt
    a = rng.GeneratorRNG(5).randn_like(torch.zeros(2, 3))
    b = rng.GeneratorRNG(5).randn_like(torch.zeros(2, 3))
    assert torch.equal(a, b)


def test_dense_voxel_boxes_are_collision_free():
    """Every box of csrc/voxel.hip's PCST_DENSE_BOXES (the voxel boxes that take the dense grid instead
    of the hash table) holds no two voxel coordinates whose int32 xor-hash -- the reference's
    voxel_hash, diffusion_model.py:90 -- is equal, so inside it a hash group is exactly one voxel
    (the dense path's grouping is the reference's); and the check itself finds the collisions
    the dense path must avoid (the 197 x 17 x 3 box holds (190, 5, 1) and (196, 16, 2))."""
    import re

    src = open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                            "pointcloud_style_transfer_amd", "csrc", "voxel.hip")).read()
    table = src[src.index("#define PCST_DENSE_BOXES"):src.index("__device__", src.index("#define PCST_DENSE_BOXES"))]
    boxes = [tuple(int(v) for v in m) for m in re.findall(r"\{(\d+), (\d+), (\d+)\}", table)]
    assert len(boxes) >= 10

    def hashes(d):
        x = np.arange(d[0], dtype=np.int64)[:, None, None]
        y = np.arange(d[1], dtype=np.int64)[None, :, None]
        z = np.arange(d[2], dtype=np.int64)[None, None, :]
        return (((x * 73856093) & 0xFFFFFFFF) ^ ((y * 19349663) & 0xFFFFFFFF)
                ^ ((z * 83492791) & 0xFFFFFFFF)).ravel()

    for d in boxes:
        h = hashes(d)
        assert np.unique(h).size == h.size, d
    h = hashes((197, 17, 3))
    assert np.unique(h).size < h.size
    assert h[np.ravel_multi_index((190, 5, 1), (197, 17, 3))] == h[np.ravel_multi_index((196, 16, 2), (197, 17, 3))]
