"""Kernel-side cross-stream signal (pcst_signal_write / pcst_signal_wait, _hip.DeviceSignal): the
sampling loop's loop -> side dependency.  Work enqueued after a wait must see everything the
producer stream wrote before the matching signal, under load and across many rounds."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_signal_orders_consumer_after_producer():
    from pointcloud_style_transfer_amd import _hip

    dev = torch.device("cuda", 0)
    prod = torch.cuda.Stream(device=dev, priority=-1)
    cons = torch.cuda.Stream(device=dev)
    sig = _hip.DeviceSignal(dev)
    a = torch.randn(2048, 2048, device=dev)
    buf = torch.zeros(2048, 2048, device=dev)
    outs = []
    for r in range(20):
        prod.wait_stream(torch.cuda.current_stream())
        prod.wait_stream(cons)  # the previous round's copy has read buf
        with torch.cuda.stream(prod):
            # a long producer chain ending in the value the consumer must see
            y = a
            for _ in range(4):
                y = torch.tanh(y @ a) * 0.5
            buf.copy_(y + float(r))
            sig.signal(prod)
        sig.wait(cons)
        with torch.cuda.stream(cons):
            outs.append((buf.clone(), r))
        buf.record_stream(cons)
    torch.cuda.synchronize()
    assert not sig.timed_out()
    y = a
    for _ in range(4):
        y = torch.tanh(y @ a) * 0.5
    for got, r in outs:
        torch.testing.assert_close(got, y + float(r), rtol=0, atol=0)


def test_signal_values_are_monotonic_per_flag():
    from pointcloud_style_transfer_amd import _hip

    dev = torch.device("cuda", 0)
    s = torch.cuda.Stream(device=dev)
    sig = _hip.DeviceSignal(dev)
    for _ in range(5):
        sig.signal(s)
        sig.wait(s)  # the same stream: already satisfied when it runs
    torch.cuda.synchronize()
    assert int(sig.flag[0].item()) == 5 and sig.value == 5 and not sig.timed_out()


def test_wait_that_times_out_is_reported():
    """A wait whose value is never signalled gives up after its poll bound (an argument of the
    call), lets its stream go on, and check() raises SignalTimeout; the MLP's last-group wait
    (pcst_noise_mlp_ex's wait) reports through the same error word."""
    from pointcloud_style_transfer_amd import _hip

    dev = torch.device("cuda", 0)
    s = torch.cuda.Stream(device=dev)
    sig = _hip.DeviceSignal(dev, max_polls=2000)
    sig.value = 1  # a value no kernel will ever write
    sig.wait(s)
    torch.cuda.synchronize()
    assert sig.timed_out()
    with pytest.raises(_hip.SignalTimeout):
        sig.check()

    from pointcloud_style_transfer_amd import packing
    from pointcloud_style_transfer_amd.config.config import Config
    from pointcloud_style_transfer_amd.models.diffusion_model import NoisePredictor

    torch.manual_seed(4)
    npred = NoisePredictor(Config(make_dirs=False, precision="bf16")).to(dev).eval()
    assert npred.precision_code == packing.BF16
    pts = torch.randn(2 * 4096, 3, device=dev)
    with torch.no_grad():
        cond = npred.cond(torch.tensor([5, 5], device=dev), torch.randn(2, 256, device=dev))
        blob, bias = npred.packed()[:2]
        ref = _hip.noise_mlp(pts, 4096, cond, blob, bias, npred.precision_code)
        sig2 = _hip.DeviceSignal(dev, max_polls=2000)
        sig2.value = 1
        out = _hip.noise_mlp(pts, 4096, cond, blob, bias, npred.precision_code, wait=sig2)
    torch.cuda.synchronize()
    assert torch.equal(out, ref)  # the rows are written before the wait
    with pytest.raises(_hip.SignalTimeout):
        sig2.check()
    assert int(sig2.flag[2].item()) == 0  # the work-group counter is reset for the next call


def _small_model(dev, precision="bf16"):
    from pointcloud_style_transfer_amd.config.config import Config
    from pointcloud_style_transfer_amd.models.diffusion_model import (DiffusionProcess,
                                                                        PointCloudDiffusionModel)

    cfg = Config(make_dirs=False, precision=precision, global_points=4096)
    torch.manual_seed(11)
    model = PointCloudDiffusionModel(cfg).to(dev).eval()
    return cfg, model, DiffusionProcess(cfg, device=str(dev))


def test_guided_loop_raises_when_a_step_wait_times_out(monkeypatch):
    """The sampling loop reads its flags' timeout words once at its end: a producer that never
    signals (simulated: signal() bumps the host value but writes nothing, and the values handed
    to producing launches -- the MLP's start signal, the kNN build's completion flag -- go to a
    scratch word instead of the flag) makes the loop raise instead of returning what the
    unsynchronised kNN query computed."""
    import ctypes

    from pointcloud_style_transfer_amd import _hip
    from pointcloud_style_transfer_amd.models import diffusion_model as dm
    from pointcloud_style_transfer_amd.synthetic import lidar_like_cloud

    dev = torch.device("cuda", 0)
    cfg, model, dp = _small_model(dev)
    src = torch.from_numpy(lidar_like_cloud(1000, 16384)[None]).to(dev)
    cond = torch.from_numpy(lidar_like_cloud(2000, 16384)[None]).to(dev)
    with torch.no_grad():
        dp.guided_sample_loop(model, src, cond, 3, 7.5)  # healthy: no raise
        monkeypatch.setattr(dm, "SIGNAL_MAX_POLLS", 2000)

        def silent(self, stream):
            self.value += 1

        scratch = torch.zeros(4, dtype=torch.int32, device=dev)
        real_next = _hip.DeviceSignal.next_value

        def silent_next(self):
            _, v = real_next(self)
            return ctypes.c_void_p(scratch.data_ptr()), v

        monkeypatch.setattr(_hip.DeviceSignal, "signal", silent)
        monkeypatch.setattr(_hip.DeviceSignal, "next_value", silent_next)
        with pytest.raises(_hip.SignalTimeout):
            dp.guided_sample_loop(model, src, cond, 3, 7.5)


def test_two_loops_on_two_threads_match_serial():
    """Two guided loops running at the same time from two host threads on one device (each with
    its own seeded draws, rng.GeneratorRNG) give the bits of the same loops run one after the
    other: the loop's streams are per thread and its flags and events per call."""
    import threading

    from pointcloud_style_transfer_amd import rng
    from pointcloud_style_transfer_amd.synthetic import lidar_like_cloud, standard_normal

    dev = torch.device("cuda", 0)
    cfg, model, dp = _small_model(dev)
    model.noise_predictor.packed()  # pack once, before the threads
    n = 16384
    jobs = []
    for k in range(2):
        jobs.append(tuple(torch.from_numpy(a).to(dev) for a in (
            lidar_like_cloud(1000 + k, n)[None], lidar_like_cloud(2000 + k, n)[None],
            standard_normal(3000 + k, (1, n, 3)))))

    def run(k, out):
        src, cond, xT = jobs[k]
        with torch.no_grad(), rng.use(rng.GeneratorRNG(100 + k)):
            out[k] = dp.guided_sample_loop(model, src, cond, 12, 7.5, x_T=xT)
        torch.cuda.current_stream(dev).synchronize()

    serial = {}
    for k in range(2):
        run(k, serial)
    conc = {}
    ths = [threading.Thread(target=run, args=(k, conc)) for k in range(2)]
    for t in ths:
        t.start()
    for t in ths:
        t.join(timeout=120)
    assert all(not t.is_alive() for t in ths)
    torch.cuda.synchronize()
    for k in range(2):
        assert torch.equal(conc[k], serial[k]), k


def test_more_loops_than_hw_queues_match_serial():
    """Six guided loops at once from six host threads on one device -- more loops than the
    GPU_MAX_HW_QUEUES hardware queues (4) HIP spreads its streams over -- give the bits of the same
    loops run one after the other, with no SignalTimeout: one loop at a time holds the device's
    overlapped layout (diffusion_model.overlap_slot); the others run the single-stream layout, which
    has no cross-stream waits to deadlock on a shared queue."""
    import threading

    from pointcloud_style_transfer_amd import rng
    from pointcloud_style_transfer_amd.synthetic import lidar_like_cloud, standard_normal

    dev = torch.device("cuda", 0)
    cfg, model, dp = _small_model(dev)
    model.noise_predictor.packed()
    n, K = 8192, 6
    jobs = [tuple(torch.from_numpy(a).to(dev) for a in (
        lidar_like_cloud(1100 + k, n)[None], lidar_like_cloud(2100 + k, n)[None],
        standard_normal(3100 + k, (1, n, 3)))) for k in range(K)]
    errors = []

    def run(k, out):
        try:
            src, cond, xT = jobs[k]
            with torch.no_grad(), rng.use(rng.GeneratorRNG(200 + k)):
                out[k] = dp.guided_sample_loop(model, src, cond, 6, 7.5, x_T=xT)
            torch.cuda.current_stream(dev).synchronize()
        except Exception as e:  # noqa: BLE001  (reported by the main thread)
            errors.append((k, repr(e)))

    serial = {}
    for k in range(K):
        run(k, serial)
    conc = {}
    ths = [threading.Thread(target=run, args=(k, conc)) for k in range(K)]
    for t in ths:
        t.start()
    for t in ths:
        t.join(timeout=120)
    assert all(not t.is_alive() for t in ths)
    torch.cuda.synchronize()
    assert not errors, errors
    for k in range(K):
        assert torch.equal(conc[k], serial[k]), k


def test_mlp_start_signal_orders_the_side_stream():
    """pcst_noise_mlp_ex's start signal (the MLP launch publishes the loop -> side flag as it
    begins): the side stream's work waits for it and sees what the loop stream wrote before the
    MLP; the MLP's rows equal the plain launch's; f32 precision takes the separate-launch form.
    signal_all (the flag once every work-group has begun, counted on the signal's word 3): the
    same ordering, and the counter is zero again after every launch."""
    from pointcloud_style_transfer_amd import _hip
    from pointcloud_style_transfer_amd.config.config import Config
    from pointcloud_style_transfer_amd.models.diffusion_model import NoisePredictor

    dev = torch.device("cuda", 0)
    loop = torch.cuda.Stream(device=dev)
    side = torch.cuda.Stream(device=dev)
    for prec, every in (("bf16", False), ("fp32", False), ("bf16", True), ("fp32", True)):
        torch.manual_seed(5)
        npred = NoisePredictor(Config(make_dirs=False, precision=prec)).to(dev).eval()
        pts = torch.randn(2 * 4096, 3, device=dev)
        with torch.no_grad():
            cond = npred.cond(torch.tensor([7, 7], device=dev), torch.randn(2, 256, device=dev))
            blob, bias = npred.packed()[:2]
            ref = _hip.noise_mlp(pts, 4096, cond, blob, bias, npred.precision_code)
            sig = _hip.DeviceSignal(dev, max_polls=1 << 24)
            buf = torch.zeros(8 << 20, device=dev)
            loop.wait_stream(torch.cuda.current_stream())
            side.wait_stream(torch.cuda.current_stream())
            outs = []
            for rep in range(3):
                with torch.cuda.stream(loop):
                    a = torch.randn(2048, 2048, device=dev)
                    for _ in range(3):
                        a = a @ a.T / 2048.0  # a delay on the loop stream before the MLP
                    buf.fill_(float(rep + 1))
                    start = sig.next_value()
                    sig.wait(side)
                    with torch.cuda.stream(side):
                        seen = buf.clone()  # ordered after the flag, hence after the fill
                    out = _hip.noise_mlp(pts, 4096, cond, blob, bias, npred.precision_code,
                                         signal=start, signal_all=every)
                outs.append((out, seen, rep))
            torch.cuda.synchronize()
        sig.check()
        assert int(sig.flag[0].item()) == 3
        assert int(sig.flag[3].item()) == 0, (prec, every)
        for out, seen, rep in outs:
            assert torch.equal(out, ref)
            assert bool((seen == float(rep + 1)).all()), (prec, rep)


def test_guided_loop_layouts_bit_identical(monkeypatch):
    """The sampling loop's three step layouts give the same bits on a small model at 1 and 3
    clouds: the rows layout (phase A beside the downsample, the voxel insert publishing the
    loop -> side flag, one placement launch, the MLP's last work-group waiting for phase A), the
    compact layout (the build beside the MLP, its flag written by the MLP launch as it begins)
    and the single-stream loop."""
    from pointcloud_style_transfer_amd.models import diffusion_model as dm
    from pointcloud_style_transfer_amd.synthetic import lidar_like_cloud, standard_normal

    dev = torch.device("cuda", 0)
    cfg, model, dp = _small_model(dev)
    for B in (1, 3):
        src = torch.from_numpy(np.stack([lidar_like_cloud(1000 + i, 16384) for i in range(B)])).to(dev)
        cond = torch.from_numpy(np.stack([lidar_like_cloud(2000 + i, 16384) for i in range(B)])).to(dev)
        xT = torch.from_numpy(np.stack([standard_normal(3000 + i, (16384, 3)) for i in range(B)])).to(dev)
        outs = []
        with torch.no_grad():
            for rows, overlap in ((True, True), (False, True), (True, False)):
                monkeypatch.setattr(dm, "ROWS_LAYOUT", rows)
                monkeypatch.setattr(dm, "OVERLAP_KNN_BUILD", overlap)
                torch.manual_seed(7)
                outs.append(dp.guided_sample_loop(model, src, cond, 8, 7.5, x_T=xT))
        assert torch.equal(outs[0], outs[1]), B
        assert torch.equal(outs[0], outs[2]), B


def test_guided_loop_voxel_prep_bit_identical(monkeypatch):
    """The step's CFG + DDIM update fused with the next downsample's statistics and zeroing
    (pcst_cfg_ddim_voxel_prep + pcst_voxel_downsample_copies_prepped, VOXEL_PREP) gives the bits
    of the separate update and full downsample, at 1 and 3 clouds."""
    from pointcloud_style_transfer_amd.models import diffusion_model as dm
    from pointcloud_style_transfer_amd.synthetic import lidar_like_cloud, standard_normal

    dev = torch.device("cuda", 0)
    cfg, model, dp = _small_model(dev)
    for B in (1, 3):
        src = torch.from_numpy(np.stack([lidar_like_cloud(1000 + i, 16384) for i in range(B)])).to(dev)
        cond = torch.from_numpy(np.stack([lidar_like_cloud(2000 + i, 16384) for i in range(B)])).to(dev)
        xT = torch.from_numpy(np.stack([standard_normal(3000 + i, (16384, 3)) for i in range(B)])).to(dev)
        outs = []
        with torch.no_grad():
            for on in (True, False):
                monkeypatch.setattr(dm, "VOXEL_PREP", on)
                torch.manual_seed(9)
                outs.append(dp.guided_sample_loop(model, src, cond, 6, 7.5, x_T=xT))
        assert torch.equal(outs[0], outs[1]), B


def test_guided_loop_pool_prep_bit_identical(monkeypatch):
    """The next downsample's pool-key histogram made by the step's update from the subset seed
    drawn one step ahead (POOL_PREP: pcst_cfg_ddim_voxel_prep's pool_seed, the insert skips the
    histogram) gives the bits of the loop that draws each seed at its downsample and builds the
    histogram in the insert, at 1 and 3 clouds; with VOXEL_PREP off the loop draws nothing ahead."""
    from pointcloud_style_transfer_amd.models import diffusion_model as dm
    from pointcloud_style_transfer_amd.synthetic import lidar_like_cloud, standard_normal

    dev = torch.device("cuda", 0)
    cfg, model, dp = _small_model(dev)
    for B in (1, 3):
        src = torch.from_numpy(np.stack([lidar_like_cloud(1100 + i, 16384) for i in range(B)])).to(dev)
        cond = torch.from_numpy(np.stack([lidar_like_cloud(2100 + i, 16384) for i in range(B)])).to(dev)
        xT = torch.from_numpy(np.stack([standard_normal(3100 + i, (16384, 3)) for i in range(B)])).to(dev)
        outs = []
        with torch.no_grad():
            for pool, prep in ((True, True), (False, True), (False, False)):
                monkeypatch.setattr(dm, "POOL_PREP", pool)
                monkeypatch.setattr(dm, "VOXEL_PREP", prep)
                torch.manual_seed(9)
                outs.append(dp.guided_sample_loop(model, src, cond, 6, 7.5, x_T=xT))
        assert torch.equal(outs[0], outs[1]), B
        assert torch.equal(outs[0], outs[2]), B


def test_pool_prepped_downsample_matches_plain():
    """pcst_voxel_downsample_copies_prepped with the pool histogram made by the update for its
    seed (pool = 1) keeps the same rows as the plain downsample of the same points and seed,
    over consecutive calls on one workspace (the emit clears the histogram between them)."""
    from pointcloud_style_transfer_amd import _hip

    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(3)
    C, N, T = 2, 60000, 15000
    ws = _hip.voxel_copies_workspace(C, N, 2, dev)
    x = torch.from_numpy(rng.standard_normal((C, N, 3)).astype(np.float32)).to(dev)
    src = torch.from_numpy(rng.standard_normal((C, N, 3)).astype(np.float32)).to(dev)
    coeffs = (np.float32(0.3), np.float32(0.95), np.float32(0.97), np.float32(0.24))
    for r in range(4):
        eps = torch.from_numpy(rng.standard_normal((2 * C, N, 3)).astype(np.float32)).to(dev)
        x_cat = torch.empty(2 * C, N, 3, device=dev)
        seed = 1234567 + 1000003 * r
        _hip.voxel_downsample(x, T, seed=seed, copies=2, ws=ws)  # the previous step's downsample
        x = _hip.cfg_ddim_voxel_prep(x, eps, src, 7.5, coeffs, x_cat, ws, pool_seed=seed)
        got = _hip.voxel_downsample(x, T, seed=seed, copies=2, ws=ws, prepped=True, pool=True)
        want = _hip.voxel_downsample(x, T, seed=seed, copies=2)
        assert torch.equal(got[1], want[1]) and torch.equal(got[0], want[0]), r


@pytest.mark.parametrize("C,N,with_src", [(1, 4096, True), (2, 4099, True), (3, 60000, False),
                                          (1, 120000, True)])
def test_cfg_voxel_prep_matches_update_and_plain_downsample(C, N, with_src):
    """pcst_cfg_ddim_voxel_prep's update (the four-point float4 path at N % 4 == 0, the per-point
    loop otherwise) writes the bits of pcst_cfg_ddim_step into x_out and both halves of x_cat,
    and its min / max partials prepare the same downsample as the plain one."""
    from pointcloud_style_transfer_amd import _hip

    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(N + C)
    T = N // 4
    x = torch.from_numpy(rng.standard_normal((C, N, 3)).astype(np.float32)).to(dev)
    eps = torch.from_numpy(rng.standard_normal((2 * C, N, 3)).astype(np.float32)).to(dev)
    src = torch.from_numpy(rng.standard_normal((C, N, 3)).astype(np.float32)).to(dev) if with_src else None
    coeffs = (np.float32(0.3), np.float32(0.95), np.float32(0.97), np.float32(0.24))
    ws = _hip.voxel_copies_workspace(C, N, 2, dev)
    x_cat = torch.empty(2 * C, N, 3, device=dev)
    got = _hip.cfg_ddim_voxel_prep(x, eps, src, 7.5, coeffs, x_cat, ws)
    want_cat = torch.empty(2 * C, N, 3, device=dev)
    want = _hip.cfg_ddim_step(x, eps[:C], eps[C:], src, 7.5, coeffs, x_cat=want_cat)
    assert torch.equal(got, want)
    assert torch.equal(x_cat, want_cat)
    a = _hip.voxel_downsample(got, T, seed=77, copies=2, ws=ws, prepped=True)
    b = _hip.voxel_downsample(got, T, seed=77, copies=2)
    assert torch.equal(a[1], b[1]) and torch.equal(a[0], b[0])


def test_waiters_launched_before_their_producer_on_a_saturated_device():
    """Forward progress of the product's in-kernel spin-waits ("Forward progress"):
    each waiter is queued BEFORE its producer's signal while a saturating kernel holds every CU
    (the bf16 noise MLP over 32 x 30000 points: 7500 work-groups of 512 threads, ~30 rounds), and
    completes without a timeout once the producer signals: (1) the voxel emit's wait for phase A
    before it places the coarse refs (pcst_voxel_downsample_rows: every emit work-group waits),
    (2) the MLP's last work-group's wait (pcst_noise_mlp_ex), (3) pcst_signal_wait.  The waiters'
    grids are far below the device's capacity (1 / 235 / 236 work-groups), so the producer's
    launches always find a CU; the results equal the unsynchronised computations'."""
    from pointcloud_style_transfer_amd import _hip
    from pointcloud_style_transfer_amd.config.config import Config
    from pointcloud_style_transfer_amd.models.diffusion_model import NoisePredictor

    dev = torch.device("cuda", 0)
    torch.manual_seed(12)
    npred = NoisePredictor(Config(make_dirs=False, precision="bf16")).to(dev).eval()
    rng = np.random.default_rng(12)
    big = torch.randn(64 * 30000, 3, device=dev)
    small = torch.randn(2 * 30000, 3, device=dev)
    N, M = 120000, 30000
    x = torch.from_numpy(rng.standard_normal((1, N, 3)).astype(np.float32)).to(dev)
    coarse = torch.randn(2, M, 3, device=dev)
    with torch.no_grad():
        cbig = npred.cond(torch.full((64,), 900, device=dev), torch.randn(64, 256, device=dev))
        csmall = npred.cond(torch.tensor([900, 900], device=dev), torch.randn(2, 256, device=dev))
        blob, bias = npred.packed()[:2]
        ref_small = _hip.noise_mlp(small, 30000, csmall, blob, bias, npred.precision_code)
        h_ref = _hip.knn3_rows_build(x, M, 2)
        _, xi_ref = _hip.voxel_downsample(x, M, seed=3, copies=2)
        _hip.knn3_rows_refs(h_ref, xi_ref)
        q_ref = _hip.knn3_rows_query(coarse, h_ref)
        h = _hip.knn3_rows_build(x, M, 2)
        torch.cuda.synchronize()
        prod = torch.cuda.Stream(device=dev)
        cons = torch.cuda.Stream(device=dev)
        s1, s2, s3 = (_hip.DeviceSignal(dev) for _ in range(3))
        for s in (prod, cons):
            s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(prod):  # the saturating kernel first, then the three signals
            _hip.noise_mlp(big, 30000, cbig, blob, bias, npred.precision_code)
            s1.signal(prod)
            s2.signal(prod)
            s3.signal(prod)
        with torch.cuda.stream(cons):  # the waiters, queued before the signals exist
            _, xi = _hip.voxel_downsample(x, M, seed=3, copies=2, rows=h, rows_wait=s1)
            out = _hip.noise_mlp(small, 30000, csmall, blob, bias, npred.precision_code, wait=s2)
            s3.wait(cons)
            q = _hip.knn3_rows_query(coarse, h)
        torch.cuda.synchronize()
    for s in (s1, s2, s3):
        assert not s.timed_out()
    assert torch.equal(xi, xi_ref)
    assert torch.equal(out, ref_small)
    assert torch.equal(q, q_ref)


def test_waiting_grids_larger_than_the_device_never_hold_every_cu():
    """The waits of phase B at many clouds ("Forward progress"): the rows downsample of
    16 clouds x 2 CFG rows (an emit launch of 3776 work-groups) is queued while its producer (phase A,
    knn3_rows_build with refs_sig, behind a saturating noise MLP on another stream) has not run.
    The emit then places nothing itself and phase B's own launch (at most max(CUs, rows) waiting
    work-groups) waits instead, so phase A finds CUs: no timeout, and the refs and the query equal
    the unsynchronised computation's.  (With the placement inside this emit, the 32-cloud step's
    waits ran into their poll bound: r6z.)"""
    from pointcloud_style_transfer_amd import _hip
    from pointcloud_style_transfer_amd.config.config import Config
    from pointcloud_style_transfer_amd.models.diffusion_model import NoisePredictor

    dev = torch.device("cuda", 0)
    torch.manual_seed(13)
    npred = NoisePredictor(Config(make_dirs=False, precision="bf16")).to(dev).eval()
    rng = np.random.default_rng(13)
    C, N, M = 16, 120000, 30000
    x = torch.from_numpy(rng.standard_normal((C, N, 3)).astype(np.float32)).to(dev)
    coarse = torch.randn(2 * C, M, 3, device=dev)
    big = torch.randn(64 * 30000, 3, device=dev)
    with torch.no_grad():
        cbig = npred.cond(torch.full((64,), 900, device=dev), torch.randn(64, 256, device=dev))
        blob, bias = npred.packed()[:2]
        h_ref = _hip.knn3_rows_build(x, M, 2)
        _, xi_ref = _hip.voxel_downsample(x, M, seed=4, copies=2)
        _hip.knn3_rows_refs(h_ref, xi_ref)
        q_ref = _hip.knn3_rows_query(coarse, h_ref)
        h = _hip.knn3_rows_build(x, M, 2)
        torch.cuda.synchronize()
        prod = torch.cuda.Stream(device=dev)
        cons = torch.cuda.Stream(device=dev)
        s1 = _hip.DeviceSignal(dev)
        for s in (prod, cons):
            s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(prod):  # phase A behind a saturating kernel
            _hip.noise_mlp(big, 30000, cbig, blob, bias, npred.precision_code)
            _hip.knn3_rows_build(x, M, 2, ws=h.ws, refs_sig=s1)
        with torch.cuda.stream(cons):  # the waiting placement, queued before phase A can run
            _, xi = _hip.voxel_downsample(x, M, seed=4, copies=2, rows=h, rows_wait=s1)
            cons.wait_stream(prod)
            q = _hip.knn3_rows_query(coarse, h)
        torch.cuda.synchronize()
    assert not s1.timed_out()
    assert h.placed
    assert torch.equal(xi, xi_ref)
    assert torch.equal(q, q_ref)


def test_multi_cu_fps_beside_a_saturating_kernel():
    """Forward progress of the multi-CU FPS's in-kernel exchange (geometry.hip fps_multi_kernel,
    DESIGN §3): its K = 30 work-groups are queued on one stream right behind a saturating kernel on
    another (the bf16 noise MLP over 64 x 30000 points, ~30 rounds of 512-thread work-groups), so
    they start one by one as the MLP's work-groups retire and the first ones poll for siblings that
    have no CU yet.  Each waits only for its siblings, which the finite MLP leaves CUs to: the
    samples equal the one-work-group kernel's (pcst_fps) and none is -1 (no poll gave up)."""
    from pointcloud_style_transfer_amd import _hip
    from pointcloud_style_transfer_amd.config.config import Config
    from pointcloud_style_transfer_amd.models.diffusion_model import NoisePredictor
    from pointcloud_style_transfer_amd.synthetic import lidar_like_cloud

    dev = torch.device("cuda", 0)
    torch.manual_seed(14)
    npred = NoisePredictor(Config(make_dirs=False, precision="bf16")).to(dev).eval()
    big = torch.randn(64 * 30000, 3, device=dev)
    xyz = torch.from_numpy(lidar_like_cloud(21, 30000)[None].astype(np.float32)).to(dev)
    start = torch.tensor([17], device=dev)
    with torch.no_grad():
        cbig = npred.cond(torch.full((64,), 900, device=dev), torch.randn(64, 256, device=dev))
        blob, bias = npred.packed()[:2]
        ref = torch.empty(1, 512, dtype=torch.int64, device=dev)
        _hip._call("pcst_fps", _hip._ptr(xyz), 1, 30000, 512, _hip._ptr(start), _hip._ptr(ref),
                   _hip._stream())
        torch.cuda.synchronize()
        sat = torch.cuda.Stream(device=dev)
        cons = torch.cuda.Stream(device=dev)
        for s in (sat, cons):
            s.wait_stream(torch.cuda.current_stream())
        outs = []
        with torch.cuda.stream(sat):
            _hip.noise_mlp(big, 30000, cbig, blob, bias, npred.precision_code)
        with torch.cuda.stream(cons):
            for _ in range(3):
                outs.append(_hip.fps(xyz, 512, start))
        torch.cuda.synchronize()
    for o in outs:
        assert torch.equal(o, ref)
