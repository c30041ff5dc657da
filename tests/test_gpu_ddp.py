"""SURVEY §8e's multi-GPU parity on one device: the DDP gradient of DiffusionTrainer equals the
gradient-accumulation gradient of the single-process trainer over the same samples and draws
(the reference's accumulation step, /root/reference/training/trainer.py:115-125).

Backend choice: both ranks run on cuda:0 with the gloo process group (the box has one GPU and
RCCL wants one device per rank); DDP's bucketed all-reduce then goes through gloo's CUDA path.
The trainer code under test is the one RCCL runs on the 8-GPU node -- only the transport
differs.  Each process is a child started with subprocess (tests/ddp_worker.py).
"""
import os
import socket
import subprocess
import sys

import re

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
WORKER = os.path.join(HERE, "ddp_worker.py")
PRE_BN_BIAS = re.compile(r"style_encoder\.encoder\.sa\d\.mlp_convs\.\d+\.bias$")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(tmp, tag, world, accum, micro, clouds=2, points=8192, amp=False, global_points=2048,
         backend="gloo", extra_env=None):
    out = os.path.join(tmp, f"{tag}.npz")
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), **(extra_env or {}))
        if world > 1:
            env.update(RANK=str(r), LOCAL_RANK="0", WORLD_SIZE=str(world))
        else:
            for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE"):
                env.pop(k, None)
        procs.append(subprocess.Popen(
            [sys.executable, WORKER, out, str(accum), str(micro), str(clouds), str(points),
             amp if isinstance(amp, str) else ("1" if amp else "0"), str(global_points), backend],
            env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
    return procs, out


def _wait(procs, timeout=100):
    logs = []
    for p in procs:
        o, _ = p.communicate(timeout=timeout)
        logs.append(o.decode(errors="replace"))
    for p, lg in zip(procs, logs):
        assert p.returncode == 0, lg[-3000:]
    return logs


def _grads(z):
    return {k[5:]: z[k] for k in z.files if k.startswith("grad:")}


@pytest.mark.parametrize("accum", [1, 2])
def test_ddp_gradient_equals_accumulation(tmp_path, accum):
    """world 2 x `accum` micro-batches (no_sync on the non-final ones) against one process
    accumulating 2 * accum micro-batches.  accum=1: each rank's gradient is the single
    process's micro-step gradient times 1/2 (exact), and one fp32 addition combines them in
    both set-ups -> bit-identical.  accum=2: the summation order differs ((a+b)+c)+d vs
    (a+b)+(c+d), so equal to fp32 rounding of the sum."""
    tmp = str(tmp_path)
    ddp, out_ddp = _run(tmp, "ddp", 2, accum, accum)
    one, out_one = _run(tmp, "one", 1, 2 * accum, 2 * accum)
    _wait(ddp + one)
    zd, zo = np.load(out_ddp), np.load(out_one)
    gd, go = _grads(zd), _grads(zo)
    assert gd.keys() == go.keys() and len(gd) == 80
    bad = []
    for n in gd:
        a, b = gd[n].astype(np.float64), go[n].astype(np.float64)
        scale = np.abs(b).max()
        err = np.abs(a - b).max()
        tol = 0.0 if accum == 1 else 4e-7 * scale + 1e-30
        if err > tol:
            bad.append(f"{n}: max|ddp - accum| {err:.3e} (max|g| {scale:.3e})")
    assert not bad, "\n".join(bad[:20])
    # the parameters after the (replicated) clip + AdamW step agree as well
    for k in zd.files:
        if k.startswith("param:"):
            np.testing.assert_allclose(zd[k], zo[k], rtol=0, atol=1e-6 if accum > 1 else 0)


def test_ddp_configs3_per_rank_size_amp(tmp_path):
    """BASELINE configs[3] at its per-rank size: 8 x 120000-point clouds per rank, use_amp with
    Config.amp_dtype "bfloat16" (the bf16 fused NoisePredictor, bf16 GEMMs; GradScaler disabled
    so the gradients compare unscaled -- bf16's fp32 exponent range keeps the halving below
    exact; the float16 case is test_ddp_fp16_amp_matches_accumulation), the real 2,549,827-gradient (10.2 MB) bucketed all-reduce through DDP's reducer.
    World 2 x 1 micro-batch against one process accumulating the same 2 micro-batches
    (trainer.py:115-125; counter-keyed draws, dropout off).  Each rank's gradient is its
    micro-batch gradient (loss / 1), DDP averages the two; the single process adds the two
    micro-batch gradients of loss / 2: (a + b) / 2 vs a / 2 + b / 2, equal in fp32 (halving is
    exact), so the bound is the accum-2 summation-order bound 4e-7 max|g| and the measured
    difference is expected to be 0.  Every rank's post-step parameters must be identical."""
    tmp = str(tmp_path)
    kw = dict(clouds=8, points=120000, amp=True, global_points=30000)
    ddp, out_ddp = _run(tmp, "ddp", 2, 1, 1, **kw)
    _wait(ddp, timeout=400)
    one, out_one = _run(tmp, "one", 1, 2, 2, **kw)
    _wait(one, timeout=400)
    zd, zo = np.load(out_ddp), np.load(out_one)
    z1 = np.load(out_ddp[:-4] + ".rank1.npz")
    gd, go = _grads(zd), _grads(zo)
    assert gd.keys() == go.keys() and len(gd) == 80
    assert sum(v.size for v in gd.values()) == 2549827
    bad, exact = [], 0
    for n in gd:
        a, b = gd[n].astype(np.float64), go[n].astype(np.float64)
        assert np.isfinite(a).all() and np.abs(b).max() > 0, n
        scale = np.abs(b).max()
        err = np.abs(a - b).max()
        exact += int(err == 0)
        if err > 4e-7 * scale + 1e-30:
            bad.append(f"{n}: max|ddp - accum| {err:.3e} (max|g| {scale:.3e})")
    print(f"configs[3] per-rank size: {exact}/80 gradients bit-identical")
    assert not bad, "\n".join(bad[:20])
    for k in zd.files:
        if k.startswith("param:"):
            np.testing.assert_array_equal(zd[k], z1[k])          # ranks identical
            np.testing.assert_allclose(zd[k], zo[k], rtol=0, atol=1e-6)


def test_ddp_fp16_amp_matches_accumulation(tmp_path):
    """The reference's float16 autocast (Config.amp_dtype default, trainer.py:50,78) under DDP,
    with the GradScaler on at a fixed scale 2^14 (unscale_ is exact; the default init 2^16
    overflows fp16 in this first step -- the scaler would skip it and halve the scale): world
    2 x 1 micro-batch against one process accumulating the same 2.  The 16-bit activation
    gradients of loss/2 are exact halves of those of loss/1 except where they fall into fp16's
    subnormal range (the style branch's, deep behind style_proj, do: round-3 measurement 0/80
    bit-identical, all within 1e-3), so the bound is 1e-3 max|g|.
    Pre-BN conv biases are skipped: their gradient is analytically zero (train-mode BN
    removes any shift) and both sides hold rounding noise.  Ranks' post-step parameters
    identical; no inf/nan (the scaler would have skipped the step)."""
    tmp = str(tmp_path)
    ddp, out_ddp = _run(tmp, "ddp", 2, 1, 1, amp="fp16")
    one, out_one = _run(tmp, "one", 1, 2, 2, amp="fp16")
    _wait(ddp + one)
    zd, zo = np.load(out_ddp), np.load(out_one)
    z1 = np.load(out_ddp[:-4] + ".rank1.npz")
    gd, go = _grads(zd), _grads(zo)
    assert gd.keys() == go.keys() and len(gd) == 80
    bad, exact, worst = [], 0, 0.0
    for n in gd:
        a, b = gd[n].astype(np.float64), go[n].astype(np.float64)
        assert np.isfinite(a).all() and np.isfinite(b).all(), n
        if PRE_BN_BIAS.search(n):
            continue
        scale = np.abs(b).max()
        err = np.abs(a - b).max()
        exact += int(err == 0)
        worst = max(worst, err / scale)
        if err > 1e-3 * scale + 1e-30:
            bad.append(f"{n}: max|ddp - accum| {err:.3e} (max|g| {scale:.3e})")
    print(f"fp16 amp DDP: {exact}/71 gradients bit-identical, worst max|ddp - accum|/max|g| "
          f"{worst:.3e}")
    assert not bad, "\n".join(bad[:20])
    for k in zd.files:
        if k.startswith("param:"):
            np.testing.assert_array_equal(zd[k], z1[k])


def test_rccl_one_rank_ddp_step_matches_plain_step(tmp_path):
    """The RCCL transport itself (the 8-GPU node's all-reduce; one GPU here): a fresh child
    process with a one-rank "nccl" process group runs DiffusionTrainer(ddp=True) for one
    optimizer step (2 micro-batches, no_sync on the first), so DDP's reducer all-reduces the
    2,549,827 gradients through RCCL.  A sum over one rank is the identity, so the gradients
    and the parameters after the step equal the plain single-process step's bit for bit
    (/root/reference/training/trainer.py:115-125).  RCCL's collective log (NCCL_DEBUG=INFO,
    subsystem COLL) must show the reducer's AllReduce calls."""
    tmp = str(tmp_path)
    rc, out_rc = _run(tmp, "rccl", 1, 2, 2, backend="nccl",
                      extra_env={"NCCL_DEBUG": "INFO", "NCCL_DEBUG_SUBSYS": "COLL"})
    log = _wait(rc, timeout=200)[0]
    one, out_one = _run(tmp, "plain", 1, 2, 2)
    _wait(one)
    zr, zo = np.load(out_rc), np.load(out_one)
    n_ar = sum("AllReduce" in ln for ln in log.splitlines())
    print(f"RCCL AllReduce log lines: {n_ar}")
    assert n_ar >= 1, log[-3000:]
    gr, go = _grads(zr), _grads(zo)
    assert gr.keys() == go.keys() and len(gr) == 80
    assert np.array_equal(zr["losses"], zo["losses"])
    for n in gr:
        assert np.array_equal(gr[n], go[n]), n
    for k in zr.files:
        if k.startswith("param:"):
            assert np.array_equal(zr[k], zo[k]), k
