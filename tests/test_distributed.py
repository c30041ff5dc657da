"""The N>1 host path on CPU: world_size-2 gloo process group, one process per rank, exactly
as torchrun launches bench.py / the trainer on the GPU node (RCCL there)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    from pointcloud_style_transfer_amd import distributed as D

    try:
        w, r, _ = D.init_from_env("gloo")
        assert (w, r) == (world, rank) and D.is_distributed()
        n = 7
        mine = D.shard(n, r, w)
        # each rank "denoises" its own clouds: no collective on the data path
        outs = [torch.full((4, 3), float(i)) for i in mine]
        t = D.max_over_ranks(0.5 + rank)
        s = D.sum_over_ranks(len(mine))
        g = D.gather_clouds(outs, n)
        res = {"rank": r, "mine": list(mine), "max": t, "sum": s,
               "gathered": None if g is None else [float(c[0, 0]) for c in g]}
        # DDP gradient averaging with the trainer's settings (rank-local BN, fp32 buckets)
        torch.manual_seed(0)
        m = torch.nn.Sequential(torch.nn.Linear(3, 8), torch.nn.BatchNorm1d(8), torch.nn.Linear(8, 1))
        ddp = torch.nn.parallel.DistributedDataParallel(m, broadcast_buffers=False, bucket_cap_mb=16)
        x = torch.arange(12, dtype=torch.float32).view(4, 3) * (rank + 1)
        ddp(x).sum().backward()
        res["grad"] = m[0].weight.grad.tolist()  # plain data through the queue
        q.put(res)
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def test_world2_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=120) for _ in ps], key=lambda d: d["rank"])
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0]["mine"] == [0, 1, 2, 3] and res[1]["mine"] == [4, 5, 6]
    assert res[0]["max"] == res[1]["max"] == 1.5
    assert res[0]["sum"] == 7
    assert res[0]["gathered"] == [float(i) for i in range(7)] and res[1]["gathered"] is None
    assert res[0]["grad"] == res[1]["grad"]  # all-reduced, identical


@pytest.mark.parametrize("n,world", [(0, 3), (5, 8), (256, 8), (13, 4)])
def test_shard_partition(n, world):
    from pointcloud_style_transfer_amd.distributed import shard

    parts = [shard(n, r, world) for r in range(world)]
    flat = [i for p in parts for i in p]
    assert flat == list(range(n))
    assert max(map(len, parts)) - min(map(len, parts)) <= 1


def _train_worker(rank, world, port, tmp, q):
    """DiffusionTrainer.train() under a world-2 gloo group on the CPU with the per-batch work
    stubbed out (the HIP kernels need the GPU): the validation losses differ per rank so a
    rank-local best/patience decision would stop the ranks at different epochs."""
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    from pointcloud_style_transfer_amd import distributed as D
    from pointcloud_style_transfer_amd.config.config import Config
    from pointcloud_style_transfer_amd.training import trainer as T

    try:
        os.chdir(tmp)  # CheckpointManager logs under ./logs, as the reference's does
        D.init_from_env("gloo")
        torch.manual_seed(0)
        cfg = Config(make_dirs=False, log_dir=tmp, checkpoint_dir=os.path.join(tmp, f"ck{rank}"),
                     num_epochs=12, val_interval=1, save_interval=1000)
        tr = T.DiffusionTrainer(cfg, device="cpu")
        tr.max_patience = 2
        # alone, rank 0 would stop at epoch 10 (best at 8) and rank 1 at epoch 2 (best at 0);
        # the rank average is best at epoch 5 (1.23) and stops at epoch 7
        curves = {0: [5, 4, 3, 2, 1, 0.5, 0.6, 0.4, 0.3, 0.7, 0.8, 0.9],
                  1: [1, 1.5, 1.8, 1.9, 1.95, 1.96, 4, 4, 4, 4, 4, 4]}
        val_calls = []

        def val_loss(self, batch):
            e = self.current_epoch
            val_calls.append(e)
            return float(curves[rank][e])

        epochs = []
        T.DiffusionTrainer._val_loss = val_loss
        T.DiffusionTrainer.train_one_epoch = lambda self, dl: epochs.append(self.current_epoch) or 0.0

        class Sampler:
            seen = []

            def set_epoch(self, e):
                self.seen.append(e)

        class Loader(list):
            sampler = Sampler()

        tr.train(Loader([None]), [None])
        # EMA shadows were built after the DDP wrap: identical on both ranks
        shadow = [s.sum().item() for s in tr.ema.shadow_params[:4]]
        q.put({"rank": rank, "epochs": epochs, "best": tr.best_val_loss,
               "set_epoch": Loader.sampler.seen, "shadow": shadow,
               "seed": torch.initial_seed()})
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def test_world2_trainer_shared_early_stop(tmp_path):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_train_worker, args=(r, 2, port, str(tmp_path), q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=180) for _ in ps], key=lambda d: d["rank"])
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0]["epochs"] == res[1]["epochs"] == list(range(8))
    assert res[0]["best"] == res[1]["best"] == (0.5 + 1.96) / 2
    assert res[0]["set_epoch"] == res[1]["set_epoch"] == list(range(8))
    assert res[0]["shadow"] == res[1]["shadow"]
    assert res[0]["seed"] != res[1]["seed"]  # per-rank draws
