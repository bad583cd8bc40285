"""Multi-process (world_size 2, gloo, CPU) tests of the data-parallel path.

The exchange step of the reference's Lightning DDP (config.yaml:127) is one
mean all-reduce of the gradients after backward.  Here each rank computes the
oracle gradients of its half of a golden batch, packs them into one flat
buffer in parameter order (as optim.FusedAdamW lays them out), and
ddp.GradReducer averages it.  Per-sample independence of the model + the
mean-reduced loss make the average equal to the full-batch gradient the
reference produced (tests/golden/metaformer_small_r1.npz).
"""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from tests.golden_util import load, config, batch_from, prefixed, rel_err

TOL = 1e-4


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _init(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    from multimodalreactiongeneration_amd.ddp import init_from_env
    r, w = init_from_env(backend="gloo")
    assert (r, w) == (rank, world)


def _worker_grads(rank, world, port, out_dir):
    torch.set_num_threads(2)
    _init(rank, world, port)
    from oracle import mrg_oracle as O
    from multimodalreactiongeneration_amd.ddp import GradReducer
    d = load("metaformer_small_r1")
    cfg = config(d)
    sd = prefixed(d, "param/")
    batch = batch_from(d)
    B = batch[0][0].shape[0]
    per = B // world
    shard = [(x[rank * per:(rank + 1) * per].clone(), n[rank * per:(rank + 1) * per].clone())
             for x, n in batch]
    _, _, grads, _ = O.run_train_step(O.metaformer_training_loss, sd, cfg["optim"], cfg["model"], shard)
    keys = list(sd.keys())
    flat = torch.cat([grads[k].reshape(-1) for k in keys])
    GradReducer(flat, bucket_elems=flat.numel() // 3 + 1).allreduce()
    np.save(os.path.join(out_dir, f"flat{rank}.npy"), flat.numpy())
    dist.destroy_process_group()


def _worker_broadcast(rank, world, port, out_dir):
    _init(rank, world, port)
    from multimodalreactiongeneration_amd.ddp import broadcast_parameters
    torch.manual_seed(100 + rank)   # different init per rank
    m = torch.nn.Sequential(torch.nn.Linear(5, 7), torch.nn.LayerNorm(7))
    broadcast_parameters(m)
    np.save(os.path.join(out_dir, f"p{rank}.npy"),
            torch.cat([p.detach().reshape(-1) for p in m.parameters()]).numpy())
    dist.destroy_process_group()


def _spawn(fn, world=2):
    out = tempfile.mkdtemp(prefix="mrg_ddp_")
    mp.spawn(fn, args=(world, _free_port(), out), nprocs=world, join=True)
    return out


def test_grad_allreduce_equals_full_batch_gradient():
    d = load("metaformer_small_r1")
    if d["in/0/x"].shape[0] % 2:
        pytest.skip("golden batch not divisible by 2")
    out = _spawn(_worker_grads)
    f0, f1 = np.load(os.path.join(out, "flat0.npy")), np.load(os.path.join(out, "flat1.npy"))
    assert np.array_equal(f0, f1), "ranks disagree after all-reduce"
    sd = prefixed(d, "param/")
    off = 0
    worst = 0.0
    for k, v in sd.items():
        n = v.numel()
        ref = d["grad/" + k]
        got = torch.from_numpy(f0[off:off + n].reshape(ref.shape))
        off += n
        if np.abs(ref).max() > 1e-6:
            worst = max(worst, rel_err(got, ref))
    assert off == f0.size
    assert worst < TOL, worst


def test_broadcast_parameters_syncs_ranks():
    out = _spawn(_worker_broadcast)
    p0, p1 = np.load(os.path.join(out, "p0.npy")), np.load(os.path.join(out, "p1.npy"))
    assert np.array_equal(p0, p1)


def test_reducer_is_noop_single_process():
    from multimodalreactiongeneration_amd.ddp import GradReducer
    g = torch.arange(10, dtype=torch.float32)
    GradReducer(g).allreduce()
    assert torch.equal(g, torch.arange(10, dtype=torch.float32))
