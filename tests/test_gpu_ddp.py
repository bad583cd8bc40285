"""The data-parallel path with the real kernels: 2 ranks sharing the one GPU of the box (gloo carries
the gradient exchange; RCCL refuses two ranks on one device), each training on half of the golden
batch.  GradReducer(overlap=True) issues bucketed all-reduces DURING backward from the library's
gradient-ready points (ddp.py); after a census step, the averaged gradients must equal the
reference's full-batch gradients (tests/golden/metaformer_small_r1.npz) and agree across ranks."""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from tests.golden_util import load, config, batch_from, prefixed, rel_err

pytestmark = pytest.mark.gpu
TOL = 1e-4


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    torch.cuda.set_device(0)
    from multimodalreactiongeneration_amd.ddp import init_from_env, GradReducer
    from multimodalreactiongeneration_amd.model import Metaformer
    from multimodalreactiongeneration_amd import functional as Fn
    init_from_env(backend="gloo")
    d = load("metaformer_small_r1")
    cfg = config(d)
    m = Metaformer(cfg["model"], cfg["optim"], cfg["metrics"])
    m.load_state_dict(prefixed(d, "param/"))
    m = m.to("cuda:0")
    opt = m.configure_optimizers()["optimizer"]
    red = GradReducer(opt.flat_grad, params=opt.plist, overlap=True, bucket_bytes=64 << 10)
    batch = batch_from(d)
    per = batch[0][0].shape[0] // world
    shard = [(x[rank * per:(rank + 1) * per].to("cuda:0"), n[rank * per:(rank + 1) * per]) for x, n in batch]
    for step in range(2):   # census, then overlapped
        opt.zero_grad()
        m.training_step([(x.clone(), n) for x, n in shard])["loss"].backward()
        red.finish()
    torch.cuda.synchronize()
    Fn.check_errors()
    assert len(red.order) == len(red.buckets) > 2
    np.save(os.path.join(out_dir, f"g{rank}.npy"), opt.flat_grad.cpu().numpy())
    red.close()
    dist.destroy_process_group()


def test_two_ranks_overlapped_allreduce_equals_full_batch_gradient():
    d = load("metaformer_small_r1")
    out = tempfile.mkdtemp(prefix="mrg_gpu_ddp_")
    mp.spawn(_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    g0, g1 = np.load(os.path.join(out, "g0.npy")), np.load(os.path.join(out, "g1.npy"))
    assert np.array_equal(g0, g1), "ranks disagree after the all-reduce"
    off, worst = 0, 0.0
    for k, v in prefixed(d, "param/").items():
        n = v.numel()
        ref = d["grad/" + k]
        if np.abs(ref).max() > 1e-6:
            worst = max(worst, rel_err(torch.from_numpy(g0[off:off + n].reshape(ref.shape)), ref))
        off += n
    assert off == g0.size
    assert worst < TOL, worst


def test_bench_multi_rank_timed_branch_on_one_gpu():
    """bench.py's N>1 timed branch (graph-replayed fwd+bwd, then the serial bucketed GradReducer
    all-reduce, then the fused AdamW, max-over-ranks timing) with the real kernels: 2 ranks on the box's
    one GPU (--shared-device-gloo: gloo carries the exchange, the ranks' replays take turns), the
    pre-flight of the driver's 8-GPU SCALE run.  Asserts (a) one JSON line with a world of 2, (b) the
    ranks' parameters bitwise equal after the timed steps, (c) one step's rank-averaged gradient equal
    to a single-rank step on the concatenated 2 x B batch (1e-4 on every parameter).
    Reference: config.yaml:121,127 (Lightning DDP)."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(OMP_NUM_THREADS="4", MASTER_ADDR="127.0.0.1")
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--shared-device-gloo", "1",
                        "--ddp-check", "1", "--batch", "8", "--seq", "120", "--steps", "3", "--warmup", "1",
                        "--secondary", "0", "--cpu-baseline", "0"],
                       env=env, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    print(json.dumps({k: out.get(k) for k in ("ms_per_step", "ranks_seen", "ddp_check",
                                               "params_bitwise_equal_across_ranks")}))
    assert out["n_gpus"] == 2 and out["ranks_seen"]["world_size"] == 2
    assert out["ranks_seen"]["backend"] == "gloo" and out["shared_device_test"] is True
    assert out["params_bitwise_equal_across_ranks"] is True
    ex = out["exchange"]          # replay and exchange timed apart at N > 1
    assert ex["replay_ms"] > 0 and ex["allreduce_ms"] > 0 and ex["allreduce_bytes"] == 13_052_678 * 4, ex
    chk = out["ddp_check"]
    assert chk["concat_batch"] == 16
    assert chk["grad_vs_concat_batch_worst_rel"] < TOL, chk     # every parameter, ReLU layers included


def test_native_rccl_communicator_one_rank():
    """libmrg's own RCCL communicator (mrg_comm_* C-ABI) on the box's one GPU: a 1-rank group's mean
    and sum of bucketed spans leave the buffer bit-identical, spans outside the list untouched."""
    from multimodalreactiongeneration_amd.ddp import NativeComm
    torch.cuda.set_device(0)
    comm = NativeComm(rank=0, world=1)
    try:
        x = torch.randn(1 << 20, device="cuda:0")
        ref = x.clone()
        comm.allreduce(x, [(0, 1000), (4096, 300000), (600000, 1 << 20)], "mean")
        comm.allreduce(x, None, "sum")
        torch.cuda.synchronize()
        assert torch.equal(x, ref)
    finally:
        comm.close()
