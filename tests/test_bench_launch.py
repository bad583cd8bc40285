"""bench.py's multi-GPU launch logic on the CPU (no GPU): ``--gpus N`` means N ranks.

Reference: Lightning DDP over every listed GPU (mr_gen/model/lstmformer/config.yaml:121,127).
* without torch.distributed.run, ``--gpus 2 --dry-run 1`` launches two gloo ranks that rendezvous on
  127.0.0.1, run the barrier + max-over-ranks timing and print ONE JSON line with ranks_seen = 2;
* ``--gpus 2`` on a host with fewer visible GPUs exits 2 instead of timing one GPU;
* under torch.distributed.run, a WORLD_SIZE different from --gpus exits 2 before any rendezvous.
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(OMP_NUM_THREADS="2", MASTER_ADDR="127.0.0.1", **kw)
    return env


def _run(args, env, timeout=240):
    return subprocess.run([sys.executable, BENCH] + args, env=env, capture_output=True, text=True, timeout=timeout)


def test_dry_run_launches_two_gloo_ranks():
    r = _run(["--gpus", "2", "--dry-run", "1", "--steps", "2", "--warmup", "1"], _env())
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout            # rank 0 only
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["steps"] == 2 and out["warmup"] == 1
    assert out["ranks_seen"]["world_size"] == 2 and out["ranks_seen"]["backend"] == "gloo"
    assert sorted(r_["rank"] for r_ in out["ranks_seen"]["ranks"]) == [0, 1]
    assert out["allreduce_mean_ok"] is True
    assert out["ms_per_step"] > 0
    assert out["exchange"]["allreduce_ms"] > 0 and out["exchange"]["allreduce_bytes"] == 13_052_678 * 4


def test_dry_run_single_rank_needs_no_launcher():
    r = _run(["--dry-run", "1", "--steps", "1", "--warmup", "0"], _env())
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert out["n_gpus"] == 1 and out["ranks_seen"]["world_size"] == 1


def test_headline_is_the_last_line_and_small():
    """a 20.7 KB line holding the secondary block was not parsed by the driver.  The
    secondary configs print as their own lines first; the headline, with full-size synthetic kernels,
    roofline (traffic included), CPU baseline and secondary summary, is the LAST stdout line, parses,
    and fits HEADLINE_MAX_BYTES (8,000) with room to spare."""
    r = _run(["--dry-run", "1", "--steps", "1", "--warmup", "0"], _env())
    assert r.returncode == 0, r.stderr[-2000:]
    lines = r.stdout.rstrip("\n").split("\n")
    assert all(ln.startswith("{") for ln in lines), r.stdout[:500]
    *sec, last = lines
    assert len(last.encode()) <= 6000, len(last)
    out = json.loads(last)
    assert "secondary" not in out or all(isinstance(v, dict) and "ms_per_step" in v for v in out["secondary"].values())
    assert out["roofline"]["family"] == "gemm" and "traffic" in out["roofline"]
    assert out["roofline"]["frac"] > 0 and out["cpu_baseline"]["cores"] == 16
    assert len(sec) == 6 and len(out["secondary"]) == 6
    for ln in sec:
        s = json.loads(ln)
        assert s["secondary"] in out["secondary"] and "cpu_baseline" in s and "whole_step_roofline" in s


def test_more_gpus_than_visible_fails_loudly():
    env = _env(HIP_VISIBLE_DEVICES="", CUDA_VISIBLE_DEVICES="")
    r = _run(["--gpus", "2", "--steps", "1"], env, timeout=120)
    assert r.returncode == 2
    assert "visible" in r.stderr and "n_gpus" not in r.stdout


def test_world_size_mismatch_fails_before_rendezvous():
    env = _env(WORLD_SIZE="3", RANK="0", LOCAL_RANK="0", MASTER_PORT="1")
    r = _run(["--gpus", "2", "--steps", "1"], env, timeout=120)
    assert r.returncode == 2
    assert "WORLD_SIZE=3" in r.stderr
