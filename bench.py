"""Benchmark: lstmformer training frames/s (BASELINE.json metric), fp32, synthetic data.

    python bench.py [--gpus N --steps K --warmup W]          (N > 1 under torch.distributed.run)

A step = Metaformer.training_step (fwd + masked Huber loss) + backward +
RCCL gradient all-reduce (N > 1) + fused AdamW, on B=64 x T=300 frames per
GPU (weak scaling).  Inputs are resident in HBM before timing.  Prints ONE
JSON line on rank 0 with the live roofline of the dominant kernel (HIP events
around its launches inside the timed region) and the CPU oracle baseline
timed on this host (rank 0, N=1 only).

At N=1 the same line carries a ``secondary`` block with the other 1-GPU
BASELINE configs, each graph-replayed with its own ms/step,
frames/s, whole-step roofline, dominant-kernel roofline and a CPU baseline on a
bounded sample: C2 simple_lstm (fp32 and bf16), C3 lstm_with_sampling scheduled
sampling, and lstmformer autoregressive generation (§8f rank 1).
"""
import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "training frames/sec/GPU, lstmformer T=300 B=64; 1→8 GPU scaling"
FP32_MFMA_PEAK_TF = 157.3   # MI355X_MICROARCH.md chip table (f32 matrix, dense)
BF16_MFMA_PEAK_TF = 2500.0  # MI355X_MICROARCH.md chip table (bf16 matrix, dense)
HBM_PEAK_GBS = 8000.0
PMC_SUMMARY = os.path.join(ROOT, "profiles", "r06_pmc_summary.json")

# probe name (functional._probe) -> kernels it brackets (descriptions and FLOP counts: DESIGN.md §4)
FAMILIES = {
    "gemm": "gemm_x6w+gemm_x6g+gemm_x6g_wgrad+splitk_reduce4",   # every GEMM of the step, 2MNK FLOP per launch
    "lstm_fwd": "lstm_fwd_kernel+lstm_fwd_mx_kernel",            # 8H^2 FLOP per (b, t) per layer direction
    "lstm_bwd": "lstm_bwd_kernel+lstm_bwd_mx_kernel",            # 8H^2 FLOP per (b, t) per layer direction
    "attn_fwd": "attn_fwd_kernel",                               # 4D FLOP per visible (q, k) pair per head
    "attn_bwd": "attn_bwd_fused_kernel",                         # 10D FLOP per visible pair per head
    "gru_fwd": "gru_fwd_kernel",                                 # 6H^2 FLOP per (b, t) per layer
    "gru_bwd": "gru_bwd_kernel",                                 # 6H^2 FLOP per (b, t) per layer
    "gen": "gen_loop_kernel (or gen_lstm+gen_linear+gen_ffn)",   # generation frame loop, 2MNK FLOP per launch
    "ssd": "ssd_loop_kernel+ssd_loop_bwd_kernel",                # C3 frame loops, their products' 2MNK FLOP
}
PEAK_NOTES = {
    "gemm": "f32 dense matrix peak; x6 bf16 split's own MFMA ceiling 416.7",
    "lstm_fwd": "latency-bound recurrence; f32 VALU peak",
    "lstm_bwd": "latency-bound recurrence; f32 VALU peak",
    "gru_fwd": "latency-bound recurrence; f32 VALU peak",
    "gru_bwd": "latency-bound recurrence; f32 VALU peak",
    "gen": "hand-off-latency-bound 8-row products (26 hand-off stages per frame, one launch); f32 matrix peak",
    "ssd": "hand-off-latency-bound 8-row products (2 forward / 3 backward hand-offs per frame); f32 matrix peak",
}
HEADLINE_MAX_BYTES = 8000   # the driver parses the LAST stdout line; keep it well inside its window
# rocprofv3 kernel-name prefix of each family in the PMC summary (tools/tools_pmc_summary.py)
PMC_KEYS = {"gemm": "gemm_all", "lstm_fwd": "lstm_fwd", "lstm_bwd": "lstm_bwd",
            "attn_fwd": "attn_fwd_kernel", "attn_bwd": "attn_bwd"}


TRACE_SUMMARY = os.path.join(ROOT, "profiles", "r06_trace_roofline.json")


def trace_check(roof):
    """The dominant family's figure recomputed from the committed rocprofv3 kernel trace of the
    graph-replayed step (tools/tools_trace_roofline.py): kernel time per step summed over every
    kernel of the family (split-K reduce included) from the trace, FLOPs per step from this run's
    probe.  None when the committed summary is missing."""
    try:
        with open(TRACE_SUMMARY) as f:
            doc = json.load(f)
        fam = doc["families"][roof["family"]]
    except (OSError, KeyError, ValueError):
        return None
    flop = roof["algorithmic_flop_per_launch"] * roof["launches_per_step"]
    out = {"source": os.path.relpath(TRACE_SUMMARY, ROOT)}
    for part in ("probe", "replay"):
        ms = fam.get(part + "_ms_per_step")
        if ms:
            tf = flop / (ms / 1e3) / 1e12
            out[part] = {"ms_per_step": ms, "achieved": round(tf, 2), "frac": round(tf / roof["peak"], 4)}
    if "probe" in out:   # the live probe vs the same launches in the committed trace
        out["live_vs_trace_probe"] = round(roof["achieved"] / out["probe"]["achieved"], 3)
    return out


def pmc_traffic(family):
    """HBM bytes per launch of a family from the committed rocprofv3 FETCH_SIZE/WRITE_SIZE passes."""
    try:
        with open(PMC_SUMMARY) as f:
            doc = json.load(f)
        fam = doc["families"].get(PMC_KEYS[family])
        return None if fam is None else round(fam["hbm_bytes_per_launch"])
    except (OSError, KeyError, ValueError):
        return None


_T0 = time.perf_counter()


def progress(msg):
    """One progress line on stderr (stdout carries only the JSON result line)."""
    print(f"[bench {time.perf_counter() - _T0:7.1f}s] {msg}", file=sys.stderr, flush=True)


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs (= ranks) of this node; without torch.distributed.run's env, N > 1 makes this "
                         "process the launcher of N ranks; under it, N must equal WORLD_SIZE (default: WORLD_SIZE or 1)")
    ap.add_argument("--dry-run", type=int, default=0,
                    help="1 = exercise the launch / rendezvous / barrier / max-over-ranks timing / JSON on the CPU "
                         "(gloo, a flat-buffer all-reduce as the step), no GPU")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--seq", type=int, default=300)
    ap.add_argument("--ratio", type=int, default=1, help="audio frames per prediction frame (8 = reference rate)")
    ap.add_argument("--graph", type=int, default=1, help="replay the step as a HIP graph")
    ap.add_argument("--cpu-baseline", type=int, default=1)
    ap.add_argument("--cpu-steps", type=int, default=5, help="timed CPU steps of the headline baseline")
    ap.add_argument("--cpu-warmup", type=int, default=2)
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = every physical core this process may use")
    ap.add_argument("--secondary", type=int, default=1, help="time the other 1-GPU BASELINE configs (N=1 only)")
    ap.add_argument("--wgrad-stream", type=int, default=1,
                    help="weight-gradient GEMMs on a side stream (functional._side); 0 = one stream")
    ap.add_argument("--wgrad-defer", type=int, default=1,
                    help="queue side-stream weight gradients to run beside the next backward recurrence "
                         "(r03: 23.67 -> 23.33 ms/step with the encoder wavefront; 0 = issue when ready)")
    ap.add_argument("--comm", default="torch", choices=["torch", "native"],
                    help="N>1 gradient all-reduce: torch.distributed (RCCL) or libmrg's mrg_comm_* RCCL communicator")
    ap.add_argument("--lstm-group", type=int, default=0, help="workgroups per LSTM row group at H=256 (8|16; 0 = library default)")
    ap.add_argument("--shared-device-gloo", type=int, default=0,
                    help="TEST ONLY: run the N>1 branch with every rank on GPU 0 and gloo carrying the exchange "
                         "(RCCL refuses two ranks on one device), so the multi-GPU timed path runs with real kernels "
                         "on a 1-GPU box; the ranks' fwd+bwd replays take turns on the device (host lock)")
    ap.add_argument("--ddp-check", type=int, default=0,
                    help="N>1: before timing, check that one step's rank-averaged gradient equals a single-rank step "
                         "on the concatenation of every rank's shard (reported as ddp_check)")
    args = ap.parse_args(argv)
    if args.shared_device_gloo and args.comm != "torch":
        ap.error("--shared-device-gloo runs the exchange on torch.distributed gloo; --comm native needs RCCL")
    return args


def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_or_check(args, argv=None):
    """Make ``--gpus N`` mean N ranks (the reference trains with Lightning DDP on every listed GPU,
    mr_gen/model/lstmformer/config.yaml:121,127).

    * Under torch.distributed.run (WORLD_SIZE set): N must equal WORLD_SIZE, else exit 2.
    * Without it and N > 1: this process becomes the launcher.  It makes no HIP call (the device count
      comes from torch.cuda.device_count(), which does not initialise the runtime on this image), exits 2
      when fewer than N GPUs are visible, and otherwise starts ``torch.distributed.run --nproc-per-node N``
      on this same script as a CHILD process (never exec) and exits with its return code.
    Returns None when this process should run the benchmark itself."""
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is not None:
        if args.gpus is None:
            args.gpus = int(env_world)
        if int(env_world) != args.gpus:
            print(f"bench.py: --gpus {args.gpus} but torch.distributed.run started WORLD_SIZE={env_world} ranks; "
                  "pass the same N to both", file=sys.stderr, flush=True)
            sys.exit(2)
        return None
    if args.gpus is None:
        args.gpus = 1
    if args.gpus <= 1:
        return None
    if not args.dry_run:
        visible = torch.cuda.device_count()
        if visible < (1 if args.shared_device_gloo else args.gpus):
            print(f"bench.py: --gpus {args.gpus} asks for {args.gpus} ranks (one per GPU) but only {visible} "
                  "GPU(s) are visible; refusing to time fewer GPUs than asked", file=sys.stderr, flush=True)
            sys.exit(2)
    import subprocess
    argv = sys.argv[1:] if argv is None else argv
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + list(argv)
    progress(f"launching {args.gpus} ranks: {' '.join(cmd[1:6])} ...")
    env = dict(os.environ)
    env.setdefault("OMP_NUM_THREADS", "4")
    rc = subprocess.call(cmd, env=env)
    if rc != 0:
        print(f"bench.py: torch.distributed.run exited {rc}", file=sys.stderr, flush=True)
    sys.exit(rc)


def ranks_seen(rank, world, dev, shared=False):
    """Every rank's (rank, local rank, device) as RCCL / gloo initialised them, gathered to all ranks;
    raises when two ranks share one GPU (the timing would then not be of N GPUs), unless ``shared``
    (--shared-device-gloo, a test of the N>1 code path, never a measurement)."""
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if dev is not None and dev.type == "cuda":
        p = torch.cuda.get_device_properties(dev)
        ident = str(getattr(p, "uuid", "")) or f"{p.name}:{dev.index}"
    else:
        ident = f"cpu:{local}"
    mine = {"rank": rank, "local_rank": local, "device": ident, "host": os.uname().nodename}
    if world <= 1:
        return {"world_size": 1, "backend": None, "ranks": [mine]}
    allr = [None] * world
    dist.all_gather_object(allr, mine)
    devs = {(r["host"], r["device"]) for r in allr}
    if dev is not None and dev.type == "cuda" and len(devs) != world and not shared:
        raise RuntimeError(f"bench.py: {world} ranks but only {len(devs)} distinct GPUs: {allr}")
    return {"world_size": dist.get_world_size(), "backend": dist.get_backend(), "distinct_devices": len(devs),
            "shared_device_test": bool(shared), "ranks": allr}


class _DeviceTurns:
    """--shared-device-gloo: the ranks' fwd+bwd work takes turns on the one GPU (an flock on a file
    keyed by the rendezvous port).  Two processes' persistent recurrences are not guaranteed
    co-resident on one device (each ring needs its members resident together), so the test mode
    serialises them; collectives stay outside the lock (a rank holding it across an all-reduce
    would wait for a rank that waits for the lock)."""

    def __init__(self, on):
        self.on = on
        self.f = None
        if on:
            import tempfile
            path = os.path.join(tempfile.gettempdir(), f"mrg_bench_dev0_{os.environ.get('MASTER_PORT', '0')}.lock")
            self.f = open(path, "a+")

    def __enter__(self):
        if self.on:
            import fcntl
            fcntl.flock(self.f, fcntl.LOCK_EX)
        return self

    def __exit__(self, *exc):
        if self.on:
            import fcntl
            torch.cuda.synchronize()
            fcntl.flock(self.f, fcntl.LOCK_UN)
        return False


def ddp_grad_check(model, opt, reducer, batch, args, rank, world, dev, turns):
    """One step's rank-averaged gradient (every rank on its own shard, then the exchange bench.py times)
    vs a single-rank step on the concatenation of all ranks' shards (what Lightning DDP's mean
    reproduces, config.yaml:127): the worst per-parameter max|a - b| / max|b| on rank 0."""
    from multimodalreactiongeneration_amd.synthetic import make_batch, clone_batch
    with turns:
        opt.zero_grad()
        model.training_step(clone_batch(batch, dev))["loss"].backward()
    reducer.allreduce()
    torch.cuda.synchronize()
    g_avg = opt.flat_grad.clone()
    res = None
    if rank == 0:
        shards = [make_batch(B=args.batch, T=args.seq, ratio=args.ratio, seed=1234 + r, device=dev)
                  for r in range(world)]
        full = [(torch.cat([s[i][0] for s in shards]), torch.cat([s[i][1] for s in shards])) for i in range(7)]
        with turns:
            opt.zero_grad()
            model.training_step(full)["loss"].backward()
        torch.cuda.synchronize()
        base = opt.flat_grad.data_ptr()
        worst = (0.0, None)
        names = {id(p): k for k, p in model.named_parameters()}
        for p in opt.plist:
            off = (p.grad.data_ptr() - base) // 4
            a, b = g_avg[off:off + p.numel()], opt.flat_grad[off:off + p.numel()]
            e = ((a - b).abs().max() / b.abs().max().clamp_min(1e-12)).item()
            if e > worst[0]:
                worst = (e, names.get(id(p), "?"))
        res = {"grad_vs_concat_batch_worst_rel": worst[0], "worst_param": worst[1],
               "concat_batch": args.batch * world}
    opt.zero_grad()
    dist.barrier()
    return res


def params_agree(opt):
    """Bitwise equality of every rank's flat parameter buffer (elementwise MAX == MIN over ranks)."""
    hi, lo = opt.flat.clone(), opt.flat.clone()
    dist.all_reduce(hi, op=dist.ReduceOp.MAX)
    dist.all_reduce(lo, op=dist.ReduceOp.MIN)
    return bool(torch.equal(hi, lo))


def timed_region(run, steps, world, dev):
    """K steps bracketed by barrier + synchronize on both sides; the MAX elapsed over ranks (seconds)."""
    cuda = dev is not None and dev.type == "cuda"
    if world > 1:
        dist.barrier()
    if cuda:
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        run()
    if cuda:
        torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev if cuda else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    return elapsed


def dry_run(args):
    """--dry-run: the launch, rendezvous, barrier / max-over-ranks timing and the JSON lines of the real
    benchmark on the CPU (gloo), with one all-reduce of a flat buffer the size of the benchmark model's
    gradients (13,052,678 fp32) as the "step".  At N = 1 rank 0 also prints full-size synthetic
    secondary lines and a headline carrying synthetic kernels / roofline / CPU baseline of the real
    line's shape, through the same formatting functions (headline_dict, secondary_summary,
    headline_json), so tests/test_bench_launch.py pins the headline's size and its position as the
    last stdout line without a GPU.  Every number in a dry-run line is synthetic (``dry_run: true``)."""
    from multimodalreactiongeneration_amd.ddp import init_from_env
    from multimodalreactiongeneration_amd import configs as C
    rank, world = init_from_env(backend="gloo")
    seen = ranks_seen(rank, world, None)
    buf = torch.full((13_052_678,), float(rank + 1))

    def run():
        if world > 1:
            t0 = time.perf_counter()
            dist.all_reduce(buf)
            buf.mul_(1.0 / world)
            ar.append(time.perf_counter() - t0)
    ar = []
    for _ in range(args.warmup):
        run()
    ar.clear()
    elapsed = timed_region(run, args.steps, world, None)
    ok = bool(torch.allclose(buf[:4], torch.full((4,), (world + 1) / 2.0)))
    if rank != 0:
        if world > 1:
            dist.destroy_process_group()
        return
    ms = 1000.0 * elapsed / max(1, args.steps)
    mc, _, _ = C.lstmformer_config(ratio=args.ratio)
    step_flop = (model_flops_per_frame(mc, args.ratio) + attn_flops_per_frame(mc, args.ratio, args.seq)) \
        * args.batch * args.seq
    fams = {"gemm": 343, "lstm_fwd": 11, "lstm_bwd": 11, "attn_fwd": 10, "attn_bwd": 10}
    kernels, roof = families({f: [(0.0417 + 1e-4 * i, 4.1296301104761906e9) for i in range(n)]
                              for f, n in fams.items()}, 1)
    roof["probe"] = {"eager_steps": 2, "preroll_ms": 300.0, "host_submit_ms": 51.3, "host_ahead": True}
    roof["trace_check"] = trace_check(roof)
    cpu = dict(value=4062.41, unit="frames/s", kind="port", cores=16, physical_cores_available=128,
               logical_cpus_available=256, cpu_model="AMD EPYC 9575F 64-Core Processor",
               thread_sweep_s_per_B8_step={"8": 0.646, "16": 0.595, "32": 1.103, "64": 2.891, "128": 9.814},
               sample="oracle/mrg_oracle.py lstmformer train step (fwd+loss+bwd+AdamW; LSTMs on the fused ATen op "
                      "nn.LSTM uses on CPU) B=64 T=300 r=1 (the full workload), median of 5 steps after 2 "
                      "warm-up, 16 threads, 2026-01-01")
    sec = {}
    if world == 1:
        names = ["C2_simple_lstm_fp32", "C2_simple_lstm_bf16", "C3_lstm_with_sampling_scheduled_sampling",
                 "lstmformer_generation", "lstmformer_gru_train", "lstmformer_r8_train"]
        for name in names:
            _put(sec, name, dict(_secondary_entry("synthetic " + name + " " + "x" * 160, 20.0, 19200, 70e6,
                                                  "fp32", (kernels, roof), cpu), dry_run=True))
    out = headline_dict(args, world, ms, None, step_flop, roof, kernels, seen,
                        "gloo (dry run)" if world > 1 else None)
    out.update(dry_run=True, allreduce_mean_ok=ok, ranks_seen=seen, cpu_baseline=cpu if world == 1 else None)
    if ar:
        out["exchange"] = {"replay_ms": 0.0, "allreduce_ms": round(1e3 * sum(ar) / len(ar), 3),
                           "allreduce_bytes": buf.numel() * 4, "buckets": 1}
    if sec:
        out["secondary"] = secondary_summary(sec)
        out["speedup_vs_cpu_baseline"] = 221.4
    print(headline_json(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def model_flops_per_frame(cfg, ratio, gates=4):
    """Algorithmic training FLOPs per prediction frame (SURVEY §8d formula; train = 3 x fwd); gates = 3
    for the GRU mixers of config_gru.yaml (every recurrent layer a GRU)."""
    H, Hb, N, E = cfg.hidden_size, cfg.bottleneck_size, cfg.num_block, cfg.encoder_num_layer
    Fa, Fm, T = 40, 6, 1.0
    L = N * T + E * ratio * T + E * T
    lstm = 4 * gates * H * H * L
    lin = (4 * T * H * Fm + 2 * ratio * T * H * Fa + 2 * H * H * L
           + N * (12 * T * H * H + 4 * H * H * (ratio * T + T) + 4 * T * H * H + 4 * T * H * Hb)
           + 2 * T * (H * Hb + Hb * Fm))
    return 3.0 * (lstm + lin)   # attention pairs are O(T) per frame; added separately by caller


def attn_flops_per_frame(cfg, ratio, T):
    H, N = cfg.hidden_size, cfg.num_block
    fwd = N * 4 * H * (ratio * T * (T + 1) / 2 + T * (T + 1) / 2) / T
    return 3.0 * fwd


def host_cpu():
    """(physical cores, logical CPUs, model name) of the CPUs this process may run on (/proc/cpuinfo
    restricted to sched_getaffinity): the CPU baseline uses every physical core."""
    allowed = os.sched_getaffinity(0)
    cores, model, cur = set(), "unknown", {}
    try:
        with open("/proc/cpuinfo") as f:
            for line in list(f) + ["\n"]:
                if not line.strip():
                    if cur.get("processor") is not None and int(cur["processor"]) in allowed:
                        cores.add((cur.get("physical id", "0"), cur.get("core id", cur["processor"])))
                        model = cur.get("model name", model)
                    cur = {}
                    continue
                k, _, v = line.partition(":")
                cur[k.strip()] = v.strip()
    except OSError:
        pass
    return max(1, len(cores)), len(allowed), model


_CPU = {}


def _cpu_setup(args):
    """Thread count of every CPU baseline, chosen once: the fastest of {8, 16, 32, 64, all physical
    cores} on a bounded lstmformer training sample (B=8, T=300), because on a shared multi-GPU host
    the oneDNN LSTM slows down past the cores it really gets (r02: 128 threads ran the headline step
    5-9x slower than 16).  --cpu-threads N pins it instead.  The sweep is reported."""
    if _CPU:
        torch.set_num_threads(_CPU["cores"])
        return dict(_CPU)
    phys, logical, model = host_cpu()
    sweep = {}
    if args.cpu_threads > 0:
        best = args.cpu_threads
    else:
        from oracle import mrg_oracle as O
        from multimodalreactiongeneration_amd import configs as C
        from multimodalreactiongeneration_amd.model import Metaformer
        from multimodalreactiongeneration_amd.synthetic import make_batch, clone_batch
        O.ATEN_LSTM = True
        mc, oc, me = C.lstmformer_config(ratio=1)
        torch.manual_seed(0)
        sd = {k: v.detach().clone() for k, v in Metaformer(mc, oc, me).state_dict().items()}
        batch = make_batch(B=8, T=300, seed=1234)
        for t in sorted({c for c in (8, 16, 32, 64, phys) if c <= phys}):
            torch.set_num_threads(t)
            O.run_train_step(O.metaformer_training_loss, sd, oc, mc, clone_batch(batch))
            t0 = time.perf_counter()
            O.run_train_step(O.metaformer_training_loss, sd, oc, mc, clone_batch(batch))
            sweep[t] = round(time.perf_counter() - t0, 3)
            progress(f"  cpu thread sweep: {t} threads {sweep[t]:.2f} s")
        best = min(sweep, key=sweep.get)
    torch.set_num_threads(best)
    _CPU.update(cores=torch.get_num_threads(), physical_cores_available=phys, logical_cpus_available=logical,
                cpu_model=model, thread_sweep_s_per_B8_step=sweep or None)
    return dict(_CPU)


def _median(xs):
    xs = sorted(xs)
    return xs[len(xs) // 2]


def _time_cpu(fn, warm, steps):
    for i in range(warm):
        fn()
        progress(f"  cpu warm-up {i + 1}/{warm}")
    times = []
    for i in range(steps):
        t0 = time.perf_counter()
        fn()
        times.append(time.perf_counter() - t0)
        progress(f"  cpu step {i + 1}/{steps}: {times[-1]:.2f} s ({torch.get_num_threads()} threads)")
    return _median(times)


def cpu_baseline(args, mc, oc):
    """The oracle (CPU fp32 restatement of the reference, same workload) on this host's cores."""
    from oracle import mrg_oracle as O
    from multimodalreactiongeneration_amd.model import Metaformer
    from multimodalreactiongeneration_amd.synthetic import make_batch, clone_batch
    info = _cpu_setup(args)
    O.ATEN_LSTM = True   # the oneDNN LSTM op the reference's nn.LSTM runs on CPU, not the parity loop
    torch.manual_seed(0)
    sd = {k: v.detach().clone() for k, v in Metaformer(mc, oc, {"use_centroid": True, "use_angle": True,
                                                                   "delta_order": 0}).state_dict().items()}
    batch = make_batch(B=args.batch, T=args.seq, ratio=args.ratio, seed=1234)
    t = _time_cpu(lambda: O.run_train_step(O.metaformer_training_loss, sd, oc, mc, clone_batch(batch)),
                  args.cpu_warmup, args.cpu_steps)
    return dict(value=round(args.batch * args.seq / t, 2), unit="frames/s", kind="port", **info,
                sample=f"oracle/mrg_oracle.py lstmformer train step (fwd+loss+bwd+AdamW; LSTMs on the fused ATen op "
                       f"nn.LSTM uses on CPU) B={args.batch} T={args.seq} r={args.ratio} (the full workload), median "
                       f"of {args.cpu_steps} steps after {args.cpu_warmup} warm-up, {info['cores']} threads, "
                       f"{time.strftime('%Y-%m-%d')}")


def families(per, nsteps):
    """Per kernel family: time, launches, algorithmic FLOPs and achieved TF/s over ``nsteps`` probed
    steps; returns (kernels, roofline of the family with the most time per step)."""
    kernels, roof = {}, None
    for f in FAMILIES:
        v = per.get(f, [])
        if not v:
            continue
        fms = sum(t for t, _ in v) / nsteps
        work = sum(w for _, w in v) / nsteps
        n = len(v) / nsteps
        tf = work / (fms / 1e3) / 1e12
        kernels[f] = {"ms_per_step": round(fms, 3), "launches_per_step": n,
                      "avg_launch_ms": round(fms / n, 4), "algorithmic_flop_per_launch": round(work / n),
                      "achieved_tflops": round(tf, 2), "frac_of_fp32_peak": round(tf / FP32_MFMA_PEAK_TF, 4)}
    if kernels:
        dom = max(kernels, key=lambda f: kernels[f]["ms_per_step"])
        k = kernels[dom]
        roof = {"kernel": FAMILIES[dom], "family": dom, "bound": "mfma", "achieved": k["achieved_tflops"],
                "peak": FP32_MFMA_PEAK_TF, "unit": "TFLOP/s", "frac": k["frac_of_fp32_peak"],
                "traffic": pmc_traffic(dom), "avg_launch_ms": k["avg_launch_ms"],
                "launches_per_step": k["launches_per_step"],
                "algorithmic_flop_per_launch": k["algorithmic_flop_per_launch"],
                "peak_note": PEAK_NOTES.get(dom, "")}
    return kernels, roof


def gen_flops_per_frame(cfg, ratio):
    """Algorithmic forward FLOPs of one generated frame (Metaformer.prediction: a T = 1 forward with
    zero recurrent state, lstmformer.py:498-521): LSTM input projections only (8H^2 per token-layer;
    h0 = 0 makes h W_hh zero work), the Linear layers at T = 1, one visible attention pair per head."""
    H, Hb, N, E = cfg.hidden_size, cfg.bottleneck_size, cfg.num_block, cfg.encoder_num_layer
    Fa, Fm = 40, 6
    L = N + E * ratio + E
    lin = (4 * H * Fm + 2 * ratio * H * Fa + 2 * H * H * L
           + N * (12 * H * H + 4 * H * H * (ratio + 1) + 4 * H * H + 4 * H * Hb) + 2 * (H * Hb + Hb * Fm))
    return 8 * H * H * L + lin + N * 4 * H * (ratio + 1)


# SURVEY §8d algorithmic training FLOPs per frame (fwd x 3), B = 64, T = 300, r = 1
C2_MFLOP_PER_FRAME = 677.3e3 / (64 * 300)      # simple_lstm: 677.3 GFLOP / step
C3_MFLOP_PER_FRAME = 97.25e3 / (64 * 300)      # lstm_with_sampling scheduled sampling: 97.25 GFLOP / step


def _timed_replay(replay, steps, warm, pre=None):
    for _ in range(warm):
        if pre is not None:
            pre()
        replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        if pre is not None:
            pre()
        replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps * 1e3


def _preroll(ms):
    """Hold the current stream for `ms` with one tiny busy kernel (mrg_debug_busy: one 64-lane
    workgroup), so the host queues the eager probe steps that follow while the GPU waits: the
    probed launches then run back to back beside each other as in the graph replay, not spaced out
    by host submission (r03: without it the eager step ran host-bound)."""
    from multimodalreactiongeneration_amd import _lib
    from multimodalreactiongeneration_amd import functional as Fn
    _lib.check(_lib.load().mrg_debug_busy(1, 64, 256, float(ms) * 1e3, Fn._stream()), "preroll")


def _probe_steps(step, n=1, preroll_ms=150.0):
    """Per-family kernel time over n eager steps with the replay's stream schedule (weight gradients
    on the side stream, as in the captured graph), every kernel of a probed library call timed by
    events bound to that kernel (functional.probe_start(kernel=True): hipExtLaunchKernelGGL), i.e.
    its own execution beside whatever runs beside it, as rocprofv3 reports it; queued behind a
    pre-roll (see _preroll).  The committed trace of the same command holds these probe steps
    (tools/tools_trace_roofline.py "probe") and the graph-replayed ones ("replay").
    Returns (kernels, roofline)."""
    from multimodalreactiongeneration_amd import functional as Fn
    torch.cuda.synchronize()
    _preroll(preroll_ms * n)
    t0 = time.perf_counter()
    Fn.probe_start(*FAMILIES, kernel=True)
    for _ in range(n):
        step()
    host_ms = (time.perf_counter() - t0) * 1e3
    per = Fn.probe_stop(with_work=True)
    kernels, roof = families(per, n)
    ahead = host_ms < preroll_ms * n
    if roof is not None:
        roof["probe"] = {"eager_steps": n, "preroll_ms": preroll_ms * n, "host_submit_ms": round(host_ms, 1),
                         "host_ahead": ahead}
    return kernels, roof


def _secondary_entry(workload, ms, frames, flop_per_frame, dtype, kern, cpu, peak=FP32_MFMA_PEAK_TF,
                     peak_note="fp32 dense matrix peak"):
    kernels, roof = kern
    if roof is not None:   # the committed PMC summary is of the headline workload, not this one
        roof = dict(roof, traffic=None)
    value = frames / ms * 1e3
    ach = flop_per_frame * value / 1e12
    return {"workload": workload, "ms_per_step": round(ms, 3), "value": round(value, 2), "unit": "frames/s",
            "dtype": dtype,
            "whole_step_roofline": {"bound": "mfma", "algorithmic_mflop_per_frame": round(flop_per_frame / 1e6, 3),
                                    "achieved_tflops": round(ach, 3), "peak": peak, "frac": round(ach / peak, 4),
                                    "peak_note": peak_note},
            "roofline": roof, "kernels": kernels, "cpu_baseline": cpu,
            "speedup_vs_cpu_baseline": None if not cpu else round(value / cpu["value"], 1)}


def emit(obj):
    """One JSON line on stdout (flushed): the secondary configs each get their own line BEFORE the
    headline, so the headline is the last stdout line and stays small (a 20.7 KB line with
    the secondary block inside was not parsed by the driver)."""
    print(json.dumps(obj), flush=True)


def _put(out, name, entry):
    out[name] = entry
    emit({"secondary": name, **entry})


def secondary_summary(sec):
    """The headline's pointer to the secondary lines: per config ms/step, frames/s, whole-step roofline
    fraction and the speed-up over its CPU baseline (full entries on the lines printed before)."""
    return {k: {"ms_per_step": v["ms_per_step"], "value": v["value"], "frac": v["whole_step_roofline"]["frac"],
                "vs_cpu": v.get("speedup_vs_cpu_baseline")} for k, v in sec.items()}


def headline_json(out):
    """The headline line, kept under HEADLINE_MAX_BYTES: if a future field pushes it over, the
    per-family ``kernels`` split is cut to ms/step first, then the secondary summary (its configs are on
    their own lines), rank list and DDP check are dropped; ``roofline`` and ``cpu_baseline`` always stay."""
    line = json.dumps(out)
    if len(line) > HEADLINE_MAX_BYTES and "kernels" in out:
        out = dict(out, kernels={k: v.get("ms_per_step") for k, v in out["kernels"].items()})
        line = json.dumps(out)
    for key in ("secondary", "ranks_seen", "ddp_check"):
        if len(line) <= HEADLINE_MAX_BYTES:
            break
        if key in out:
            progress(f"headline over {HEADLINE_MAX_BYTES} bytes: dropping {key}")
            out = {k: v for k, v in out.items() if k != key}
            line = json.dumps(out)
    return line


def headline_dict(args, world, ms, value, step_flop, roof, kernels, seen, allreduce):
    """The headline line's fields (BASELINE.json metric, the driver's contract); the caller adds the
    N>1 checks, the secondary summary and the CPU baseline."""
    return {
        "metric": METRIC, "value": None if value is None else round(value, 2), "unit": "frames/s",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "fp32", "data": "synthetic",
        "config": {"workload": "lstmformer train step (fwd+Huber+bwd+AdamW), BASELINE configs[3]/[4]",
                   "model": "lstmformer H=256 blocks=5 enc_layers=5 heads=4 bottleneck=64 (13,052,678 params)",
                   "global_batch": args.batch * world, "seq_len": args.seq, "audio_ratio": args.ratio,
                   "parallelism": f"dp{world}", "hip_graph": bool(args.graph), "allreduce": allreduce,
                   "wgrad_side_stream": bool(args.wgrad_stream),
                   "wgrad_beside_recurrence": bool(args.wgrad_stream and args.wgrad_defer)},
        "whole_step_roofline": {"bound": "mfma", "algorithmic_tflop_per_step": round(step_flop / 1e12, 4),
                                "achieved_tflops": round(step_flop / (ms / 1000.0) / 1e12, 3),
                                "peak": FP32_MFMA_PEAK_TF,
                                "frac": round(step_flop / (ms / 1000.0) / 1e12 / FP32_MFMA_PEAK_TF, 4)},
        "roofline": roof,
        "kernels": kernels,
        "cpu_baseline": None,
        "ranks_seen": {k: v for k, v in seen.items() if k != "ranks"} | {"devices": [r["device"] for r in seen["ranks"]]},
    }


def secondary(args, dev):
    """The other 1-GPU BASELINE configs (configs[1], configs[2]) and lstmformer generation (§8f1)."""
    import numpy as np
    from multimodalreactiongeneration_amd import configs as C
    from multimodalreactiongeneration_amd import functional as Fn
    from multimodalreactiongeneration_amd.graphs import capture
    from multimodalreactiongeneration_amd.model import LSTMwithSample, SimpleLSTM, Metaformer
    from multimodalreactiongeneration_amd.synthetic import make_batch, make_simple_batch
    out = {}
    K, W, B, T = 10, 3, 64, 300
    cpu_on = args.cpu_baseline
    from oracle import mrg_oracle as O  # CPU baselines only (bounded samples)
    O.ATEN_LSTM = True

    # C2 simple_lstm, B=64 T=300 (BASELINE configs[1])
    for dtype in ("fp32", "bf16"):
        cfg, oc, me = C.simple_lstm_config()
        torch.manual_seed(0)
        m = SimpleLSTM(cfg, oc, me).set_precision("32" if dtype == "fp32" else "bf16")
        sd = {k: v.detach().clone() for k, v in m.state_dict().items()}
        m = m.to(dev)
        opt = m.configure_optimizers()["optimizer"]
        batch = make_simple_batch(B=B, T=T, device=dev)

        def step_c2():
            opt.zero_grad()
            m.training_step(batch)["loss"].backward()
            opt.step()
        progress(f"C2 simple_lstm {dtype}")
        replay = capture(step_c2, 2, preserve=opt.state_tensors())
        ms = _timed_replay(replay, K, W)
        kern = _probe_steps(step_c2)
        cpu = None
        if cpu_on and dtype == "fp32":   # one CPU reference (fp32) serves both precisions
            info = _cpu_setup(args)
            cb = 8
            a, mo, tg = make_simple_batch(B=cb, T=T, seed=1234)
            t = _time_cpu(lambda: O.run_train_step(O.simple_lstm_training_loss, sd, oc, cfg, a, mo, tg), 1, 1)
            cpu = dict(value=round(cb * T / t, 2), unit="frames/s", kind="port", **info,
                       sample=f"oracle simple_lstm train step (fwd+MSE+bwd+AdamW, fused ATen LSTMs) on a bounded "
                              f"sample B={cb} T={T} (same per-clip work as B=64), 1 timed after 1 warm-up")
        if dtype == "bf16":
            cpu = out["C2_simple_lstm_fp32"]["cpu_baseline"]
            _put(out, f"C2_simple_lstm_{dtype}", _secondary_entry(
                "simple_lstm train step B=64 T=300 (BASELINE configs[1]) with model.precision='bf16': GEMM "
                "operands bf16 on the bf16 matrix cores, fp32 accumulation; recurrence, LayerNorm, softmax, "
                "loss and AdamW fp32; HIP graph", ms, B * T, C2_MFLOP_PER_FRAME * 1e6,
                "bf16 (GEMM operands) / fp32 accumulate", kern, cpu, peak=BF16_MFMA_PEAK_TF,
                peak_note="bf16 dense matrix peak (the configured compute dtype)"))
        else:
            _put(out, f"C2_simple_lstm_{dtype}", _secondary_entry(
                "simple_lstm train step B=64 T=300 (BASELINE configs[1] shape) in fp32, HIP graph", ms, B * T,
                C2_MFLOP_PER_FRAME * 1e6, dtype, kern, cpu))
        del m, opt, replay

    progress("C3 scheduled sampling")
    # C3 lstm_with_sampling, scheduled sampling (BASELINE configs[2])
    mc, oc, me = C.lstm_with_sampling_config(use_scheduled_sampling=True)
    torch.manual_seed(0)
    m = LSTMwithSample(mc, oc, me)
    m.current_epoch = 30
    sd = {k: v.detach().clone() for k, v in m.state_dict().items()}
    m = m.to(dev)
    opt = m.configure_optimizers()["optimizer"]
    batch = make_batch(B=B, T=T, lead=12, seed=1234, device=dev)
    mask = torch.from_numpy(np.random.RandomState(7).rand(T) < 0.5).to(dev)
    rng = np.random.RandomState(7)

    def refresh():  # the host draw of lstm_with_sample.py:389 into the static device mask
        mask.copy_(torch.from_numpy(rng.rand(T) < 0.5), non_blocking=True)

    def step_c3():
        opt.zero_grad()
        m.training_step(batch, sampling_mask=mask)["loss"].backward()
        opt.step()
    replay = capture(step_c3, 2, preserve=opt.state_tensors())
    ms = _timed_replay(replay, K, W, pre=refresh)
    # per-family kernel time from kernel-bound probes: the frame loops are two launches (the "ssd"
    # family), the rest ~100 launches (sampler recurrences, products over all frames)
    refresh()
    kern = _probe_steps(step_c3)
    cpu = None
    if cpu_on:
        info = _cpu_setup(args)
        cb = 16
        cbatch = make_batch(B=cb, T=T, lead=12, seed=1234)
        cmask = torch.from_numpy(np.random.RandomState(7).rand(T) < 0.5)
        t = _time_cpu(lambda: O.run_train_step(O.lstm_with_sample_training_loss, sd, oc, mc, cbatch,
                                               sampling_mask=cmask), 1, 2)
        cpu = dict(value=round(cb * T / t, 2), unit="frames/s", kind="port", **info,
                   sample=f"oracle lstm_with_sampling scheduled-sampling train step (300 AR frames, mask "
                          f"RandomState(7)<0.5, lead 12) on a bounded sample B={cb} T={T}, median of 2 after 1 warm-up")
    _put(out, "C3_lstm_with_sampling_scheduled_sampling", _secondary_entry(
        "lstm_with_sampling scheduled-sampling train step B=64 T=300 lead 12 (BASELINE configs[2]), HIP graph, "
        "mask refreshed from the host RNG before every replay", ms, B * T, C3_MFLOP_PER_FRAME * 1e6, "fp32",
        kern, cpu))
    del m, opt, replay

    progress("lstmformer generation")
    # lstmformer autoregressive generation (Metaformer.prediction, full generation)
    mc, oc, me = C.lstmformer_config(ratio=1)
    torch.manual_seed(0)
    m = Metaformer(mc, oc, me)
    sd = {k: v.detach().clone() for k, v in m.state_dict().items()}
    m = m.to(dev).eval()
    batch = make_batch(B=B, T=T, lead=12, seed=1234, device=dev)
    gmask = torch.ones(T, dtype=torch.bool, device=dev)

    def gen():
        with torch.no_grad():
            m._generate(batch, sampling_mask=gmask)
    replay = capture(gen, 2)
    ms = _timed_replay(replay, 5, 2)
    kern = _probe_steps(gen)   # every frame-loop kernel timed by kernel-bound events (generate.py probes)
    cpu = None
    if cpu_on:
        info = _cpu_setup(args)
        ct = 40
        cbatch = make_batch(B=B, T=ct, lead=12, seed=1234)
        with torch.no_grad():
            t = _time_cpu(lambda: O.metaformer_prediction(sd, mc, cbatch, torch.ones(ct, dtype=torch.bool)), 0, 1)
        cpu = dict(value=round(B * ct / t, 2), unit="frames/s", kind="port", **info,
                   sample=f"oracle Metaformer.prediction (full generation, no grad) on a bounded sample of "
                          f"{ct} frames x B={B} (per-frame cost is independent of T), 1 run")
    _put(out, "lstmformer_generation", _secondary_entry(
        "lstmformer autoregressive generation (Metaformer.prediction, full_generation, eval, no grad) "
        "B=64 x 300 frames, HIP graph; one step = one 64-clip batch; fused frame loop (generate.py: other "
        "modalities' encoders and one-key attention hoisted over all frames, 26 launches per frame)", ms, B * T,
        gen_flops_per_frame(mc, 1), "fp32",
        kern, cpu))
    del m, replay

    progress("lstmformer GRU config")
    # lstmformer with config_gru.yaml's mixers (every recurrent layer a GRU)
    mc, oc, me = C.lstmformer_config(ratio=1, emb_mixers=("gru", "gru", "gru"))
    torch.manual_seed(0)
    m = Metaformer(mc, oc, me)
    sd = {k: v.detach().clone() for k, v in m.state_dict().items()}
    m = m.to(dev)
    opt = m.configure_optimizers()["optimizer"]
    batch = make_batch(B=B, T=T, seed=1234, device=dev)

    def step_gru():
        opt.zero_grad()
        m.training_step(list(batch))["loss"].backward()
        opt.step()
    replay = capture(step_gru, 2, preserve=opt.state_tensors())
    ms = _timed_replay(replay, K, W)
    kern = _probe_steps(step_gru)
    cpu = None
    if cpu_on:
        info = _cpu_setup(args)
        cb = 8
        cbatch = make_batch(B=cb, T=T, seed=1234)
        t = _time_cpu(lambda: O.run_train_step(O.metaformer_training_loss, sd, oc, mc, list(cbatch)), 1, 1)
        cpu = dict(value=round(cb * T / t, 2), unit="frames/s", kind="port", **info,
                   sample=f"oracle lstmformer train step with GRU mixers (fwd+loss+bwd+AdamW, the fused ATen GRU "
                          f"nn.GRU runs on CPU) on a bounded sample B={cb} T={T} r=1, 1 timed after 1 warm-up")
    _put(out, "lstmformer_gru_train", _secondary_entry(
        "lstmformer train step with config_gru.yaml's GRU mixers (persistent GRU recurrences), B=64 T=300 r=1, "
        "HIP graph", ms, B * T, model_flops_per_frame(mc, 1, gates=3) + attn_flops_per_frame(mc, 1, T), "fp32",
        kern, cpu))
    del m, opt, replay

    progress("lstmformer r=8")
    # the reference-faithful audio rate (pred_fps 12.5: audio T = 8 x 300 = 2400, config.yaml:200; SURVEY §8
    # conventions, secondary row): same step as the headline at ratio 8
    mc, oc, me = C.lstmformer_config(ratio=8)
    torch.manual_seed(0)
    m = Metaformer(mc, oc, me)
    sd = {k: v.detach().clone() for k, v in m.state_dict().items()}
    m = m.to(dev)
    opt = m.configure_optimizers()["optimizer"]
    batch = make_batch(B=B, T=T, ratio=8, seed=1234, device=dev)
    one = torch.ones((), device=dev)

    def step_r8():
        opt.zero_grad()
        m.training_step(list(batch))["loss"].backward(one)
        opt.step()
    replay = capture(step_r8, 2, preserve=opt.state_tensors())
    ms = _timed_replay(replay, K, W)
    kern = _probe_steps(step_r8)
    cpu = None
    if cpu_on:
        info = _cpu_setup(args)
        cb = 4
        cbatch = make_batch(B=cb, T=T, ratio=8, seed=1234)
        t = _time_cpu(lambda: O.run_train_step(O.metaformer_training_loss, sd, oc, mc, list(cbatch)), 1, 1)
        cpu = dict(value=round(cb * T / t, 2), unit="frames/s", kind="port", **info,
                   sample=f"oracle lstmformer train step r=8 (audio T=2400; fwd+loss+bwd+AdamW, fused ATen LSTMs) "
                          f"on a bounded sample B={cb} T={T}, 1 timed after 1 warm-up")
    _put(out, "lstmformer_r8_train", _secondary_entry(
        "lstmformer train step at the reference-faithful audio rate r=8 (pred_fps 12.5, audio T=2400), B=64 T=300, "
        "HIP graph", ms, B * T, model_flops_per_frame(mc, 8) + attn_flops_per_frame(mc, 8, T), "fp32", kern, cpu))
    del m, opt, replay
    Fn.check_errors()
    return out


def main():
    args = parse()
    launch_or_check(args)          # N > 1 without torch.distributed.run: launches N ranks and exits
    if args.dry_run:
        return dry_run(args)
    from multimodalreactiongeneration_amd import configs as C
    from multimodalreactiongeneration_amd import functional as Fn
    from multimodalreactiongeneration_amd.graphs import capture
    from multimodalreactiongeneration_amd.ddp import init_from_env, broadcast_parameters, GradReducer, NativeComm
    from multimodalreactiongeneration_amd.model import Metaformer
    from multimodalreactiongeneration_amd.synthetic import make_batch

    shared = bool(args.shared_device_gloo)
    local = 0 if shared else int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)    # before the process group, so RCCL binds rank -> its own GPU
    rank, world = init_from_env(backend="gloo" if shared else None)
    dev = torch.device("cuda", local)
    seen = ranks_seen(rank, world, dev, shared=shared)
    turns = _DeviceTurns(shared and world > 1)
    if world != args.gpus:
        raise RuntimeError(f"bench.py: --gpus {args.gpus} but {world} ranks initialised")
    mc, oc, me = C.lstmformer_config(ratio=args.ratio)
    if args.lstm_group:
        from multimodalreactiongeneration_amd import _lib
        _lib.check(_lib.load().mrg_lstm_config(args.lstm_group), "mrg_lstm_config")
    Fn.set_wgrad_stream(bool(args.wgrad_stream))
    Fn.set_wgrad_defer(bool(args.wgrad_defer))
    torch.manual_seed(0)
    model = Metaformer(mc, oc, me).to(dev)
    broadcast_parameters(model)
    opt = model.configure_optimizers()["optimizer"]
    comm = NativeComm() if (args.comm == "native" and world > 1) else None
    reducer = GradReducer(opt.flat_grad, comm=comm)
    batch = make_batch(B=args.batch, T=args.seq, ratio=args.ratio, seed=1234 + rank, device=dev)

    one = torch.ones((), device=dev)   # d loss / d loss, made once (backward() would fill a new one per step)

    def fwd_bwd():
        opt.zero_grad()
        loss = model.training_step(list(batch))["loss"]
        loss.backward(one)
        return loss

    def step():
        loss = fwd_bwd()
        reducer.allreduce()
        opt.step()
        return loss

    split = []       # N > 1: per-step [start, after replay, after all-reduce] events
    check = None
    if args.ddp_check and world > 1:
        check = ddp_grad_check(model, opt, reducer, batch, args, rank, world, dev, turns)

    run = step
    if args.graph:
        # capture fwd+bwd(+AdamW at N=1) once; the RCCL all-reduce stays eager between replays at N>1
        captured = step if world == 1 else fwd_bwd
        with turns:
            replay = capture(captured, max(2, args.warmup), preserve=opt.state_tensors())
        if world == 1:
            run = replay
        else:
            def run():
                # HIP events on the current stream bracket the replay and the exchange of every step,
                # so the line reports them apart (allreduce_ms: the bucketed all-reduce, which the
                # current stream waits for, plus the error-flag agreement)
                e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
                e[0].record()
                with turns:
                    replay()
                e[1].record()
                reducer.allreduce()
                e[2].record()
                opt.step()
                split.append(e)
    else:
        for _ in range(args.warmup):
            step()
    for _ in range(args.warmup):
        run()
    torch.cuda.synchronize()
    Fn.check_errors()

    split.clear()
    elapsed = timed_region(run, args.steps, world, dev)
    Fn.check_errors()
    exchange = None
    if split:
        rep_ms = sum(e[0].elapsed_time(e[1]) for e in split) / len(split)
        ar_ms = sum(e[1].elapsed_time(e[2]) for e in split) / len(split)
        exchange = {"replay_ms": round(rep_ms, 3), "allreduce_ms": round(ar_ms, 3),
                    "allreduce_bytes": opt.flat_grad.numel() * 4, "buckets": len(reducer.buckets)}
    ms = 1000.0 * elapsed / args.steps
    frames = args.batch * args.seq * world
    value = frames * args.steps / elapsed

    # live per-family kernel timing: HIP events recorded on the launch stream around every library
    # call of two eager steps right after the timed region (a graph replay cannot be bracketed);
    # each launch carries its algorithmic FLOPs (functional._probe), so achieved = FLOPs / time
    # (the replay's stream schedule: weight gradients on the side stream, so a bracketed launch runs
    # beside the same work as in the graph; a weight-gradient bracket includes its split-K reduce)
    # (every rank steps, the all-reduce is collective; rank 0 records)
    if shared:
        kernels, roof = {}, None    # a test of the code path: ranks take turns, no kernel figures
    elif rank == 0:
        kernels, roof = _probe_steps(step, 2)
        if roof is not None:
            roof["trace_check"] = trace_check(roof)
    else:
        for _ in range(2):
            step()
        kernels, roof = {}, None
    agree = params_agree(opt) if world > 1 else None
    Fn.check_errors()
    step_flop = (model_flops_per_frame(mc, args.ratio) + attn_flops_per_frame(mc, args.ratio, args.seq)) \
        * args.batch * args.seq
    out = headline_dict(args, world, ms, value, step_flop, roof, kernels, seen,
                        ("mrg_comm (libmrg RCCL)" if comm is not None else "torch.distributed RCCL")
                        if world > 1 else None)
    if world > 1:
        out["params_bitwise_equal_across_ranks"] = agree
        if exchange is not None:     # rank 0's split; the step time above is the max over ranks
            out["exchange"] = exchange
        if check is not None:
            out["ddp_check"] = check
    if shared:
        out["value"] = None   # ranks shared one GPU and took turns: a test of the N>1 path, not a measurement
        out["shared_device_test"] = True
    if rank == 0:
        progress(f"headline {ms:.3f} ms/step")
    if rank == 0 and world == 1 and args.secondary:

        out["secondary"] = secondary_summary(secondary(args, dev))
    if rank == 0 and world == 1 and args.cpu_baseline:
        progress("headline CPU baseline")
        out["cpu_baseline"] = cpu_baseline(args, mc, oc)
        out["speedup_vs_cpu_baseline"] = round(out["value"] / out["cpu_baseline"]["value"], 1)
    if rank == 0:
        print(headline_json(out), flush=True)     # the LAST stdout line
    if comm is not None:
        comm.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
