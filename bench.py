"""Benchmark: lstmformer training frames/s (BASELINE.json metric), fp32, synthetic data.

    python bench.py [--gpus N --steps K --warmup W]          (N > 1 under torch.distributed.run)

A step = Metaformer.training_step (fwd + masked Huber loss) + backward +
RCCL gradient all-reduce (N > 1) + fused AdamW, on B=64 x T=300 frames per
GPU (weak scaling).  Inputs are resident in HBM before timing.  Prints ONE
JSON line on rank 0 with the live roofline of the dominant kernel (HIP events
around its launches inside the timed region) and the CPU oracle baseline
timed on this host (rank 0, N=1 only).
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
HBM_PEAK_GBS = 8000.0
PMC_SUMMARY = os.path.join(ROOT, "profiles", "r01_pmc_summary.json")

# probe name (functional._probe) -> kernels it brackets; FLOPs are algorithmic
FAMILIES = {
    "gemm": "gemm_x6_kernel (+ splitk_reduce4_kernel): every GEMM of the step, 2MNK FLOP per launch",
    "lstm_fwd": "lstm_fwd_kernel<256,8,BS>: persistent recurrence, 8H^2 FLOP per (b, t) per layer",
    "lstm_bwd": "lstm_bwd_kernel<256,8,BS>: persistent reverse recurrence, 8H^2 FLOP per (b, t) per layer",
    "attn_fwd": "attn_fwd_kernel<64>: block-causal flash attention, 4D FLOP per visible (q, k) pair per head",
    "attn_bwd": "attn_bwd_dq_kernel<64> + attn_bwd_dkv_kernel<64>: 10D FLOP per visible pair per head",
}
PEAK_NOTES = {
    "gemm": "peak = f32 dense matrix peak (the dtype's); the GEMMs compute fp32 as a three-plane bf16 split "
            "(6 bf16 MFMAs per product, fp32-class error), whose own MFMA ceiling is 2500/6 = 416.7 TFLOP/s",
    "lstm_fwd": "latency-bound (one cross-CU hand-off per time step); VALU v_pk_fma_f32 peak = 157.3",
    "lstm_bwd": "latency-bound (one cross-CU hand-off per time step); VALU v_pk_fma_f32 peak = 157.3",
}
# rocprofv3 kernel-name prefix of each family in the PMC summary (tools/tools_pmc_summary.py)
PMC_KEYS = {"gemm": "gemm_x6_kernel", "lstm_fwd": "lstm_fwd_kernel", "lstm_bwd": "lstm_bwd_kernel",
            "attn_fwd": "attn_fwd_kernel", "attn_bwd": "attn_bwd"}


def pmc_traffic(family):
    """HBM bytes per launch of a family from the committed rocprofv3 FETCH_SIZE/WRITE_SIZE passes."""
    try:
        with open(PMC_SUMMARY) as f:
            doc = json.load(f)
        fam = doc["families"].get(PMC_KEYS[family])
        return None if fam is None else round(fam["hbm_bytes_per_launch"])
    except (OSError, KeyError, ValueError):
        return None


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--seq", type=int, default=300)
    ap.add_argument("--ratio", type=int, default=1, help="audio frames per prediction frame (8 = reference rate)")
    ap.add_argument("--graph", type=int, default=1, help="replay the step as a HIP graph")
    ap.add_argument("--cpu-baseline", type=int, default=1)
    ap.add_argument("--cpu-steps", type=int, default=2)
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--wgrad-stream", type=int, default=1,
                    help="weight-gradient GEMMs on a side stream (functional._side); 0 = one stream")
    ap.add_argument("--lstm-group", type=int, default=0, help="workgroups per LSTM row group at H=256 (8|16; 0 = library default)")
    return ap.parse_args()


def model_flops_per_frame(cfg, ratio):
    """Algorithmic training FLOPs per prediction frame (SURVEY §8d formula; train = 3 x fwd)."""
    H, Hb, N, E = cfg.hidden_size, cfg.bottleneck_size, cfg.num_block, cfg.encoder_num_layer
    Fa, Fm, T = 40, 6, 1.0
    L = N * T + E * ratio * T + E * T
    lstm = 16 * H * H * L
    lin = (4 * T * H * Fm + 2 * ratio * T * H * Fa + 2 * H * H * L
           + N * (12 * T * H * H + 4 * H * H * (ratio * T + T) + 4 * T * H * H + 4 * T * H * Hb)
           + 2 * T * (H * Hb + Hb * Fm))
    return 3.0 * (lstm + lin)   # attention pairs are O(T) per frame; added separately by caller


def attn_flops_per_frame(cfg, ratio, T):
    H, N = cfg.hidden_size, cfg.num_block
    fwd = N * 4 * H * (ratio * T * (T + 1) / 2 + T * (T + 1) / 2) / T
    return 3.0 * fwd


def cpu_baseline(args, mc, oc):
    """The oracle (CPU fp32 restatement of the reference, same workload) on this host's cores."""
    from oracle import mrg_oracle as O
    from multimodalreactiongeneration_amd.model import Metaformer
    from multimodalreactiongeneration_amd.synthetic import make_batch, clone_batch
    torch.set_num_threads(args.cpu_threads)
    O.ATEN_LSTM = True   # the oneDNN LSTM op the reference's nn.LSTM runs on CPU, not the parity loop
    torch.manual_seed(0)
    sd = {k: v.detach().clone() for k, v in Metaformer(mc, oc, {"use_centroid": True, "use_angle": True,
                                                                   "delta_order": 0}).state_dict().items()}
    batch = make_batch(B=args.batch, T=args.seq, ratio=args.ratio, seed=1234)
    times = []
    for i in range(1 + args.cpu_steps):
        t0 = time.perf_counter()
        O.run_train_step(O.metaformer_training_loss, sd, oc, mc, clone_batch(batch))
        times.append(time.perf_counter() - t0)
    t = sorted(times[1:])[len(times[1:]) // 2]
    return {"value": round(args.batch * args.seq / t, 2), "unit": "frames/s", "cores": torch.get_num_threads(),
            "kind": "port",
            "sample": f"oracle/mrg_oracle.py lstmformer train step (fwd+loss+bwd+AdamW; LSTMs on the "
                      f"fused ATen op nn.LSTM uses on CPU) B={args.batch} T={args.seq} r={args.ratio}, median of "
                      f"{args.cpu_steps} steps after 1 warm-up, {torch.get_num_threads()} threads, "
                      f"{time.strftime('%Y-%m-%d')}"}


def main():
    args = parse()
    from multimodalreactiongeneration_amd import configs as C
    from multimodalreactiongeneration_amd import functional as Fn
    from multimodalreactiongeneration_amd.graphs import capture
    from multimodalreactiongeneration_amd.ddp import init_from_env, broadcast_parameters, GradReducer
    from multimodalreactiongeneration_amd.model import Metaformer
    from multimodalreactiongeneration_amd.synthetic import make_batch

    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)    # before the process group, so RCCL binds rank -> its own GPU
    rank, world = init_from_env()
    dev = torch.device("cuda", local)
    mc, oc, me = C.lstmformer_config(ratio=args.ratio)
    if args.lstm_group:
        from multimodalreactiongeneration_amd import _lib
        _lib.check(_lib.load().mrg_lstm_config(args.lstm_group), "mrg_lstm_config")
    Fn.set_wgrad_stream(bool(args.wgrad_stream))
    torch.manual_seed(0)
    model = Metaformer(mc, oc, me).to(dev)
    broadcast_parameters(model)
    opt = model.configure_optimizers()["optimizer"]
    reducer = GradReducer(opt.flat_grad)
    batch = make_batch(B=args.batch, T=args.seq, ratio=args.ratio, seed=1234 + rank, device=dev)

    def fwd_bwd():
        opt.zero_grad()
        loss = model.training_step(list(batch))["loss"]
        loss.backward()
        return loss

    def step():
        loss = fwd_bwd()
        reducer.allreduce()
        opt.step()
        return loss

    run = step
    if args.graph:
        # capture fwd+bwd(+AdamW at N=1) once; the RCCL all-reduce stays eager between replays at N>1
        captured = step if world == 1 else fwd_bwd
        replay = capture(captured, max(2, args.warmup))
        if world == 1:
            run = replay
        else:
            def run():
                replay()
                reducer.allreduce()
                opt.step()
    else:
        for _ in range(args.warmup):
            step()
    for _ in range(args.warmup):
        run()
    torch.cuda.synchronize()
    Fn.check_errors()

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        run()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    Fn.check_errors()
    ms = 1000.0 * elapsed / args.steps
    frames = args.batch * args.seq * world
    value = frames * args.steps / elapsed

    # live per-family kernel timing: HIP events recorded on the launch stream around every library
    # call of two eager steps right after the timed region (a graph replay cannot be bracketed);
    # each launch carries its algorithmic FLOPs (functional._probe), so achieved = FLOPs / time
    # (weight gradients on the current stream here, so the brackets time uncontended launches)
    fams = tuple(FAMILIES)
    side = Fn.set_wgrad_stream(False)
    if rank == 0:
        Fn.probe_start(*fams)
    for _ in range(2):      # every rank steps (the all-reduce is collective); rank 0 records
        step()
    per = Fn.probe_stop(with_work=True) if rank == 0 else {}
    Fn.set_wgrad_stream(side)
    kernels, roof = {}, None
    if rank == 0:
        for f in fams:
            v = per.get(f, [])
            if not v:
                continue
            fms = sum(t for t, _ in v) / 2.0
            work = sum(w for _, w in v) / 2.0
            n = len(v) / 2.0
            tf = work / (fms / 1e3) / 1e12
            kernels[f] = {"kernel": FAMILIES[f], "ms_per_step": round(fms, 3), "launches_per_step": n,
                          "avg_launch_ms": round(fms / n, 4), "algorithmic_flop_per_launch": work / n,
                          "achieved_tflops": round(tf, 2), "frac_of_fp32_peak": round(tf / FP32_MFMA_PEAK_TF, 4)}
        if kernels:
            dom = max(kernels, key=lambda f: kernels[f]["ms_per_step"])
            k = kernels[dom]
            roof = {"kernel": k["kernel"], "family": dom, "bound": "mfma", "achieved": k["achieved_tflops"],
                    "peak": FP32_MFMA_PEAK_TF, "unit": "TFLOP/s", "frac": k["frac_of_fp32_peak"],
                    "traffic": pmc_traffic(dom), "avg_launch_ms": k["avg_launch_ms"],
                    "launches_per_step": k["launches_per_step"],
                    "algorithmic_flop_per_launch": k["algorithmic_flop_per_launch"],
                    "peak_note": PEAK_NOTES.get(dom, "")}
    step_flop = (model_flops_per_frame(mc, args.ratio) + attn_flops_per_frame(mc, args.ratio, args.seq)) \
        * args.batch * args.seq
    out = {
        "metric": METRIC, "value": round(value, 2), "unit": "frames/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "fp32", "data": "synthetic",
        "config": {"workload": "lstmformer train step (fwd+Huber+bwd+AdamW), BASELINE configs[3]/[4]",
                   "model": "lstmformer H=256 blocks=5 enc_layers=5 heads=4 bottleneck=64 (13,052,678 params)",
                   "global_batch": args.batch * world, "seq_len": args.seq, "audio_ratio": args.ratio,
                   "parallelism": f"dp{world}", "hip_graph": bool(args.graph),
                   "wgrad_side_stream": bool(args.wgrad_stream)},
        "whole_step_roofline": {"bound": "mfma", "algorithmic_tflop_per_step": round(step_flop / 1e12, 4),
                                "achieved_tflops": round(step_flop / (ms / 1000.0) / 1e12, 3),
                                "peak": FP32_MFMA_PEAK_TF,
                                "frac": round(step_flop / (ms / 1000.0) / 1e12 / FP32_MFMA_PEAK_TF, 4)},
        "roofline": roof,
        "kernels": kernels,
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and args.cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(args, mc, oc)
        out["speedup_vs_cpu_baseline"] = round(out["value"] / out["cpu_baseline"]["value"], 1)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
