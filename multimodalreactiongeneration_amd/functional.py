"""Autograd functions of the MI355X path; every FLOP runs in libmrg.so (include/mrg.h).

torch is used for device memory (caching allocator), the current HIP stream
and the autograd graph only.  Parameter gradients are written straight into
``param.grad`` by the fused backward GEMMs (beta = 1 accumulation; the
functions return ``None`` for parameters), so a step needs no per-parameter
gradient copies and a flat gradient buffer (optim.FusedAdamW, ddp.GradReducer)
sees them in place.

Reference ops replaced (file:line in /root/reference):
  linear / FFN        nn.Linear + ReLU            mixer_block.py:37-87, lstm_block.py:88-96
  lstm                nn.LSTM (cuDNN RNN)         mixer_block.py:237-252, lstm_block.py:21-46,
                                                  lstm_sampler.py:16-34
  mha                 nn.MultiheadAttention       for_sequential.py:27-51, multi_modal_att.py:12-31
  residual_layernorm  ResidualConnection          residual_connection.py:20-37
  masked_loss         training_step / lossfun     lstmformer.py:313-325,372-380
"""
from __future__ import annotations

import contextlib
import ctypes
import functools
import math
import os
from typing import List, Optional, Sequence

import torch
from torch.autograd import Function

from . import _lib

F32 = 4
_ERR = {}
_CNT = {}

# --- optional live kernel timing (bench.py).  Default: HIP events recorded on the launch stream
# around each library call.  kernel=True: the library times every kernel of a tagged call with
# kernel-bound events (mrg_probe_*, hipExtLaunchKernelGGL), i.e. the kernels' own execution as
# rocprofv3 reports it, without the packet dispatch a stream event pair also holds.
_PROBE_ON = set()
_PROBES = {}
_NATIVE = [False]
_CALLS = []          # native mode: (name, work) per tagged library call
_PROBE_CAP = 1 << 15


class _probe:
    """Bracket one library launch with timing events when ``name`` is being probed.

    ``work``: the launch's algorithmic FLOPs (or bytes), kept with its time for rooflines."""
    __slots__ = ("name", "e0", "work", "tagged")

    def __init__(self, name, work=0.0):
        self.name = name
        self.e0 = None
        self.work = work
        self.tagged = False

    def __enter__(self):
        if self.name in _PROBE_ON:
            if _NATIVE[0]:
                _lib.load().mrg_probe_tag(len(_CALLS))
                _CALLS.append((self.name, self.work))
                self.tagged = True
            else:
                self.e0 = torch.cuda.Event(enable_timing=True)
                self.e0.record()
        return self

    def __exit__(self, *exc):
        if self.tagged:
            _lib.load().mrg_probe_tag(-1)
        elif self.e0 is not None:
            e1 = torch.cuda.Event(enable_timing=True)
            e1.record()
            _PROBES.setdefault(self.name, []).append((self.e0, e1, self.work))
        return False


def probe_start(*names, kernel=False):
    _PROBE_ON.clear()
    _PROBE_ON.update(names)
    _PROBES.clear()
    _CALLS.clear()
    _NATIVE[0] = bool(kernel)
    if kernel:
        _lib.check(_lib.load().mrg_probe_start(_PROBE_CAP), "probe start")


def probe_stop(with_work=False):
    """Stop probing; returns {name: [ms per launch]} or, with_work, {name: [(ms, work)]} (synchronises).
    In kernel mode a launch's ms is the sum of its kernels' own execution times."""
    _PROBE_ON.clear()
    torch.cuda.synchronize()
    if _NATIVE[0]:
        _NATIVE[0] = False
        ms = (ctypes.c_float * _PROBE_CAP)()
        tags = (ctypes.c_int * _PROBE_CAP)()
        n = _lib.load().mrg_probe_stop(ms, tags, _PROBE_CAP)
        if n < 0:
            raise RuntimeError(f"probe stop: {_lib.load().mrg_last_error().decode()}")
        per_call = [0.0] * len(_CALLS)
        for i in range(n):
            per_call[tags[i]] += ms[i]
        out = {}
        for (name, work), t in zip(_CALLS, per_call):
            out.setdefault(name, []).append((t, work) if with_work else t)
        _CALLS.clear()
        return out
    if with_work:
        out = {k: [(a.elapsed_time(b), w) for a, b, w in v] for k, v in _PROBES.items()}
    else:
        out = {k: [a.elapsed_time(b) for a, b, _ in v] for k, v in _PROBES.items()}
    _PROBES.clear()
    return out


def _ptr(t: Optional[torch.Tensor], elem_offset: int = 0):
    if t is None:
        return None
    return ctypes.c_void_p(t.data_ptr() + elem_offset * t.element_size())


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _ws(nbytes: int, device) -> torch.Tensor:
    t = torch.empty(max(1, (int(nbytes) + 3) // 4), dtype=torch.float32, device=device)
    _hold_if_side(t)
    return t


# MRG_SIDE_HOLD=0 turns the hold off (diagnostic only: tests/test_gpu_capture.py)
_HOLD_SIDE_SCRATCH = [os.environ.get("MRG_SIDE_HOLD", "1") == "1"]


def _hold_if_side(t: torch.Tensor):
    """A scratch tensor allocated on the weight-gradient side stream stays referenced until the
    backward's join (see _ensure_join).  Freed earlier, its block could go to an allocation on the
    main stream while the side-stream kernel that uses it has not run yet: inside a HIP-graph capture
    the private pool does not keep the two streams' blocks apart (measured: the encoder stack's
    replayed gradients were corrupted by split-K slabs reused as main-stream temporaries)."""
    if not (_SIDE and _HOLD_SIDE_SCRATCH[0]):
        return
    dev = t.device.index or 0
    s = _SIDE.get(dev)
    cur = torch.cuda.current_stream(t.device)
    if (s is not None and (cur == s or cur == _REC.get(dev)) and dev in _JOIN_PENDING
            and torch.cuda.is_current_stream_capturing()):
        _SIDE_HOLD.setdefault(dev, []).append(t)


def _counters(device) -> torch.Tensor:
    """Split-K tickets of the in-launch slab combine (mrg_gemm_f32_ex): zeroed once, every launch
    leaves them at zero again.  One buffer per (device, stream): launches on different streams
    (e.g. a weight-gradient product on the side stream) never share tickets."""
    key = (torch.device(device).index or 0, torch.cuda.current_stream(device).cuda_stream)
    if key not in _CNT:
        _CNT[key] = torch.zeros(4096, dtype=torch.int32, device=device)  # MRG_GEMM_COUNTERS
    return _CNT[key]


def _err_flag(device) -> torch.Tensor:
    key = torch.device(device).index or 0
    if key not in _ERR:
        _ERR[key] = torch.zeros(1, dtype=torch.int32, device=device)
    return _ERR[key]


def check_errors(device=None):
    """Synchronise and raise if a persistent kernel reported a hand-off timeout."""
    for k, t in _ERR.items():
        if device is not None and (torch.device(device).index or 0) != k:
            continue
        if int(t.item()) != 0:
            t.zero_()
            raise RuntimeError("libmrg: LSTM recurrence hand-off timed out (grid not co-resident?)")


# Gradient-ready listener (ddp.GradReducer with overlap): every parameter-gradient write goes
# through _gbuf() just before its launch, so a touched parameter is announced to the listener when
# the NEXT autograd Function's backward starts (every launch of the previous one is issued by then)
# or at the end of the backward pass.
_GRAD_LISTENER = [None]
_TOUCHED = []


def set_grad_listener(listener):
    """listener.ready(params) is called with parameters whose gradient writes have been issued
    (at most one autograd Function late); listener.end_of_backward() once per backward pass."""
    _GRAD_LISTENER[0] = listener
    _TOUCHED.clear()


def _flush_touched():
    lst = _GRAD_LISTENER[0]
    if lst is not None and _TOUCHED:
        ready = list(_TOUCHED)
        _TOUCHED.clear()
        lst.ready(ready)


def _gbuf(p: torch.Tensor) -> Optional[torch.Tensor]:
    """The tensor a parameter's gradient accumulates into (created zero-filled on first use)."""
    if p is None or not p.requires_grad:
        return None
    if p.grad is None:
        p.grad = torch.zeros_like(p)
    if _GRAD_LISTENER[0] is not None:
        _GRAD_LISTENER[0].touch()
        _TOUCHED.append(p)
    return p.grad


# --- compute precision (mixed-precision configs, BASELINE configs[1] "bf16"): None = fp32 arithmetic
# (the library's GEMM mode: x6 split or exact f32), "bf16" = GEMM operands rounded to bf16 with fp32
# accumulation (mrg_gemm_bf16_ex).  Set by the model's forward; every autograd Function records it in
# forward and restores it around its backward (which runs on autograd's thread, after the context).
_ARITH = [None]
PRECISIONS = {None: None, "32": None, 32: None, "fp32": None, "32-true": None,
              "bf16": "bf16", "bf16-mixed": "bf16", "bf16-true": "bf16"}


@contextlib.contextmanager
def precision(p):
    """Compute precision of the enclosed ops: '32'/'fp32' or 'bf16'/'bf16-mixed' (Lightning names)."""
    if p not in PRECISIONS:
        raise ValueError(f"unsupported precision {p!r} (one of {sorted(map(str, PRECISIONS))})")
    prev = _ARITH[0]
    _ARITH[0] = PRECISIONS[p]
    try:
        yield
    finally:
        _ARITH[0] = prev


def _keeps_precision(fn):
    """Decorator for autograd Function forward/backward: forward records the active precision in ctx,
    backward runs under it."""
    @functools.wraps(fn)
    def wrapper(ctx, *args):
        if fn.__name__ == "forward":
            ctx.arith = _ARITH[0]
            return fn(ctx, *args)
        _flush_touched()  # the previous Function's gradient writes are all issued
        prev = _ARITH[0]
        _ARITH[0] = getattr(ctx, "arith", None)
        try:
            return fn(ctx, *args)
        finally:
            _ARITH[0] = prev
    return wrapper


def gemm(M, N, K, A, transA, lda, B, transB, ldb, C, ldc, *, alpha=1.0, beta=0.0, bias=None,
         epi=0, aux=None, ldaux=0, a_hi=0, a_div=0, b_hi=0, b_div=0, splits=1, device=None,
         asum_out=None, asum_out2=None, asum_beta=1.0):
    """C = epi(alpha op(A) op(B) + beta C + bias); A/B/C/bias/aux are ctypes pointers.

    asum_out (optional ctypes pointer): += row sums of op(A) over k, i.e. the bias gradient of a
    weight-gradient GEMM dY^T X, fused into the GEMM (mrg_gemm_f32_ex)."""
    if M == 0 or N == 0:
        return
    lib = _lib.load()
    if splits == 1 and not transA:
        splits = act_splits(M, N, K)
    ws = None
    if splits > 1 or asum_out is not None:
        ws = _ws(lib.mrg_gemm_workspace_bytes(M, N, splits), device)
    fn = lib.mrg_gemm_bf16_ex if _ARITH[0] == "bf16" else lib.mrg_gemm_f32_ex
    with _probe("gemm", 2.0 * M * N * K):
        rc = fn(M, N, K, alpha, A, transA, lda, a_hi, a_div, B, transB, ldb, b_hi, b_div,
                                 beta, C, ldc, bias, epi, aux, ldaux, _ptr(ws), splits, asum_out, asum_out2,
                                 asum_beta, _ptr(_counters(device)) if splits > 1 else None, _stream())
    _lib.check(rc, "gemm")


def act_splits(M, N, K):
    """split-K factor for activation products with few output tiles (65..~2000 rows): a handful of
    64x64 tiles walking K >= 512 is latency-bound, so spread K over the CUs."""
    tiles = ((M + 63) // 64) * ((N + 63) // 64)
    if M <= 64 or tiles >= 64 or K < 512 or (_lib.load().mrg_gemm_get_mode() != 1 and _ARITH[0] is None):
        return 1  # M <= 64: the few-row kernel (gemm_rows_kernel) needs no split
    # <= 4 slices of 64x64 tiles: the slabs (<= 64 KB per tile) are combined in-launch
    return int(max(1, min(4, K // 64, 128 // tiles)))


# Workgroups a weight-gradient product aims at.  256 (half the split-K slices of round 2's 512): most
# products run beside a recurrence with the grid capped at one block per CU (_DEFER), where fewer
# slices measured faster (tools/tools_wgrad_sweep.py, capped grid: LSTM dW 1024 x 256 102 -> 98 us at
# 16 instead of 32 slices, 256 x 256 41 -> 36 us at 64 instead of 128, 512 x 256 62 -> 55 us at 32
# instead of 64) and the slab reduce reads half the slabs: 22.93 -> 22.48 ms/step on one box (128:
# 23.7).  One target for every schedule, so the split (and the summation order) depends on the shape
# only and the side-stream / deferred schedules stay bitwise equal to the single-stream one.
_WG_TARGET = int(os.environ.get("MRG_WGRAD_TARGET_WG", "256"))


def wgrad_splits(M, N, K):
    """split-K factor for weight-gradient GEMMs (small M x N output, long B*T reduction).

    About _WG_TARGET workgroups: 128x128 tiles under the x6 arithmetic (chunks of >= 128 rows),
    64x64 tiles under exact f32 (chunks of >= 256 rows); tools/tools_gemm_sweep.py measured both.
    """
    if _lib.load().mrg_gemm_get_mode() == 1 or _ARITH[0] == "bf16":
        tiles = ((M + 127) // 128) * ((N + 127) // 128)
        s = max(1, _WG_TARGET // max(1, tiles))
        return int(max(1, min(s, K // 128, 128)))
    tiles = ((M + 63) // 64) * ((N + 63) // 64)
    s = max(1, 512 // max(1, tiles))
    return int(max(1, min(s, K // 256, 64)))


def colsum(rows, N, X, ld, out, *, out2=None, beta=1.0, ld_hi=0, rdiv=0, device=None):
    if N == 0:
        return
    lib = _lib.load()
    ws = _ws(lib.mrg_colsum_workspace_bytes(rows, N), device)
    _lib.check(lib.mrg_colsum_f32(rows, N, X, ld, ld_hi, rdiv, beta, out, out2, _ptr(ws), _stream()),
               "colsum")


# --- weight gradients on a side stream
# Parameter gradients are consumed only by the optimizer / all-reduce, so the weight-gradient
# GEMMs (dW = dY^T X, fused bias sums) leave the backward's critical path: they run on one side
# stream per device, forked from the current stream when their operands are ready and joined back
# at the end of the backward pass (an autograd final callback), so `loss.backward()` returns with
# every gradient ordered before anything the caller issues next (graph capture included).  Their
# operands are record_stream'ed so the caching allocator does not recycle them early.  Products
# over fewer than _SIDE_MIN_ROWS rows (the T = 1 decode steps of the autoregressive loops, where
# a fork/join per frame costs more than it hides: C3 scheduled sampling 80 -> 130 ms measured)
# stay on the current stream; if the side stream already has work in this backward pass, the
# current stream first waits for it, so the writes into any one gradient buffer stay in order.
# MRG_WGRAD_STREAM=0 (or set_wgrad_stream(False)) issues everything on the current stream.
_WGRAD_SIDE = [os.environ.get("MRG_WGRAD_STREAM", "1") != "0"]
_SIDE_MIN_ROWS = 2048
_SIDE = {}
_SIDE_HOLD = {}   # device -> side-stream scratch tensors kept alive until the join (_hold_if_side)
# device -> autograd graph-task id whose final callback will join the side stream back.  Keyed by
# the task (torch._C._current_graph_task_id), not a bare flag: a backward that raised after a fork
# never ran its callback, and a stale flag would make every later backward skip the join.
_JOIN_PENDING = {}


def set_wgrad_stream(on: bool) -> bool:
    """Enable / disable side-stream weight gradients; returns the previous setting."""
    prev = _WGRAD_SIDE[0]
    _WGRAD_SIDE[0] = bool(on)
    return prev


# Deferred weight gradients (on by default, MRG_WGRAD_DEFER=0 turns it off; neutral in round 2, -0.34 ms/step
# with round 3's encoder wavefront, whose MFMA recurrences leave room on every CU): a side-stream product is not issued
# when its operands are ready but queued until the backward reaches its next persistent recurrence
# (_LSTMFn.backward marks the current stream right before mrg_lstm_bwd and issues the queue right
# after it, ordered after the mark only: fork_beside_recurrence / flush_beside_recurrence), on the
# side stream with the GEMM grids capped at one block per CU while the recurrence runs at one
# workgroup per CU (mrg_lstm_set_blocks_per_cu): the latency-bound recurrence leaves most of each
# CU idle, and the dW products fill it instead of running beside the dX chain's GEMMs (which
# already fill the GPU).  The end-of-backward join issues whatever is still queued.  Queue order is
# side-stream order, so the writes into each gradient buffer keep their order; a write issued on the
# current stream (fewer than _SIDE_MIN_ROWS rows) first flushes the queue.  Not used while a
# gradient-ready listener (DDP bucket overlap) needs each write issued when it is reported.
_DEFER = [os.environ.get("MRG_WGRAD_DEFER", "1") == "1"]
_PENDING = {}
# The queue flushed beside the recurrences runs on a stream of its own (_REC), the rest of the side
# work (the end-of-backward flush: the products of the layers below the last recurrence) on _SIDE, so
# that flush starts when its operands are ready instead of behind the recurrence stream's backlog
# (in-graph wall-clock stamps, tools/side_timing.py: that backlog outlasts the main stream by ~1.7 ms;
# headline 20.55 -> 20.23 ms, A/B on one box).  Writes into one gradient buffer stay ordered: every
# queued item names the buffers it writes (_on_side(writes=...)), and a flush on _SIDE whose items
# touch a buffer the recurrence stream has written in this backward, or name none, waits for it
# first.  MRG_REC_STREAM=0 keeps everything on _SIDE.
_REC_ON = [os.environ.get("MRG_REC_STREAM", "1") != "0"]
_REC = {}          # device -> the recurrence-beside stream
_REC_USED = {}     # device -> True once it has work in this backward
_REC_WRITES = {}   # device -> {(ptr, nbytes)} written on it in this backward (None: unknown)


def set_wgrad_defer(on: bool) -> bool:
    """Enable / disable deferring side-stream weight gradients to the next recurrence; returns the old value."""
    prev = _DEFER[0]
    _DEFER[0] = bool(on)
    return prev


# --- fork points under capture.  Measured (round 4, tools/tools_fork_variants.py, tools_fork_race.py):
# several side-stream forks from ONE point of the main stream (no main-stream node between them, e.g.
# one fork per weight-gradient product) capture into a graph whose edges are exactly the streams'
# order (tools/tools_capture_dot.py + tools_dot_deps.py), with no cross-stream address reuse
# (tools/tools_capture_alias.py) and no hand-off timeout, and the eager step is bitwise right with
# either stream delayed; yet its replay gives wrong gradients, deterministically, unless the HIP graph
# executor runs on one queue (DEBUG_HIP_FORCE_GRAPH_QUEUES=1) or a main-stream node separates the forks.
# So the executor mis-orders that topology (each fork's first side node has two predecessors: the
# same main node again and the previous side node).  The guard: a fork from the main-stream point
# the side stream already waited on adds no second wait (the side stream is ordered after that point
# already), so the redundant edges are never captured.
_HIP_CAPINFO = [None]
_LAST_FORK = {}   # device -> the capture point (capture id, main-stream dependency nodes) of the last fork
_FORK_GUARD = [os.environ.get("MRG_FORK_GUARD", "1") != "0"]   # 0: diagnostics only (tools_fork_variants.py)


def _capture_point(stream):
    """(capture id, the stream's current dependency node handles) while `stream` is capturing, else None."""
    if _HIP_CAPINFO[0] is None:
        f = ctypes.CDLL("libamdhip64.so").hipStreamGetCaptureInfo_v2
        f.restype = ctypes.c_int
        f.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_ulonglong),
                      ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.POINTER(ctypes.c_void_p)),
                      ctypes.POINTER(ctypes.c_size_t)]
        _HIP_CAPINFO[0] = f
    st, cid, graph = ctypes.c_int(0), ctypes.c_ulonglong(0), ctypes.c_void_p()
    deps, n = ctypes.POINTER(ctypes.c_void_p)(), ctypes.c_size_t(0)
    rc = _HIP_CAPINFO[0](ctypes.c_void_p(stream.cuda_stream), ctypes.byref(st), ctypes.byref(cid),
                         ctypes.byref(graph), ctypes.byref(deps), ctypes.byref(n))
    if rc != 0 or st.value != 1:   # hipStreamCaptureStatusActive
        return None
    return (cid.value,) + tuple(deps[i] for i in range(n.value))


def _fork(key, s, cur):
    """s.wait_stream(cur), skipped under capture when s already waited on cur's current point."""
    point = _capture_point(cur) if _FORK_GUARD[0] and torch.cuda.is_current_stream_capturing() else None
    if point is None or _LAST_FORK.get(key) != (point, s.cuda_stream):
        s.wait_stream(cur)
    _LAST_FORK[key] = None if point is None else (point, s.cuda_stream)


def reset_fork_point(key=None):
    """Forget the recorded fork point (all devices when key is None): called wherever the main and side
    streams are joined or ordered outside _fork, and at the end of every capture (graphs.capture), so
    the guard only ever skips a wait that an earlier _fork of the same capture really issued."""
    if key is None:
        _LAST_FORK.clear()
    else:
        _LAST_FORK.pop(key, None)


def _ensure_join(key, cur, s, task):
    if key not in _JOIN_PENDING:
        def join(cur=cur, s=s, key=key):
            _flush_deferred(key, cur.device)
            cur.wait_stream(s)
            if _REC_USED.pop(key, False):
                cur.wait_stream(_REC[key])
            _REC_WRITES.pop(key, None)
            reset_fork_point(key)
            _JOIN_PENDING.pop(key, None)
            _SIDE_HOLD.pop(key, None)   # their blocks are reusable now: later work is ordered after the wait
        torch.autograd.Variable._execution_engine.queue_callback(join)
        _JOIN_PENDING[key] = task


def _defers(device, rows) -> bool:
    return (_WGRAD_SIDE[0] and _DEFER[0] and rows >= _SIDE_MIN_ROWS and _GRAD_LISTENER[0] is None
            and torch._C._current_graph_task_id() >= 0)


def _flush_deferred(key, device, cap=0, after=None):
    """Issue the queued weight-gradient products on the side stream (GEMM grids capped at `cap`
    blocks per CU while they run beside a recurrence), ordered after event `after` when given, else
    after the current stream's work so far."""
    items = _PENDING.pop(key, None)
    if not items:
        return
    dev = torch.device(device)
    cur = torch.cuda.current_stream(dev)
    s = _SIDE[key]
    if _REC_ON[0] and after is not None:
        s = _REC.get(key)
        if s is None:
            s = _REC[key] = torch.cuda.Stream(device=dev)
        _REC_USED[key] = True
        w = _REC_WRITES.setdefault(key, set())
        for _, _, _, writes in items:
            if writes is None or w is None:
                _REC_WRITES[key] = w = None
            else:
                w.update(writes)
        s.wait_event(after)
    else:
        if _REC_USED.get(key) and _conflicts(items, _REC_WRITES.get(key, set())):
            s.wait_stream(_REC[key])   # same gradient buffers (or unknown): keep their write order
        if after is None:
            _fork(key, s, cur)
        else:
            s.wait_event(after)
            _LAST_FORK[key] = None
    lib = _lib.load()
    prev = lib.mrg_gemm_set_blocks_per_cu(cap) if cap else None
    try:
        with torch.cuda.stream(s):
            for fn, keep, arith, _ in items:
                for t in keep:
                    if t is not None:
                        t.record_stream(s)
                old = _ARITH[0]
                _ARITH[0] = arith
                try:
                    fn()
                finally:
                    _ARITH[0] = old
    finally:
        if cap:
            lib.mrg_gemm_set_blocks_per_cu(prev)


def fork_beside_recurrence(device):
    """Called right before a backward recurrence launch: returns (the recurrence's workgroups-per-CU
    cap: 1 when deferring, else 0; a fork mark for flush_beside_recurrence, or None)."""
    if not (_WGRAD_SIDE[0] and _DEFER[0] and _GRAD_LISTENER[0] is None):
        return 0, None
    dev = torch.device(device)
    if not _PENDING.get(dev.index or 0):
        return 1, None
    mark = torch.cuda.Event()
    mark.record(torch.cuda.current_stream(dev))
    return 1, mark


def flush_beside_recurrence(device, mark) -> None:
    """Called right after the recurrence launch: issues the queued weight-gradient products on the side
    stream, ordered after `mark` (the work before the recurrence) but not after the recurrence.
    Measured (r03, headline step, graph replay): issued BEFORE the recurrence launch the products were
    dispatched first and delayed its start (23.06 ms/step); issued after it, 21.80.  Joining the main
    stream to them right after (so they must finish beside this recurrence) measured 23.6: the
    recurrence runs ~25 % slower beside them and they outlast it, so the join is left to the end of
    the backward and the executor places them where the main stream leaves room."""
    if mark is None:
        return
    _flush_deferred(torch.device(device).index or 0, device, cap=1, after=mark)


def _writes(tensors):
    """{(data_ptr, nbytes)} of the gradient buffers an item writes (None entries skipped)."""
    return {(t.data_ptr(), t.numel() * t.element_size()) for t in tensors if t is not None}


def _conflicts(items, rec_writes) -> bool:
    """True when an item of a flush writes a buffer the recurrence stream wrote (or either is unknown)."""
    if rec_writes is None:
        return True
    for _, _, _, writes in items:
        if writes is None:
            return True
        for p, n in writes:
            for q, m in rec_writes:
                if p < q + m and q < p + n:
                    return True
    return False


def _on_side(device, rows, keep, fn, writes=None):
    """Run fn() (weight-gradient launches) on the side stream now, or queue it (see _DEFER).
    writes: the gradient tensors fn writes (ordering across the two side streams), None = unknown."""
    if not _defers(device, rows):
        with _side(device, rows, keep):
            fn()
        return
    dev = torch.device(device)
    key = dev.index or 0
    cur = torch.cuda.current_stream(dev)
    task = torch._C._current_graph_task_id()
    if key in _JOIN_PENDING and _JOIN_PENDING[key] != task:
        _flush_deferred(key, dev)
        cur.wait_stream(_SIDE[key])
        if _REC_USED.pop(key, False):
            cur.wait_stream(_REC[key])
        _REC_WRITES.pop(key, None)
        reset_fork_point(key)
        del _JOIN_PENDING[key]
    s = _SIDE.get(key)
    if s is None:
        s = _SIDE[key] = torch.cuda.Stream(device=dev)
    _ensure_join(key, cur, s, task)
    _PENDING.setdefault(key, []).append((fn, tuple(keep), _ARITH[0], None if writes is None else _writes(writes)))


class _side:
    """Issue the enclosed launches on the device's weight-gradient stream (see above)."""
    __slots__ = ("dev", "rows", "keep", "ctx")

    def __init__(self, device, rows, keep=()):
        self.dev, self.rows, self.keep, self.ctx = device, rows, keep, None

    def __enter__(self):
        if not _WGRAD_SIDE[0]:
            return self
        dev = torch.device(self.dev)
        key = dev.index or 0
        cur = torch.cuda.current_stream(dev)
        task = torch._C._current_graph_task_id()
        s = _SIDE.get(key)
        if key in _JOIN_PENDING and _JOIN_PENDING[key] != task:
            # left over from a backward that did not finish: order after its side-stream work
            _flush_deferred(key, dev)
            cur.wait_stream(s)
            if _REC_USED.pop(key, False):
                cur.wait_stream(_REC[key])
            _REC_WRITES.pop(key, None)
            reset_fork_point(key)
            del _JOIN_PENDING[key]
        if self.rows < _SIDE_MIN_ROWS:
            if key in _JOIN_PENDING:  # order this write after the side streams' pending ones
                _flush_deferred(key, dev)
                cur.wait_stream(s)
                if _REC_USED.get(key):
                    cur.wait_stream(_REC[key])
                reset_fork_point(key)
            return self
        if task < 0:  # not inside a backward pass: stay on the current stream
            return self
        if s is None:
            s = _SIDE[key] = torch.cuda.Stream(device=dev)
        _ensure_join(key, cur, s, task)
        _fork(key, s, cur)
        for t in self.keep:
            if t is not None:
                t.record_stream(s)
        self.ctx = torch.cuda.stream(s)
        self.ctx.__enter__()
        return self

    def __exit__(self, *exc):
        if self.ctx is not None:
            self.ctx.__exit__(*exc)
        return False


def _wgrad(dY, ldy, X, ldx, rows, Nout, Nin, gw, device, *, dy_hi=0, dy_div=0, x_hi=0, x_div=0, gb=None,
           gb2=None, keep=()):
    """gw[Nout, Nin] += sum_rows dY[row, :]^T X[row, :]; gb (and gb2) += sum_rows dY[row, :] (fused).

    keep: the tensors behind the dY / X pointers (side-stream lifetime, see _side)."""
    def issue():
        if gw is None:
            if gb is not None:
                colsum(rows, Nout, dY, ldy, _ptr(gb), out2=_ptr(gb2), ld_hi=dy_hi, rdiv=dy_div, device=device)
            return
        gemm(Nout, Nin, rows, dY, 1, ldy, X, 0, ldx, _ptr(gw), Nin, beta=1.0, a_hi=dy_hi, a_div=dy_div,
             b_hi=x_hi, b_div=x_div, splits=wgrad_splits(Nout, Nin, rows), device=device,
             asum_out=_ptr(gb), asum_out2=_ptr(gb2))
    _on_side(device, rows, keep, issue, writes=(gw, gb, gb2))


# --- [in][out] weight copies for the input-gradient products.  dX = dY W reads W [out][in] along
# n (not k): the product runs as a k-contiguous one, dY (W^T)^T, on the LDS-DMA x6 kernel
# (gemm_glds.hip) when the weight's transposed copy exists.  The forwards note the weights of their
# large products (>= _WT_MIN_ROWS rows, >= 256 inputs); the backward's first use transposes every
# noted weight in ONE launch (mrg_transpose_batched) and later uses hit the cache.  A weight noted
# again (the next step's forward: the optimizer has rewritten it in place) drops its stale copy.
# MRG_DX_TRANSPOSED=0 keeps the [out][in] operand (the register-staged kernel's n-contiguous path).
_WT_ON = [os.environ.get("MRG_DX_TRANSPOSED", "1") != "0"]
_WT_MIN_ROWS = 2048
_WT_PENDING = {}
_WT_CACHE = {}


def set_dx_transposed(on: bool) -> bool:
    prev = _WT_ON[0]
    _WT_ON[0] = bool(on)
    return prev


def _wt_key(w):
    return (w.data_ptr(), tuple(w.shape))


def _wt_note(w, rows, need=True):
    """Forward side (inside autograd Function.forward: pass ctx.needs_input_grad of the input): w
    [out][in] (a contiguous 2-D view) will serve a dX product over `rows` rows."""
    if not (need and _WT_ON[0] and rows >= _WT_MIN_ROWS and w.shape[1] >= 256 and w.shape[0] % 32 == 0
            and w.is_contiguous()) or _plane_operand(w, True) is not None:
        return
    k = _wt_key(w)
    _WT_CACHE.pop(k, None)
    _WT_PENDING[k] = w


def _wt(w):
    """Backward side: the [in][out] copy of w, or None when w was not noted in this step's forward.
    Copies are valid only within the backward pass (autograd graph task) that made them: a copy keyed
    by a pointer that a later model reuses, or made before an optimizer step, is never handed out."""
    k = _wt_key(w)
    task = torch._C._current_graph_task_id()
    t = _WT_CACHE.get(k)
    if t is not None and t[0] == task:
        return t[1]
    if k not in _WT_PENDING:
        return None
    items = list(_WT_PENDING.values())
    _WT_PENDING.clear()
    outs = [torch.empty(x.shape[1], x.shape[0], device=x.device, dtype=torch.float32) for x in items]
    n = len(items)
    VP = ctypes.c_void_p
    _lib.check(_lib.load().mrg_transpose_batched(
        n, (VP * n)(*[_ptr(x) for x in items]), (VP * n)(*[_ptr(o) for o in outs]),
        (ctypes.c_int * n)(*[x.shape[0] for x in items]), (ctypes.c_int * n)(*[x.shape[1] for x in items]),
        _stream()), "transpose")
    for x, o in zip(items, outs):
        _WT_CACHE[_wt_key(x)] = (task, o)
    return _WT_CACHE[k][1]


# --- pre-split weights: the three bf16 planes of every weight (and of its transpose), made once per
# optimizer step in ONE launch (mrg_split_planes_batched) by prepare_weight_planes at the start of a
# training forward; the forward products x W^T and the input-gradient products dY W then run on the
# LDS-DMA x6 kernel with only the activation operand split in the loop (mrg_gemm_x6_planes).  Keyed
# by the weight's storage; a row slice of a prepared weight (the Q / K,V blocks of in_proj_weight)
# resolves to its parent's planes.  On by default (MRG_WEIGHT_PLANES=0 / set_weight_planes(False) turns
# it off): with the row-owning kernel (gemm_wide.hip) and the batched plane products the headline step
# is 0.55 ms faster with it (21.10 -> 20.55 ms, A/B on one box).
_PL_ON = [os.environ.get("MRG_WEIGHT_PLANES", "1") == "1"]
_PLANES = {}


def set_weight_planes(on: bool) -> bool:
    prev = _PL_ON[0]
    _PL_ON[0] = bool(on)
    if not on:
        _PLANES.clear()
    return prev


def invalidate_weight_planes():
    """The weights changed (optimizer step): forget their planes and their [in][out] copies (_WT_CACHE)
    until the next forward notes them again, so no backward can use a transpose of old weights."""
    _PLANES.clear()
    _WT_CACHE.clear()
    _WT_PENDING.clear()


def prepare_weight_planes(weights):
    """Split every 2-D fp32 weight (rows and cols multiples of 32... any size) into bf16 planes, both
    orientations, in one launch.  Called per step before the forward (the optimizer rewrote them)."""
    _PLANES.clear()
    if not (_PL_ON[0] and _ARITH[0] is None and _lib.load().mrg_gemm_get_mode() == 1):
        return
    ws = [w for w in weights if w.dim() == 2 and w.is_cuda and w.dtype == torch.float32 and w.is_contiguous()
          and min(w.shape) >= 32]
    if not ws:
        return
    srcs, dsts, rows, cols, trs = [], [], [], [], []
    for w in ws:
        O, I = w.shape
        pw = torch.empty(3, O, I, device=w.device, dtype=torch.int16)
        pt = torch.empty(3, I, O, device=w.device, dtype=torch.int16)
        _PLANES[w.data_ptr()] = (w, pw, pt, w._version)
        for dst, tr in ((pw, 0), (pt, 1)):
            srcs.append(_ptr(w)); dsts.append(_ptr(dst)); rows.append(O); cols.append(I); trs.append(tr)
    n = len(srcs)
    VP, CI = ctypes.c_void_p, ctypes.c_int
    _lib.check(_lib.load().mrg_split_planes_batched(n, (VP * n)(*srcs), (VP * n)(*dsts), (CI * n)(*rows),
                                                    (CI * n)(*cols), (CI * n)(*trs), _stream()), "split planes")


def _plane_operand(w, transposed):
    """(pointer, ldb, plane stride) of the planes of w (or of w^T), w a prepared weight or a row slice
    of one; None when w has no planes."""
    if not _PLANES:
        return None
    ent = _PLANES.get(w.data_ptr())
    r0 = 0
    if ent is None or ent[0].shape[1] != w.shape[1]:
        ent = None
        for cand in _PLANES.values():
            par = cand[0]
            off = w.data_ptr() - par.data_ptr()
            if par.shape[1] == w.shape[1] and 0 <= off < par.numel() * 4 and off % (4 * par.shape[1]) == 0:
                ent, r0 = cand, off // (4 * par.shape[1])
                break
        if ent is None:
            return None
    par, pw, pt, ver = ent
    if par._version != ver:   # rewritten through torch since the split: stale
        return None
    O, I = par.shape
    if not transposed:   # rows r0.. of W: [rows][I]
        return ctypes.c_void_p(pw.data_ptr() + 2 * r0 * I), I, O * I
    return ctypes.c_void_p(pt.data_ptr() + 2 * r0), O, I * O   # columns r0.. of W^T: [I][O]


def _planes_gemm(M, N, K, A, lda, planes, C, ldc, *, beta=0.0, bias=None, epi=0, aux=None, ldaux=0, a_hi=0,
                 a_div=0, device=None):
    bp, ldb, bplane = planes
    with _probe("gemm", 2.0 * M * N * K):
        rc = _lib.load().mrg_gemm_x6_planes(M, N, K, 1.0, A, lda, a_hi, a_div, bp, ldb, bplane, beta, C, ldc, bias,
                                           epi, aux, ldaux, _stream())
    _lib.check(rc, "gemm (weight planes)")


def planes_batched(M, N, K, items, lda, ldc, *, epi=0, ldaux=0, beta=0.0, transposed=False):
    """Same-shape products C_p = epi(A_p w_p^T ...) (transposed: dY_p w_p, on the planes of w_p^T) in ONE
    launch on the weights' pre-split planes (mrg_gemm_x6_planes_batched); items = [(A ptr, w, C ptr,
    bias ptr | None, aux ptr | None)].  Returns False (nothing launched) when a weight has no planes
    or the planes' strides differ, so the caller takes its fp32-operand path."""
    if not (M >= _WT_MIN_ROWS and K % 32 == 0 and _ARITH[0] is None and 0 < len(items) <= 16):
        return False
    pls = [_plane_operand(w, transposed) for _, w, _, _, _ in items]
    if any(p is None for p in pls) or len({(p[1], p[2]) for p in pls}) != 1:
        return False
    n, VP = len(items), ctypes.c_void_p
    arr = lambda xs: (VP * n)(*xs)  # noqa: E731
    with _probe("gemm", 2.0 * M * N * K * n):
        rc = _lib.load().mrg_gemm_x6_planes_batched(
            n, M, N, K, 1.0, arr([it[0] for it in items]), lda, arr([p[0] for p in pls]), pls[0][1], pls[0][2], beta,
            arr([it[2] for it in items]), ldc, None if all(it[3] is None for it in items) else arr([it[3] for it in items]),
            epi, None if all(it[4] is None for it in items) else arr([it[4] for it in items]), ldaux, _stream())
    _lib.check(rc, "batched gemm (weight planes)")
    return True


def _fwd_gemm(M, N, K, A, lda, w, C, ldc, **kw):
    """C[M, N] = epi(A[M, K] w[N, K]^T ...): on the weight planes when w has them."""
    pl = _plane_operand(w, False) if (M >= _WT_MIN_ROWS and K % 32 == 0 and _ARITH[0] is None) else None
    if pl is not None:
        kw.pop("device", None)
        _planes_gemm(M, N, K, A, lda, pl, C, ldc, **kw)
    else:
        gemm(M, N, K, A, 0, lda, _ptr(w), 1, K, C, ldc, **kw)


def _dx_gemm(M, In, N, dY, ldy, w, dx, ldx, **kw):
    """dx[M, In] = epi(dY[M, N] w[N, In] ...): on the planes of w^T, else through w's [in][out] copy
    when one exists, else reading w along n."""
    if M >= _WT_MIN_ROWS and N % 32 == 0 and _ARITH[0] is None:
        pl = _plane_operand(w, True)
        if pl is not None:
            kw.pop("device", None)
            _planes_gemm(M, In, N, dY, ldy, pl, dx, ldx, **kw)
            return
    wt = _wt(w) if M >= _WT_MIN_ROWS else None
    if wt is not None:
        gemm(M, In, N, dY, 0, ldy, _ptr(wt), 1, N, dx, ldx, **kw)
    else:
        gemm(M, In, N, dY, 0, ldy, _ptr(w), 0, In, dx, ldx, **kw)


# ------------------------------------------------------------------ Linear
class _LinearFn(Function):
    @staticmethod
    @_keeps_precision
    def forward(ctx, x, w, b):
        _lib.require_device(x)
        In, N = w.shape[1], w.shape[0]
        x2 = x.reshape(-1, In).contiguous()
        M = x2.shape[0]
        y = torch.empty(M, N, device=x.device, dtype=torch.float32)
        _fwd_gemm(M, N, In, _ptr(x2), In, w, _ptr(y), N, bias=_ptr(b), device=x.device)
        _wt_note(w, M, ctx.needs_input_grad[0])
        ctx.save_for_backward(x2, w, b)
        ctx.xshape = x.shape
        return y.view(*x.shape[:-1], N)

    @staticmethod
    @_keeps_precision
    def backward(ctx, dy):
        x2, w, b = ctx.saved_tensors
        N, In = w.shape
        dy2 = dy.reshape(-1, N).contiguous()
        M = dy2.shape[0]
        dev = dy.device
        _wgrad(_ptr(dy2), N, _ptr(x2), In, M, N, In, _gbuf(w), dev, gb=_gbuf(b), keep=(dy2, x2))
        dx = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty(M, In, device=dev, dtype=torch.float32)
            _dx_gemm(M, In, N, _ptr(dy2), N, w, _ptr(dx), In, device=dev)
            dx = dx.view(ctx.xshape)
        return dx, None, None


def linear(x, weight, bias=None):
    return _LinearFn.apply(x, weight, bias)


# ------------------------------------------------------------------ FFN (Linear -> ReLU -> Linear)
# Test hook (None in the product path): when a dict, every FFN forward stores the ReLU's side per
# element, {w1.data_ptr(): bool [..., Hb] (pre-activation > 0)}, so a test can evaluate the float64
# oracle at exactly this forward's kinks (oracle.RELU_MASKS; tests/test_gpu_models.py).
RELU_TAP = None


def _tap_relu(w1, h, lead_shape):
    if RELU_TAP is not None:
        RELU_TAP[w1.data_ptr()] = (h > 0).view(*lead_shape, h.shape[-1])


class _FFNFn(Function):
    @staticmethod
    @_keeps_precision
    def forward(ctx, x, w1, b1, w2, b2):
        _lib.require_device(x)
        In, Hb, N = w1.shape[1], w1.shape[0], w2.shape[0]
        x2 = x.reshape(-1, In).contiguous()
        M = x2.shape[0]
        dev = x.device
        h = torch.empty(M, Hb, device=dev, dtype=torch.float32)
        gemm(M, Hb, In, _ptr(x2), 0, In, _ptr(w1), 1, In, _ptr(h), Hb, bias=_ptr(b1), epi=1, device=dev)
        z = torch.empty(M, N, device=dev, dtype=torch.float32)
        _fwd_gemm(M, N, Hb, _ptr(h), Hb, w2, _ptr(z), N, bias=_ptr(b2), device=dev)
        _wt_note(w1, M, ctx.needs_input_grad[0])
        _tap_relu(w1, h, x.shape[:-1])
        ctx.save_for_backward(x2, h, w1, b1, w2, b2)
        ctx.xshape = x.shape
        return z.view(*x.shape[:-1], N)

    @staticmethod
    @_keeps_precision
    def backward(ctx, dz):
        x2, h, w1, b1, w2, b2 = ctx.saved_tensors
        Hb, In = w1.shape
        N = w2.shape[0]
        dz2 = dz.reshape(-1, N).contiguous()
        M = dz2.shape[0]
        dev = dz.device
        # d(pre-activation) = (dz W2) * (h > 0): relu backward fused into the GEMM epilogue
        dh = torch.empty(M, Hb, device=dev, dtype=torch.float32)
        gemm(M, Hb, N, _ptr(dz2), 0, N, _ptr(w2), 0, Hb, _ptr(dh), Hb, epi=2, aux=_ptr(h), ldaux=Hb,
             device=dev)
        _wgrad(_ptr(dz2), N, _ptr(h), Hb, M, N, Hb, _gbuf(w2), dev, gb=_gbuf(b2), keep=(dz2, h))
        _wgrad(_ptr(dh), Hb, _ptr(x2), In, M, Hb, In, _gbuf(w1), dev, gb=_gbuf(b1), keep=(dh, x2))
        dx = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty(M, In, device=dev, dtype=torch.float32)
            _dx_gemm(M, In, Hb, _ptr(dh), Hb, w1, _ptr(dx), In, device=dev)
            dx = dx.view(ctx.xshape)
        return dx, None, None, None, None


def ffn(x, w1, b1, w2, b2):
    return _FFNFn.apply(x, w1, b1, w2, b2)


# ------------------------------------------------------------------ residual + LayerNorm
class _ResLNFn(Function):
    @staticmethod
    @_keeps_precision
    def forward(ctx, a, b, gamma, beta, eps):
        _lib.require_device(a)
        E = a.shape[-1]
        a2 = a.reshape(-1, E).contiguous()
        b2 = b.reshape(-1, E).contiguous()
        rows = a2.shape[0]
        dev = a.device
        y = torch.empty_like(a2)
        mean = torch.empty(rows, device=dev, dtype=torch.float32)
        rstd = torch.empty(rows, device=dev, dtype=torch.float32)
        _lib.check(_lib.load().mrg_residual_layernorm_fwd(rows, E, _ptr(a2), _ptr(b2), _ptr(gamma),
                                                          _ptr(beta), eps, _ptr(y), _ptr(mean),
                                                          _ptr(rstd), _stream()), "layernorm fwd")
        ctx.save_for_backward(a2, b2, gamma, beta, mean, rstd)
        ctx.shape = a.shape
        return y.view(a.shape)

    @staticmethod
    @_keeps_precision
    def backward(ctx, dy):
        a2, b2, gamma, beta, mean, rstd = ctx.saved_tensors
        dy2 = dy.reshape(-1, a2.shape[1]).contiguous()
        dx = _resln_bwd(dy2, a2, b2, gamma, beta, mean, rstd).view(ctx.shape)
        return dx, dx, None, None, None


def residual_layernorm(y, x, gamma, beta, eps=1e-5):
    """LayerNorm(y + x) — ResidualConnection with use_layer_norm (residual_connection.py:29-31)."""
    return _ResLNFn.apply(y, x, gamma, beta, eps)


def _resln_fwd(a2, b2, gamma, beta, eps):
    """u = LN(a + b) over [rows, E] (both contiguous); returns (u, mean, rstd)."""
    rows, E = a2.shape
    dev = a2.device
    y = torch.empty_like(a2)
    mean = torch.empty(rows, device=dev, dtype=torch.float32)
    rstd = torch.empty(rows, device=dev, dtype=torch.float32)
    _lib.check(_lib.load().mrg_residual_layernorm_fwd(rows, E, _ptr(a2), _ptr(b2), _ptr(gamma), _ptr(beta), eps,
                                                      _ptr(y), _ptr(mean), _ptr(rstd), _stream()), "layernorm fwd")
    return y, mean, rstd


def _resln_bwd(dy2, a2, b2, gamma, beta, mean, rstd):
    """g = dL/d(a + b) of u = LN(a + b); dgamma / dbeta accumulate into the parameters' grads."""
    rows, E = a2.shape
    dev = a2.device
    g = torch.empty_like(a2)
    lib = _lib.load()
    ws = _ws(lib.mrg_residual_layernorm_bwd_workspace_bytes(rows, E), dev)
    gg, gb = _gbuf(gamma), _gbuf(beta)
    _lib.check(lib.mrg_residual_layernorm_bwd(
        rows, E, _ptr(dy2), _ptr(a2), _ptr(b2), _ptr(gamma), _ptr(mean), _ptr(rstd), _ptr(g),
        None, None, 1, _ptr(ws), _stream()), "layernorm bwd")
    if gg is not None or gb is not None:
        # dgamma / dbeta from the per-block partials: parameter gradients, off the critical path
        def reduce():
            scratch = None
            if gg is None or gb is None:
                scratch = _ws(2 * E * 4, dev).view(2, E)
            _lib.check(lib.mrg_residual_layernorm_param_reduce(
                rows, E, _ptr(ws), _ptr(gg if gg is not None else scratch[0]),
                _ptr(gb if gb is not None else scratch[1]), 1, _stream()), "layernorm param reduce")
        _on_side(dev, rows, (ws,), reduce, writes=(gg, gb))
    return g


# ------------------------------------------------------------------ Linear / FFN + residual LayerNorm
# LN(f(x) + x) with f's input-gradient GEMM taking the residual branch in its epilogue
# (dx = g W + g, epilogue 3): the add autograd would run for the two uses of x disappears.
class _LinResLNFn(Function):
    """LN(x W^T + b + x): FeedForward(nonlinearity none, residual, LN) (mixer_block.py:63-83)."""

    @staticmethod
    @_keeps_precision
    def forward(ctx, x, w, b, gamma, beta, eps):
        _lib.require_device(x)
        E = w.shape[0]
        x2 = x.reshape(-1, E).contiguous()
        M = x2.shape[0]
        z = torch.empty(M, E, device=x.device, dtype=torch.float32)
        _fwd_gemm(M, E, E, _ptr(x2), E, w, _ptr(z), E, bias=_ptr(b), device=x.device)
        _wt_note(w, M, ctx.needs_input_grad[0])
        y, mean, rstd = _resln_fwd(z, x2, gamma, beta, eps)
        ctx.save_for_backward(x2, w, b, z, gamma, beta, mean, rstd)
        ctx.xshape = x.shape
        return y.view(x.shape)

    @staticmethod
    @_keeps_precision
    def backward(ctx, dy):
        x2, w, b, z, gamma, beta, mean, rstd = ctx.saved_tensors
        M, E = x2.shape
        dev = dy.device
        g = _resln_bwd(dy.reshape(M, E).contiguous(), z, x2, gamma, beta, mean, rstd)
        _wgrad(_ptr(g), E, _ptr(x2), E, M, E, E, _gbuf(w), dev, gb=_gbuf(b), keep=(g, x2))
        dx = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty(M, E, device=dev, dtype=torch.float32)
            _dx_gemm(M, E, E, _ptr(g), E, w, _ptr(dx), E, epi=3, aux=_ptr(g), ldaux=E, device=dev)
            dx = dx.view(ctx.xshape)
        return dx, None, None, None, None, None


def linear_residual_layernorm(x, weight, bias, gamma, beta, eps=1e-5):
    return _LinResLNFn.apply(x, weight, bias, gamma, beta, eps)


class _FFNResLNFn(Function):
    """LN(W2 relu(W1 x + b1) + b2 + x): the metaformer block FeedForward (multi_modal_metaformer.py:328)."""

    @staticmethod
    @_keeps_precision
    def forward(ctx, x, w1, b1, w2, b2, gamma, beta, eps):
        _lib.require_device(x)
        Hb, E = w1.shape
        x2 = x.reshape(-1, E).contiguous()
        M = x2.shape[0]
        dev = x.device
        h = torch.empty(M, Hb, device=dev, dtype=torch.float32)
        gemm(M, Hb, E, _ptr(x2), 0, E, _ptr(w1), 1, E, _ptr(h), Hb, bias=_ptr(b1), epi=1, device=dev)
        z = torch.empty(M, E, device=dev, dtype=torch.float32)
        _fwd_gemm(M, E, Hb, _ptr(h), Hb, w2, _ptr(z), E, bias=_ptr(b2), device=dev)
        _wt_note(w1, M, ctx.needs_input_grad[0])
        _tap_relu(w1, h, x.shape[:-1])
        y, mean, rstd = _resln_fwd(z, x2, gamma, beta, eps)
        ctx.save_for_backward(x2, h, z, w1, b1, w2, b2, gamma, beta, mean, rstd)
        ctx.xshape = x.shape
        return y.view(x.shape)

    @staticmethod
    @_keeps_precision
    def backward(ctx, dy):
        x2, h, z, w1, b1, w2, b2, gamma, beta, mean, rstd = ctx.saved_tensors
        Hb, E = w1.shape
        M = x2.shape[0]
        dev = dy.device
        g = _resln_bwd(dy.reshape(M, E).contiguous(), z, x2, gamma, beta, mean, rstd)
        dh = torch.empty(M, Hb, device=dev, dtype=torch.float32)
        gemm(M, Hb, E, _ptr(g), 0, E, _ptr(w2), 0, Hb, _ptr(dh), Hb, epi=2, aux=_ptr(h), ldaux=Hb, device=dev)
        _wgrad(_ptr(g), E, _ptr(h), Hb, M, E, Hb, _gbuf(w2), dev, gb=_gbuf(b2), keep=(g, h))
        _wgrad(_ptr(dh), Hb, _ptr(x2), E, M, Hb, E, _gbuf(w1), dev, gb=_gbuf(b1), keep=(dh, x2))
        dx = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty(M, E, device=dev, dtype=torch.float32)
            _dx_gemm(M, E, Hb, _ptr(dh), Hb, w1, _ptr(dx), E, epi=3, aux=_ptr(g), ldaux=E, device=dev)
            dx = dx.view(ctx.xshape)
        return dx, None, None, None, None, None, None, None


def ffn_residual_layernorm(x, w1, b1, w2, b2, gamma, beta, eps=1e-5):
    return _FFNResLNFn.apply(x, w1, b1, w2, b2, gamma, beta, eps)


# ------------------------------------------------------------------ LSTM
class _LSTMFn(Function):
    """``nprob`` same-shape single-layer LSTM directions in one persistent launch.

    tensors = [x, w_ih, w_hh, b_ih, b_hh, h0, c0] * nprob (h0/c0 may be None).
    concat: True = all problems share x and write one [B, T, nprob*H] output (bidirectional layer:
    forward then reverse, like nn.LSTM); an int g = consecutive groups of g problems, each group
    sharing its x and writing one [B, T, g*H] output (several bidirectional layers on different
    inputs in one launch: g = 2); False = one output per problem.
    Outputs: (y...) then (hT_i, cT_i) per problem.
    """

    @staticmethod
    @_keeps_precision
    def forward(ctx, spec, *tensors):
        nprob, concat, reverse, force_bs, eps = spec
        # unused outputs (hT, cT of the stateless mixers) get no gradient: None, not a
        # zero-filled tensor (the recurrence takes null dhT / dcT as zero)
        ctx.set_materialize_grads(False)
        resln = eps is not None  # per problem LN(y + x) (ResidualConnection around LSTMMixer)
        K = 9 if resln else 7
        probs = [tensors[K * i:K * i + K] for i in range(nprob)]
        x0 = probs[0][0]
        _lib.require_device(x0)
        dev = x0.device
        B, T, In = x0.shape
        H = probs[0][2].shape[1]
        lib = _lib.load()
        if not lib.mrg_lstm_supported_hidden(H):
            raise RuntimeError(f"LSTM hidden size {H} not supported by libmrg (16/32/64/128/256)")
        xs = [p[0].contiguous() for p in probs]
        gs = nprob if concat is True else (1 if concat is False else int(concat))   # problems per output
        if nprob % gs or (resln and gs > 1):
            raise ValueError(f"lstm: {nprob} problems do not form groups of {gs}")
        concat = gs > 1
        gxs, ys, y_ptrs, y_bs, y_ts = [], [], [], [], []
        if concat:
            ycats = [torch.empty(B, T, gs * H, device=dev, dtype=torch.float32) for _ in range(nprob // gs)]
        for i, p in enumerate(probs):
            x, w_ih, b_ih = xs[i], p[1], p[3]
            In_i = x.shape[2]
            gx = torch.empty(B, T, 4 * H, device=dev, dtype=torch.float32)
            _fwd_gemm(B * T, 4 * H, In_i, _ptr(x), In_i, w_ih, _ptr(gx), 4 * H, bias=_ptr(b_ih), device=dev)
            _wt_note(w_ih, B * T, ctx.needs_input_grad[1 + K * i])
            gxs.append(gx)
            if concat:
                y_ptrs.append(_ptr(ycats[i // gs], (i % gs) * H))
                y_bs.append(T * gs * H)
                y_ts.append(gs * H)
            else:
                y = torch.empty(B, T, H, device=dev, dtype=torch.float32)
                ys.append(y)
                y_ptrs.append(_ptr(y))
                y_bs.append(T * H)
                y_ts.append(H)
        gates = [torch.empty(B, T, 4 * H, device=dev, dtype=torch.float32) for _ in range(nprob)]
        cs = [torch.empty(B, T, H, device=dev, dtype=torch.float32) for _ in range(nprob)]
        hT = [torch.empty(B, H, device=dev, dtype=torch.float32) for _ in range(nprob)]
        cT = [torch.empty(B, H, device=dev, dtype=torch.float32) for _ in range(nprob)]
        xb_elems = lib.mrg_lstm_fwd_xbuf_bytes(B, H) // 8
        xbuf = zeros(nprob, xb_elems, dtype=torch.int64, device=dev)
        h0 = [None if p[5] is None else p[5].contiguous() for p in probs]
        c0 = [None if p[6] is None else p[6].contiguous() for p in probs]

        def arr(ctype, vals):
            return (ctype * nprob)(*vals)
        VP = ctypes.c_void_p
        pr = _probe("lstm_fwd", 8.0 * H * H * B * T * nprob).__enter__()  # recurrent h W_hh^T FLOPs
        rc = lib.mrg_lstm_fwd(
            nprob, B, T, H,
            arr(VP, [_ptr(g) for g in gxs]), arr(ctypes.c_long, [T * 4 * H] * nprob),
            arr(ctypes.c_long, [4 * H] * nprob),
            arr(VP, [_ptr(p[2]) for p in probs]), arr(VP, [_ptr(p[4]) for p in probs]),
            arr(VP, [_ptr(h) for h in h0]), arr(VP, [_ptr(c) for c in c0]),
            arr(VP, y_ptrs), arr(ctypes.c_long, y_bs), arr(ctypes.c_long, y_ts),
            arr(VP, [_ptr(g) for g in gates]), arr(VP, [_ptr(c) for c in cs]),
            arr(VP, [_ptr(h) for h in hT]), arr(VP, [_ptr(c) for c in cT]),
            arr(ctypes.c_int, [int(r) for r in reverse]),
            arr(VP, [_ptr(xbuf[i]) for i in range(nprob)]), None, _ptr(_err_flag(dev)),
            _lib.cu_count(dev.index or 0), force_bs, _stream())
        pr.__exit__()
        _lib.check(rc, "lstm fwd")
        ctx.spec = (nprob, gs, tuple(reverse), force_bs, B, T, H, resln)
        ctx.has_h0 = [h is not None for h in h0]
        ctx.has_c0 = [c is not None for c in c0]
        ctx.y_layout = (y_bs, y_ts)
        yout = ycats if concat else ys
        save = []
        uout = []
        for i, p in enumerate(probs):
            save += [xs[i], p[1], p[2], p[3], p[4], gates[i], cs[i], h0[i], c0[i]]
            if resln:
                u, mean, rstd = _resln_fwd(ys[i].view(B * T, H), xs[i].view(B * T, H), p[7], p[8], eps)
                uout.append(u.view(B, T, H))
                save += [p[7], p[8], mean, rstd]
        save += yout
        ctx.save_for_backward(*save)
        # each problem's x owner: the first problem holding the same tensor (its dx collects theirs)
        ctx.x_owner = [next(k for k in range(i + 1) if probs[k][0] is probs[i][0]) for i in range(nprob)]
        outs = list(uout if resln else yout)
        for i in range(nprob):
            outs += [hT[i], cT[i]]
        return tuple(outs)

    @staticmethod
    @_keeps_precision
    def backward(ctx, *grads):
        nprob, gs, reverse, force_bs, B, T, H, resln = ctx.spec
        concat = gs > 1
        saved = ctx.saved_tensors
        S = 13 if resln else 9
        per = [saved[S * i:S * i + S] for i in range(nprob)]
        yout = saved[S * nprob:]
        dev = yout[0].device
        lib = _lib.load()
        ny = nprob // gs
        gy = list(grads[:ny])
        gstate = grads[ny:]
        res = [None] * nprob  # residual-branch gradient g_i of LN(y_i + x_i), added by the dX GEMM
        if resln:
            for i in range(nprob):
                if gy[i] is None:
                    continue
                gamma, beta, mean, rstd = per[i][9:13]
                res[i] = _resln_bwd(gy[i].reshape(B * T, H).contiguous(), yout[i].view(B * T, H),
                                    per[i][0].view(B * T, H), gamma, beta, mean, rstd)
                gy[i] = res[i].view(B, T, H)
        y_bs, y_ts = ctx.y_layout
        dy_ptr, dy_bs, dy_ts = [], [], []
        for i in range(nprob):
            g = gy[i // gs]
            if g is None:
                dy_ptr.append(None)
                dy_bs.append(0)
                dy_ts.append(0)
            else:
                g = g.contiguous()
                if concat:
                    gy[i // gs] = g
                    dy_ptr.append(_ptr(g, (i % gs) * H))
                else:
                    gy[i] = g
                    dy_ptr.append(_ptr(g))
                dy_bs.append(y_bs[i])
                dy_ts.append(y_ts[i])
        dhT = [None if gstate[2 * i] is None else gstate[2 * i].contiguous() for i in range(nprob)]
        dcT = [None if gstate[2 * i + 1] is None else gstate[2 * i + 1].contiguous() for i in range(nprob)]
        dG = [torch.empty(B, T, 4 * H, device=dev, dtype=torch.float32) for _ in range(nprob)]
        need = ctx.needs_input_grad  # index 0 is spec
        K = 9 if resln else 7
        dh0 = [torch.empty(B, H, device=dev, dtype=torch.float32)
               if ctx.has_h0[i] and need[1 + K * i + 5] else None for i in range(nprob)]
        dc0 = [torch.empty(B, H, device=dev, dtype=torch.float32)
               if ctx.has_c0[i] and need[1 + K * i + 6] else None for i in range(nprob)]
        xb_elems = lib.mrg_lstm_bwd_xbuf_bytes(B, H) // 8
        xbuf = zeros(nprob, xb_elems, dtype=torch.int64, device=dev)

        def arr(ctype, vals):
            return (ctype * nprob)(*vals)
        VP = ctypes.c_void_p
        cap, mark = fork_beside_recurrence(dev)
        lib.mrg_lstm_set_blocks_per_cu(cap)
        pr = _probe("lstm_bwd", 8.0 * H * H * B * T * nprob).__enter__()  # dG W_hh FLOPs
        rc = lib.mrg_lstm_bwd(
            nprob, B, T, H,
            arr(VP, [_ptr(p[2]) for p in per]), arr(VP, [_ptr(p[5]) for p in per]),
            arr(VP, [_ptr(p[6]) for p in per]), arr(VP, [_ptr(p[8]) for p in per]),
            arr(VP, dy_ptr), arr(ctypes.c_long, dy_bs), arr(ctypes.c_long, dy_ts),
            arr(VP, [_ptr(t) for t in dhT]), arr(VP, [_ptr(t) for t in dcT]),
            arr(VP, [_ptr(t) for t in dG]), arr(VP, [_ptr(t) for t in dh0]),
            arr(VP, [_ptr(t) for t in dc0]), arr(ctypes.c_int, [int(r) for r in reverse]),
            arr(VP, [_ptr(xbuf[i]) for i in range(nprob)]), None, _ptr(_err_flag(dev)),
            _lib.cu_count(dev.index or 0), force_bs, _stream())
        pr.__exit__()
        _lib.check(rc, "lstm bwd")
        flush_beside_recurrence(dev, mark)

        out = [None]
        dx_of = {}   # first problem of each shared x -> its dx (the others add into it)
        for i in range(nprob):
            x, w_ih, w_hh, b_ih, b_hh, _g, _c, h0, _c0 = per[i][:9]
            In = x.shape[2]
            g = dG[i]
            rows = B * T
            gw = _gbuf(w_hh)
            if gw is not None and T > 1:
                # sum_t dG_t^T h_{t-1}: forward dir pairs (dG[t], y[t-1]); reverse (dG[t], y[t+1])
                yb = yout[i // gs]
                yoff = (i % gs) * H
                a_off = 0 if reverse[i] else 4 * H
                b_off = yoff + (y_ts[i] if reverse[i] else 0)
                _wgrad(_ptr(g, a_off), 4 * H, _ptr(yb, b_off), y_ts[i], B * (T - 1), 4 * H, H, gw, dev,
                       dy_hi=T * 4 * H, dy_div=T - 1, x_hi=y_bs[i], x_div=T - 1, keep=(g, yb))
            if gw is not None and h0 is not None:
                t0 = T - 1 if reverse[i] else 0
                _on_side(dev, B * T, (g, h0),
                         lambda g=g, h0=h0, gw=gw, t0=t0: gemm(4 * H, H, B, _ptr(g, t0 * 4 * H), 1, T * 4 * H,
                                                               _ptr(h0), 0, H, _ptr(gw), H, beta=1.0, device=dev),
                         writes=(gw,))
            gbi, gbh = _gbuf(b_ih), _gbuf(b_hh)
            first = gbi if gbi is not None else gbh
            second = gbh if gbi is not None else None
            _wgrad(_ptr(g), 4 * H, _ptr(x), In, rows, 4 * H, In, _gbuf(w_ih), dev, gb=first, gb2=second,
                   keep=(g, x))
            dx = None
            if need[1 + K * i]:
                owner = ctx.x_owner[i]
                if owner != i and owner in dx_of:
                    _dx_gemm(rows, In, 4 * H, _ptr(g), 4 * H, w_ih, _ptr(dx_of[owner]), In, beta=1.0, device=dev)
                else:
                    dx = torch.empty(B, T, In, device=dev, dtype=torch.float32)
                    if res[i] is not None:  # dx = dG W_ih + g (residual branch in the epilogue)
                        _dx_gemm(rows, In, 4 * H, _ptr(g), 4 * H, w_ih, _ptr(dx), In, epi=3, aux=_ptr(res[i]),
                                 ldaux=In, device=dev)
                    else:
                        _dx_gemm(rows, In, 4 * H, _ptr(g), 4 * H, w_ih, _ptr(dx), In, device=dev)
                    dx_of[i] = dx
            out += [dx, None, None, None, None, dh0[i], dc0[i]] + ([None, None] if resln else [])
        return tuple(out)


class _LSTMCellFn(Function):
    """One time step (T = 1) of one nn.LSTM direction: gate pre-activations by the GEMMs
    (x W_ih^T + b_ih, + h0 W_hh^T with a state) and the element-wise cell kernels.  The per-frame
    decode of lstm_with_sampling's scheduled sampling (lstm_with_sample.py:410-433) runs 300 of
    these per training step; a persistent recurrence launch per frame would be pure overhead."""

    @staticmethod
    @_keeps_precision
    def forward(ctx, x, w_ih, w_hh, b_ih, b_hh, h0, c0):
        _lib.require_device(x)
        dev = x.device
        B, _, In = x.shape
        H = w_hh.shape[1]
        lib = _lib.load()
        x2 = x.reshape(B, In).contiguous()
        h0c = None if h0 is None else h0.contiguous()
        c0c = None if c0 is None else c0.contiguous()
        gates = torch.empty(B, 4 * H, device=dev, dtype=torch.float32)
        c = torch.empty(B, H, device=dev, dtype=torch.float32)
        y = torch.empty(B, 1, H, device=dev, dtype=torch.float32)
        hT = torch.empty(B, H, device=dev, dtype=torch.float32)
        if _ARITH[0] is None and In % 4 == 0 and H % 4 == 0 and In + H <= 512:
            # gates GEMMs + cell in one launch (decode.hip lstm_step_fwd_kernel)
            _lib.check(lib.mrg_lstm_step_fwd(B, H, In, _ptr(x2), _ptr(h0c), _ptr(c0c), _ptr(w_ih), _ptr(w_hh),
                                             _ptr(b_ih), _ptr(b_hh), _ptr(gates), _ptr(c), _ptr(y), H, _ptr(hT),
                                             _stream()), "lstm step fwd")
        else:
            pre = torch.empty(B, 4 * H, device=dev, dtype=torch.float32)
            gemm(B, 4 * H, In, _ptr(x2), 0, In, _ptr(w_ih), 1, In, _ptr(pre), 4 * H, bias=_ptr(b_ih), device=dev)
            if h0c is not None:
                gemm(B, 4 * H, H, _ptr(h0c), 0, H, _ptr(w_hh), 1, H, _ptr(pre), 4 * H, beta=1.0, device=dev)
            _lib.check(lib.mrg_lstm_cell_fwd(B, H, _ptr(pre), 4 * H, _ptr(b_hh), _ptr(c0c), _ptr(gates), _ptr(c),
                                             _ptr(y), H, _ptr(hT), _stream()), "lstm cell fwd")
        ctx.save_for_backward(x2, w_ih, w_hh, b_ih, b_hh, h0c, c0c, gates, c)
        ctx.set_materialize_grads(False)  # an unused final state costs no zero-filled gradient
        return y, hT, c

    @staticmethod
    @_keeps_precision
    def backward(ctx, dy, dhT, dcT):
        x2, w_ih, w_hh, b_ih, b_hh, h0c, c0c, gates, c = ctx.saved_tensors
        B, In = x2.shape
        H = w_hh.shape[1]
        dev = x2.device
        lib = _lib.load()
        dy = None if dy is None else dy.contiguous()
        dhT = None if dhT is None else dhT.contiguous()
        dcT = None if dcT is None else dcT.contiguous()
        dG = torch.empty(B, 4 * H, device=dev, dtype=torch.float32)
        need = ctx.needs_input_grad
        dc0 = torch.empty(B, H, device=dev, dtype=torch.float32) if (c0c is not None and need[6]) else None
        _lib.check(lib.mrg_lstm_cell_bwd(B, H, _ptr(gates), _ptr(c), _ptr(c0c), _ptr(dy), H, _ptr(dhT), _ptr(dcT),
                                         _ptr(dG), _ptr(dc0), _stream()), "lstm cell bwd")
        gbi, gbh = _gbuf(b_ih), _gbuf(b_hh)
        first = gbi if gbi is not None else gbh
        _wgrad(_ptr(dG), 4 * H, _ptr(x2), In, B, 4 * H, In, _gbuf(w_ih), dev, gb=first,
               gb2=gbh if gbi is not None else None, keep=(dG, x2))
        gw = _gbuf(w_hh)  # zero state: dW_hh = dG^T h0 = 0 (the buffer still exists, as with nn.LSTM)
        if gw is not None and h0c is not None:
            _wgrad(_ptr(dG), 4 * H, _ptr(h0c), H, B, 4 * H, H, gw, dev, keep=(dG, h0c))
        dx = dh0 = None
        if need[0]:
            dx = torch.empty(B, 1, In, device=dev, dtype=torch.float32)
            gemm(B, In, 4 * H, _ptr(dG), 0, 4 * H, _ptr(w_ih), 0, In, _ptr(dx), In, device=dev)
        if h0c is not None and need[5]:
            dh0 = torch.empty(B, H, device=dev, dtype=torch.float32)
            gemm(B, H, 4 * H, _ptr(dG), 0, 4 * H, _ptr(w_hh), 0, H, _ptr(dh0), H, device=dev)
        return dx, None, None, None, None, dh0, dc0


def lstm_layer(x, w_ih, w_hh, b_ih, b_hh, h0=None, c0=None, reverse=False, force_bs=0):
    """One direction of one nn.LSTM layer (batch_first).  Returns (y, hT, cT)."""
    if x.shape[1] == 1 and force_bs == 0:
        return _LSTMCellFn.apply(x, w_ih, w_hh, b_ih, b_hh, h0, c0)
    y, hT, cT = _LSTMFn.apply((1, False, (reverse,), force_bs, None), x, w_ih, w_hh, b_ih, b_hh, h0, c0)
    return y, hT, cT


def lstm_residual_layernorm(x, w_ih, w_hh, b_ih, b_hh, gamma, beta, eps=1e-5, h0=None, c0=None,
                            force_bs=0):
    """LN(LSTM(x) + x) for one unidirectional layer (ResidualConnection(LSTMMixer), mixer_block.py:
    479-507); the LSTM's dX GEMM takes the residual gradient in its epilogue.  Returns (u, hT, cT)."""
    if x.shape[1] == 1 and force_bs == 0:
        y, hT, cT = _LSTMCellFn.apply(x, w_ih, w_hh, b_ih, b_hh, h0, c0)
        return residual_layernorm(y, x, gamma, beta, eps), hT, cT
    u, hT, cT = _LSTMFn.apply((1, False, (False,), force_bs, float(eps)), x, w_ih, w_hh, b_ih, b_hh, h0, c0,
                              gamma, beta)
    return u, hT, cT


def lstm_layers_batched(problems: Sequence[Sequence], force_bs=0):
    """Several independent same-shape unidirectional layers in ONE persistent launch.

    problems: [(x, w_ih, w_hh, b_ih, b_hh)] -> [y_i]; zero initial state.
    """
    flat = []
    eps = None
    for p in problems:
        x, w_ih, w_hh, b_ih, b_hh = p[:5]
        flat += [x, w_ih, w_hh, b_ih, b_hh, None, None]
        if len(p) > 5:  # (.., gamma, beta, eps): LN(LSTM(x) + x) per problem
            flat += [p[5], p[6]]
            eps = float(p[7])
    if eps is not None and any(len(p) <= 5 for p in problems):
        raise ValueError("lstm_layers_batched: residual LayerNorm must be given for every problem or none")
    n = len(problems)
    if problems[0][0].shape[1] == 1 and force_bs == 0:
        return [lstm_layer(*p[:5])[0] if len(p) <= 5 else lstm_residual_layernorm(*p[:5], p[5], p[6], p[7])[0]
                for p in problems]
    outs = _LSTMFn.apply((n, False, (False,) * n, force_bs, eps), *flat)
    return list(outs[:n])


def lstm_bidirectional_layers(layers, force_bs=0):
    """Several independent bidirectional nn.LSTM layers (zero initial state) in ONE persistent launch:
    layers = [(x [B, T, In_i], fw, bw)] with fw / bw = (w_ih, w_hh, b_ih, b_hh), the same B, T and
    hidden size.  Returns [(y [B, T, 2H], hT [2, B, H], cT [2, B, H])] per layer."""
    flat, rev = [], []
    for x, fw, bw in layers:
        flat += [x, *fw, None, None, x, *bw, None, None]
        rev += [False, True]
    n = len(layers)
    outs = _LSTMFn.apply((2 * n, 2, tuple(rev), force_bs, None), *flat)
    ys, st = outs[:n], outs[n:]
    return [(ys[k], torch.stack([st[4 * k], st[4 * k + 2]]), torch.stack([st[4 * k + 1], st[4 * k + 3]]))
            for k in range(n)]


def lstm_bidirectional_layer(x, fw, bw, h0=None, c0=None, force_bs=0):
    """One bidirectional nn.LSTM layer: fw/bw = (w_ih, w_hh, b_ih, b_hh); returns (y[B,T,2H], hT[2,B,H], cT)."""
    h0f = h0b = c0f = c0b = None
    if h0 is not None:
        h0f, h0b = h0[0], h0[1]
    if c0 is not None:
        c0f, c0b = c0[0], c0[1]
    outs = _LSTMFn.apply((2, True, (False, True), force_bs, None), x, *fw, h0f, c0f, x, *bw, h0b, c0b)
    y, hTf, cTf, hTb, cTb = outs
    return y, torch.stack([hTf, hTb]), torch.stack([cTf, cTb])


# ------------------------------------------------------------------ multi-head attention
class _GRUFn(Function):
    """One direction of one torch.nn.GRU layer (gate order r, z, n; mixer_block.py:169-208), batch
    first: the input GEMM for all steps, then per step the few-row recurrent GEMM h W_hh^T and the
    fused cell (gru.hip); backward runs the cell derivative and dh_{t-1} += dGH_t W_hh per step, then
    the weight / bias / input gradients as GEMMs over all steps.  Returns (y [B, T, H], hT [B, H])."""

    @staticmethod
    @_keeps_precision
    def forward(ctx, reverse, x, w_ih, w_hh, b_ih, b_hh, h0):
        _lib.require_device(x)
        dev = x.device
        B, T, In = x.shape
        H = w_hh.shape[1]
        H3 = 3 * H
        lib = _lib.load()
        x = x.contiguous()
        gx = torch.empty(B, T, H3, device=dev, dtype=torch.float32)
        gemm(B * T, H3, In, _ptr(x), 0, In, _ptr(w_ih), 1, In, _ptr(gx), H3, bias=_ptr(b_ih), device=dev)
        y = torch.empty(B, T, H, device=dev, dtype=torch.float32)
        gates = torch.empty(B, T, H3, device=dev, dtype=torch.float32)
        ghn = torch.empty(B, T, H, device=dev, dtype=torch.float32)
        h0c = None if h0 is None else h0.contiguous()
        ctx.persist = _GRU_PERSIST[0] and T > 1 and bool(lib.mrg_gru_supported_hidden(H))
        if ctx.persist:   # one persistent launch for all steps (gru_rec.hip)
            xb = zeros(max(1, lib.mrg_gru_xbuf_bytes(B, H) // 8), dtype=torch.int64, device=dev)
            with _probe("gru_fwd", 6.0 * H * H * B * T):
                rc = lib.mrg_gru_fwd(B, T, H, _ptr(gx), T * H3, H3, _ptr(w_hh), _ptr(b_hh), _ptr(h0c), _ptr(y), T * H,
                                     H, _ptr(gates), T * H3, H3, _ptr(ghn), T * H, H, int(bool(reverse)), _ptr(xb),
                                     _ptr(_err_flag(dev)), _lib.cu_count(dev.index or 0), _stream())
            _lib.check(rc, "gru fwd")
            prev = 0 if reverse else T - 1
            hT = y[:, prev].clone()
            ctx.reverse = bool(reverse)
            ctx.save_for_backward(x, w_ih, w_hh, b_ih, b_hh, h0c, y, gates, ghn)
            ctx.set_materialize_grads(False)
            return y, hT
        gh = torch.empty(B, H3, device=dev, dtype=torch.float32)
        zero = torch.zeros(B, H3, device=dev, dtype=torch.float32) if h0 is None else None
        prev = None
        for t in (range(T - 1, -1, -1) if reverse else range(T)):
            if prev is None:
                hp, hp_ld = _ptr(h0c), H
            else:
                hp, hp_ld = _ptr(y, prev * H), T * H
            if hp is not None:
                gemm(B, H3, H, hp, 0, hp_ld, _ptr(w_hh), 1, H, _ptr(gh), H3, device=dev)
            _lib.check(lib.mrg_gru_cell_fwd(B, H, _ptr(gx, t * H3), T * H3, _ptr(gh if hp is not None else zero),
                                            _ptr(b_hh), hp, hp_ld, _ptr(y, t * H), T * H, _ptr(gates, t * H3), T * H3,
                                            _ptr(ghn, t * H), T * H, _stream()), "gru cell fwd")
            prev = t
        hT = y[:, prev].clone() if T > 0 else (h0c.clone() if h0c is not None else torch.zeros(B, H, device=dev))
        ctx.reverse = bool(reverse)
        ctx.save_for_backward(x, w_ih, w_hh, b_ih, b_hh, h0c, y, gates, ghn)
        ctx.set_materialize_grads(False)
        return y, hT

    @staticmethod
    @_keeps_precision
    def backward(ctx, dy, dhT):
        x, w_ih, w_hh, b_ih, b_hh, h0c, y, gates, ghn = ctx.saved_tensors
        reverse = ctx.reverse
        dev = x.device
        B, T, In = x.shape
        H = w_hh.shape[1]
        H3 = 3 * H
        lib = _lib.load()
        dy = None if dy is None else dy.contiguous()
        dGX = torch.empty(B, T, H3, device=dev, dtype=torch.float32)
        dGH = torch.empty(B, T, H3, device=dev, dtype=torch.float32)
        dh_next = None if dhT is None else dhT.contiguous()
        need = ctx.needs_input_grad
        if ctx.persist:
            xb = zeros(max(1, lib.mrg_gru_xbuf_bytes(B, H) // 8), dtype=torch.int64, device=dev)
            dh_next = torch.empty(B, H, device=dev, dtype=torch.float32) if (h0c is not None and need[6]) else None
            # deferred weight gradients (functional._DEFER) run beside this recurrence, as beside the LSTM's
            _cap, mark = fork_beside_recurrence(dev)
            with _probe("gru_bwd", 6.0 * H * H * B * T):
                rc = lib.mrg_gru_bwd(B, T, H, _ptr(w_hh), _ptr(gates), T * H3, H3, _ptr(ghn), T * H, H, _ptr(y), T * H,
                                     H, _ptr(h0c), _ptr(dy), T * H, H, _ptr(None if dhT is None else dhT.contiguous()),
                                     _ptr(dGX), _ptr(dGH), T * H3, H3, _ptr(dh_next), int(reverse), _ptr(xb),
                                     _ptr(_err_flag(dev)), _lib.cu_count(dev.index or 0), _stream())
            _lib.check(rc, "gru bwd")
            flush_beside_recurrence(dev, mark)
        for t in ((range(T) if reverse else range(T - 1, -1, -1)) if not ctx.persist else ()):
            pt = t + 1 if reverse else t - 1
            if 0 <= pt < T:
                hp, hp_ld = _ptr(y, pt * H), T * H
            else:
                hp, hp_ld = _ptr(h0c), H
            dhp = torch.empty(B, H, device=dev, dtype=torch.float32)
            _lib.check(lib.mrg_gru_cell_bwd(B, H, _ptr(gates, t * H3), T * H3, _ptr(ghn, t * H), T * H, hp, hp_ld,
                                            _ptr(dy, t * H) if dy is not None else None, T * H, _ptr(dh_next),
                                            _ptr(dGX, t * H3), _ptr(dGH, t * H3), T * H3, _ptr(dhp), _stream()),
                       "gru cell bwd")
            gemm(B, H, H3, _ptr(dGH, t * H3), 0, T * H3, _ptr(w_hh), 0, H, _ptr(dhp), H, beta=1.0, device=dev)
            dh_next = dhp
        dh0 = dh_next if (h0c is not None and need[6]) else None
        _wgrad(_ptr(dGX), H3, _ptr(x), In, B * T, H3, In, _gbuf(w_ih), dev, gb=_gbuf(b_ih), keep=(dGX, x))
        gw = _gbuf(w_hh)
        if gw is not None and T > 1:
            # sum_t dGH_t^T h_{t-1}: forward pairs (dGH[t], y[t-1]), reverse (dGH[t], y[t+1])
            a_off = 0 if reverse else H3
            b_off = H if reverse else 0
            _wgrad(_ptr(dGH, a_off), H3, _ptr(y, b_off), H, B * (T - 1), H3, H, gw, dev,
                   dy_hi=T * H3, dy_div=T - 1, x_hi=T * H, x_div=T - 1, keep=(dGH, y))
        if gw is not None and h0c is not None:
            t0 = T - 1 if reverse else 0
            _on_side(dev, B * T, (dGH, h0c),
                     lambda: gemm(H3, H, B, _ptr(dGH, t0 * H3), 1, T * H3, _ptr(h0c), 0, H, _ptr(gw), H, beta=1.0,
                                  device=dev), writes=(gw,))
        gbh = _gbuf(b_hh)
        if gbh is not None:
            _on_side(dev, B * T, (dGH,), lambda: colsum(B * T, H3, _ptr(dGH), H3, _ptr(gbh), device=dev),
                     writes=(gbh,))
        dx = None
        if need[1]:
            dx = torch.empty(B, T, In, device=dev, dtype=torch.float32)
            gemm(B * T, In, H3, _ptr(dGX), 0, H3, _ptr(w_ih), 0, In, _ptr(dx), In, device=dev)
        return None, dx, None, None, None, None, dh0


# persistent GRU recurrences (gru_rec.hip); MRG_GRU_PERSIST=0 runs the per-step products + cells
_GRU_PERSIST = [os.environ.get("MRG_GRU_PERSIST", "1") == "1"]


def gru_layer(x, w_ih, w_hh, b_ih, b_hh, h0=None, reverse=False):
    """One direction of one nn.GRU layer (batch_first).  Returns (y, hT)."""
    return _GRUFn.apply(bool(reverse), x, w_ih, w_hh, b_ih, b_hh, h0)


def visible_pairs(Tq, Tk, causal):
    """(query, key) pairs the block-causal rule admits per (sample, head) (gen_attention_mask rules)."""
    if not causal:
        return Tq * Tk
    if Tk >= Tq:
        r = Tk // Tq
        return sum(min((i + 1) * r, Tk) for i in range(Tq))
    r = Tq // Tk
    return sum(min(i // r + 1, Tk) for i in range(Tq))


class _MHAFn(Function):
    @staticmethod
    @_keeps_precision
    def forward(ctx, spec, q_in, kv_in, in_w, in_b, out_w, out_b, qpad, kpad, gamma=None, beta=None):
        heads, causal, eps = spec  # eps not None: return LN(attn + q) (ResidualConnection(MHAMixer))
        _lib.require_device(q_in)
        dev = q_in.device
        B, Tq, E = q_in.shape
        Tk = kv_in.shape[1]
        D = E // heads
        q2 = q_in.contiguous()
        kv2 = kv_in.contiguous()
        Q = torch.empty(B, Tq, E, device=dev, dtype=torch.float32)
        _fwd_gemm(B * Tq, E, E, _ptr(q2), E, in_w[:E], _ptr(Q), E, bias=_ptr(in_b), device=dev)
        KV = torch.empty(B, Tk, 2 * E, device=dev, dtype=torch.float32)
        _fwd_gemm(B * Tk, 2 * E, E, _ptr(kv2), E, in_w[E:], _ptr(KV), 2 * E, bias=_ptr(in_b, E), device=dev)
        O = torch.empty(B, Tq, E, device=dev, dtype=torch.float32)
        lse = torch.empty(B, heads, Tq, device=dev, dtype=torch.float32)
        scale = 1.0 / math.sqrt(D)
        lib = _lib.load()
        with _probe("attn_fwd", 4.0 * D * B * heads * visible_pairs(Tq, Tk, causal)):
            rc = lib.mrg_attention_fwd(B, heads, Tq, Tk, D, _ptr(Q), Tq * E, E, _ptr(KV), Tk * 2 * E,
                                         2 * E, _ptr(KV, E), Tk * 2 * E, 2 * E, _ptr(O), Tq * E, E,
                                       _ptr(lse), _ptr(qpad), _ptr(kpad), int(causal), scale,
                                       _stream())
        _lib.check(rc, "attention fwd")
        out = torch.empty(B, Tq, E, device=dev, dtype=torch.float32)
        _fwd_gemm(B * Tq, E, E, _ptr(O), E, out_w, _ptr(out), E, bias=_ptr(out_b), device=dev)
        # dO = dout W_out runs in every backward (the in_proj weight gradient needs dO even when
        # neither input does), so out_w is noted unconditionally (a stale copy is never reused)
        _wt_note(out_w, B * Tq)
        _wt_note(in_w[:E], B * Tq, ctx.needs_input_grad[1])
        _wt_note(in_w[E:], B * Tk, ctx.needs_input_grad[2])
        extra = []
        res = out
        if eps is not None:
            u, mean, rstd = _resln_fwd(out.view(B * Tq, E), q2.view(B * Tq, E), gamma, beta, eps)
            res = u.view(B, Tq, E)
            extra = [out, gamma, beta, mean, rstd]
        ctx.save_for_backward(q2, kv2, Q, KV, O, lse, in_w, in_b, out_w, out_b, qpad, kpad, *extra)
        ctx.spec = (heads, causal, scale, eps is not None)
        return res

    @staticmethod
    @_keeps_precision
    def backward(ctx, dout):
        saved = ctx.saved_tensors
        q2, kv2, Q, KV, O, lse, in_w, in_b, out_w, out_b, qpad, kpad = saved[:12]
        heads, causal, scale, resln = ctx.spec
        B, Tq, E = q2.shape
        Tk = kv2.shape[1]
        D = E // heads
        dev = dout.device
        lib = _lib.load()
        g = None  # residual-branch gradient of LN(attn + q), added by the dq GEMM's epilogue
        if resln:
            out, gamma, beta, mean, rstd = saved[12:]
            g = _resln_bwd(dout.reshape(B * Tq, E).contiguous(), out.view(B * Tq, E), q2.view(B * Tq, E),
                           gamma, beta, mean, rstd)
            do2 = g.view(B, Tq, E)
        else:
            do2 = dout.contiguous()
        dO = torch.empty(B, Tq, E, device=dev, dtype=torch.float32)
        _dx_gemm(B * Tq, E, E, _ptr(do2), E, out_w, _ptr(dO), E, device=dev)
        _wgrad(_ptr(do2), E, _ptr(O), E, B * Tq, E, E, _gbuf(out_w), dev, gb=_gbuf(out_b), keep=(do2, O))
        dQ = torch.empty(B, Tq, E, device=dev, dtype=torch.float32)
        dKV = torch.empty(B, Tk, 2 * E, device=dev, dtype=torch.float32)
        ws = _ws(lib.mrg_attention_bwd_workspace_bytes(B, heads, Tq), dev)
        with _probe("attn_bwd", 10.0 * D * B * heads * visible_pairs(Tq, Tk, causal)):
            rc = lib.mrg_attention_bwd(
            B, heads, Tq, Tk, D, _ptr(Q), Tq * E, E, _ptr(KV), Tk * 2 * E, 2 * E, _ptr(KV, E), Tk * 2 * E,
            2 * E, _ptr(O), Tq * E, E, _ptr(lse), _ptr(qpad), _ptr(kpad), int(causal), scale,
            _ptr(dO), Tq * E, E, _ptr(dQ), Tq * E, E, _ptr(dKV), Tk * 2 * E, 2 * E, _ptr(dKV, E),
            Tk * 2 * E, 2 * E, _ptr(ws), _stream())
        _lib.check(rc, "attention bwd")
        gw, gb = _gbuf(in_w), _gbuf(in_b)
        _wgrad(_ptr(dQ), E, _ptr(q2), E, B * Tq, E, E, None if gw is None else gw[:E], dev,
               gb=None if gb is None else gb[:E], keep=(dQ, q2))
        _wgrad(_ptr(dKV), 2 * E, _ptr(kv2), E, B * Tk, 2 * E, E, None if gw is None else gw[E:], dev,
               gb=None if gb is None else gb[E:], keep=(dKV, kv2))
        dq_in = dkv_in = None
        if ctx.needs_input_grad[1]:
            dq_in = torch.empty(B, Tq, E, device=dev, dtype=torch.float32)
            if g is not None:
                _dx_gemm(B * Tq, E, E, _ptr(dQ), E, in_w[:E], _ptr(dq_in), E, epi=3, aux=_ptr(g), ldaux=E,
                         device=dev)
            else:
                _dx_gemm(B * Tq, E, E, _ptr(dQ), E, in_w[:E], _ptr(dq_in), E, device=dev)
        elif g is not None:
            dq_in = None
        if ctx.needs_input_grad[2]:
            dkv_in = torch.empty(B, Tk, E, device=dev, dtype=torch.float32)
            _dx_gemm(B * Tk, E, 2 * E, _ptr(dKV), 2 * E, in_w[E:], _ptr(dkv_in), E, device=dev)
        return None, dq_in, dkv_in, None, None, None, None, None, None, None, None


class _MHAOneKeyFn(Function):
    """nn.MultiheadAttention when every query sees exactly one key (Tq = Tk = 1: a frame of the
    generation loops attending to one partner / audio frame, lstmformer.py:498-521).  Softmax over a
    single visible key is exactly 1, so the attention output IS the value projection (bitwise the
    SDPA result: P = exp(s - s) / 1 = 1, O = 1 * V); the query / key projections and the attention
    kernel are skipped.  A row the mask rules hide entirely (query AND key padding) is NaN, as the
    softmax over an all -inf row is.  Gradients: dV = dO; the query and key projections get none
    (the reference's dS = P (dP - rowsum(dO O)) is 0 up to rounding there)."""

    @staticmethod
    @_keeps_precision
    def forward(ctx, eps, q_in, kv_in, in_w, in_b, out_w, out_b, qpad, kpad, gamma=None, beta=None):
        _lib.require_device(q_in)
        dev = q_in.device
        B, _, E = q_in.shape
        q2 = q_in.reshape(B, E).contiguous()
        kv2 = kv_in.reshape(B, E).contiguous()
        V = torch.empty(B, E, device=dev, dtype=torch.float32)
        gemm(B, E, E, _ptr(kv2), 0, E, _ptr(in_w, 2 * E * E), 1, E, _ptr(V), E, bias=_ptr(in_b, 2 * E), device=dev)
        hide = None
        O = V
        if qpad is not None and kpad is not None:
            hide = (qpad.reshape(B, 1) & kpad.reshape(B, 1)).bool()
            O = torch.where(hide, torch.full_like(V, float("nan")), V)
        out = torch.empty(B, E, device=dev, dtype=torch.float32)
        gemm(B, E, E, _ptr(O), 0, E, _ptr(out_w), 1, E, _ptr(out), E, bias=_ptr(out_b), device=dev)
        res = out
        extra = []
        if eps is not None:
            u, mean, rstd = _resln_fwd(out, q2, gamma, beta, eps)
            res = u
            extra = [out, gamma, beta, mean, rstd]
        ctx.save_for_backward(q2, kv2, O, in_w, in_b, out_w, out_b, *extra)
        ctx.hide = hide
        ctx.resln = eps is not None
        return res.view(B, 1, E)

    @staticmethod
    @_keeps_precision
    def backward(ctx, dout):
        saved = ctx.saved_tensors
        q2, kv2, O, in_w, in_b, out_w, out_b = saved[:7]
        B, E = q2.shape
        dev = dout.device
        g = None
        if ctx.resln:
            out, gamma, beta, mean, rstd = saved[7:]
            g = _resln_bwd(dout.reshape(B, E).contiguous(), out, q2, gamma, beta, mean, rstd)
            do2 = g
        else:
            do2 = dout.reshape(B, E).contiguous()
        dO = torch.empty(B, E, device=dev, dtype=torch.float32)
        gemm(B, E, E, _ptr(do2), 0, E, _ptr(out_w), 0, E, _ptr(dO), E, device=dev)
        _wgrad(_ptr(do2), E, _ptr(O), E, B, E, E, _gbuf(out_w), dev, gb=_gbuf(out_b), keep=(do2, O))
        if ctx.hide is not None:  # hidden rows: O is the constant NaN, nothing flows to V
            dO = torch.where(ctx.hide, torch.zeros_like(dO), dO)
        gw, gb = _gbuf(in_w), _gbuf(in_b)
        _wgrad(_ptr(dO), E, _ptr(kv2), E, B, E, E, None if gw is None else gw[2 * E:], dev,
               gb=None if gb is None else gb[2 * E:], keep=(dO, kv2))
        dkv = None
        if ctx.needs_input_grad[2]:
            dkv = torch.empty(B, 1, E, device=dev, dtype=torch.float32)
            gemm(B, E, E, _ptr(dO), 0, E, _ptr(in_w, 2 * E * E), 0, E, _ptr(dkv), E, device=dev)
        dq = g.view(B, 1, E) if (g is not None and ctx.needs_input_grad[1]) else None
        return None, dq, dkv, None, None, None, None, None, None, None, None


def _one_key(q, kv):
    return q.dim() == 3 and q.shape[1] == 1 and kv.shape[1] == 1 and kv.shape[-1] == q.shape[-1]


def mha(q, kv, in_proj_weight, in_proj_bias, out_weight, out_bias, heads, causal=False,
        qpad=None, kpad=None):
    """nn.MultiheadAttention(batch_first, kdim=vdim=E)(q, kv, kv) with the reference mask rules."""
    if in_proj_weight.shape[0] != 3 * q.shape[-1]:
        raise ValueError("in_proj_weight must be [3E, E]")
    if _one_key(q, kv):
        return _MHAOneKeyFn.apply(None, q, kv, in_proj_weight, in_proj_bias, out_weight, out_bias, qpad, kpad)
    return _MHAFn.apply((heads, bool(causal), None), q, kv, in_proj_weight, in_proj_bias, out_weight,
                        out_bias, qpad, kpad)


def mha_residual_layernorm(q, kv, in_proj_weight, in_proj_bias, out_weight, out_bias, heads, gamma, beta,
                           eps=1e-5, causal=False, qpad=None, kpad=None):
    """LN(MHA(q, kv, kv) + q): ResidualConnection(MHAMixer) (mixer_block.py:567-603); the query
    projection's input-gradient GEMM takes the residual gradient in its epilogue."""
    if in_proj_weight.shape[0] != 3 * q.shape[-1]:
        raise ValueError("in_proj_weight must be [3E, E]")
    if _one_key(q, kv):
        return _MHAOneKeyFn.apply(float(eps), q, kv, in_proj_weight, in_proj_bias, out_weight, out_bias, qpad, kpad,
                                  gamma, beta)
    return _MHAFn.apply((heads, bool(causal), float(eps)), q, kv, in_proj_weight, in_proj_bias, out_weight,
                        out_bias, qpad, kpad, gamma, beta)


def padding_flags(x: torch.Tensor, padding_value: float = -100.0) -> torch.Tensor:
    """uint8 [B, T]: frame is padding (x[:, :, 0] == -100), as gen_attention_mask tests it
    (one library kernel on the device; torch on the host, e.g. for the CPU mask goldens)."""
    if not (x.is_cuda and x.dtype == torch.float32 and x.dim() == 3):
        return (x[:, :, 0] == padding_value).to(torch.uint8).contiguous()
    B, T, _ = x.shape
    out = torch.empty(B, T, dtype=torch.uint8, device=x.device)
    _lib.check(_lib.load().mrg_padding_flags(B, T, _ptr(x), x.stride(0), x.stride(1), float(padding_value), _ptr(out),
                                             _stream()), "padding flags")
    return out


def zero_padding(x: torch.Tensor, padding_value: float = -100.0) -> torch.Tensor:
    """x * (x != -100) (training_step's zeroing of padded motion_self frames, lstmformer.py:365-366)."""
    if not (x.is_cuda and x.dtype == torch.float32 and x.is_contiguous() and x.data_ptr() % 16 == 0):
        return x * (x != padding_value).to(x.dtype)
    y = torch.empty_like(x)
    _lib.check(_lib.load().mrg_zero_padding(x.numel(), _ptr(x), float(padding_value), _ptr(y), _stream()),
               "zero padding")
    return y


def zero_(t: torch.Tensor) -> torch.Tensor:
    """In-place zero of a contiguous device tensor on the current stream (mrg_fill_zero)."""
    if t.numel():
        if not (t.is_cuda and t.is_contiguous()):
            raise ValueError("functional.zero_: contiguous device tensor required")
        _lib.check(_lib.load().mrg_fill_zero(_ptr(t), t.numel() * t.element_size(), _stream()), "fill zero")
    return t


def zeros(*shape, dtype=torch.float32, device=None) -> torch.Tensor:
    """torch.zeros through the library's fill kernel (no at::native kernel in the replayed step)."""
    return zero_(torch.empty(*shape, dtype=dtype, device=device))


# ------------------------------------------------------------------ loss
_LOSS_TYPES = {"huber": 0, "mse": 1, "mae": 2, "smoothl1": 3}


class _LossFn(Function):
    @staticmethod
    def forward(ctx, y, target, lead, spec):
        _lib.require_device(y)
        y = y.contiguous()
        target = target.contiguous()
        B, Ttot, F = y.shape
        T = target.shape[1]
        if Ttot - lead != T or target.shape[0] != B or target.shape[2] != F:
            raise RuntimeError(f"loss shape mismatch: y{tuple(y.shape)}[:, {lead}:] vs target{tuple(target.shape)}")
        lib = _lib.load()
        loss = torch.empty(1, device=y.device, dtype=torch.float32)
        ws = _ws(lib.mrg_loss_workspace_bytes(B, T, F), y.device)
        _lib.check(lib.mrg_masked_loss_fwd(B, T, F, _ptr(y, lead * F), Ttot * F, _ptr(target), *spec,
                                           _ptr(loss), _ptr(ws), _stream()), "loss fwd")
        ctx.save_for_backward(y, target)
        ctx.lead, ctx.spec = lead, spec
        return loss.view(())

    @staticmethod
    def backward(ctx, gout):
        y, target = ctx.saved_tensors
        B, Ttot, F = y.shape
        T = target.shape[1]
        dy = zeros(y.shape, dtype=y.dtype, device=y.device)
        go = gout.reshape(1).contiguous()
        _lib.check(_lib.load().mrg_masked_loss_bwd(B, T, F, _ptr(y, ctx.lead * F), Ttot * F, _ptr(target),
                                                   *ctx.spec, _ptr(go), _ptr(dy, ctx.lead * F), _stream()),
                   "loss bwd")
        return dy, None, None, None


def masked_loss(y, target, lead=0, loss_type="huber", delta=1.0, beta=1.0, mask_padding=True,
                delta_order=0, delta_loss_scale=1.0):
    """Masked regression loss of the reference training_step on y[:, lead:] vs target."""
    F = y.shape[2]
    spec = (_LOSS_TYPES[loss_type], float(delta), float(beta), int(mask_padding),
            int(F // (delta_order + 1)), float(math.sqrt(delta_loss_scale)))
    return _LossFn.apply(y, target, int(lead), spec)


class _BcastLossFn(Function):
    """Mean loss over the reference's broadcast [Tm, B, T, F] target, analytically."""

    @staticmethod
    def forward(ctx, y, target, ms, spec):
        _lib.require_device(y)
        y = y.contiguous()
        target = target.contiguous()
        B, T, F = y.shape
        if tuple(target.shape) != (B, T, F) or ms.shape[0] != B or ms.shape[2] != F or ms.stride(2) != 1:
            raise RuntimeError(f"broadcast loss shapes: y{tuple(y.shape)} target{tuple(target.shape)} "
                               f"motion_self{tuple(ms.shape)}")
        lib = _lib.load()
        loss = torch.empty(1, device=y.device, dtype=torch.float32)
        ws = _ws(lib.mrg_broadcast_loss_workspace_bytes(B, T, F), y.device)
        _lib.check(lib.mrg_broadcast_loss_fwd(B, T, F, _ptr(y), T * F, _ptr(target), _ptr(ms), ms.stride(0),
                                              ms.stride(1), ms.shape[1], *spec, _ptr(loss), _ptr(ws), _stream()),
                   "broadcast loss fwd")
        ctx.save_for_backward(y, target, ms)
        ctx.spec = spec
        return loss.view(())

    @staticmethod
    def backward(ctx, gout):
        y, target, ms = ctx.saved_tensors
        B, T, F = y.shape
        lib = _lib.load()
        dy = torch.empty_like(y)
        ws = _ws(lib.mrg_broadcast_loss_workspace_bytes(B, T, F), y.device)
        go = gout.reshape(1).contiguous()
        _lib.check(lib.mrg_broadcast_loss_bwd(B, T, F, _ptr(y), T * F, _ptr(target), _ptr(ms), ms.stride(0),
                                              ms.stride(1), ms.shape[1], *ctx.spec, _ptr(go), _ptr(dy), _ptr(ws),
                                              _stream()), "broadcast loss bwd")
        return dy, None, None, None


def broadcast_masked_loss(pred, target, motion_self, loss_type="huber", delta=1.0, beta=1.0, scaler=True,
                          delta_order=0, delta_loss_scale=1.0):
    """The loss the reference takes on Metaformer.prediction's output (lstmformer.py:372-380 in the
    scheduled-sampling training_step, :413-418 in generation_step): pred [B, T, F] against
    target * motion_s_mask, which broadcasts to [Tm, B, T, F], mean over all of it.
    motion_self: the raw (-100 padded) self motion [B, Tm, F] the mask comes from.  scaler: the
    training step's sqrt(delta_loss_scale) on the T axis from T // (delta_order + 1)."""
    T = pred.shape[1]
    t_start = T // (delta_order + 1) if scaler else T + 1
    spec = (_LOSS_TYPES[loss_type], float(delta), float(beta), int(t_start),
            float(math.sqrt(delta_loss_scale)) if scaler else 1.0)
    return _BcastLossFn.apply(pred, target, motion_self, spec)
