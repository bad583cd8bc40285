"""Data-parallel gradient all-reduce over RCCL (torch.distributed backend "nccl" == RCCL on ROCm).

Reference: Lightning ``strategy: ddp`` (mr_gen/model/lstmformer/config.yaml:127)
= one process per GPU, gradients averaged across ranks after backward.  Here
the gradients already live in ONE flat fp32 buffer (optim.FusedAdamW), so the
exchange is a single in-place all-reduce (ReduceOp.AVG) of 52.2 MB for the
benchmark model, issued on a dedicated communication stream so it can be
overlapped with other work; the optimizer stream waits on it.  With the gloo
backend (CPU tests) AVG is emulated by SUM then a scale.

``overlap=True`` does what Lightning's DDP does during backward: the flat buffer
is cut into buckets at parameter boundaries in reverse registration order (the
order backward produces them), and each bucket's all-reduce is issued on the comm
stream as soon as every gradient write into it has been issued (functional's
gradient-ready listener), ordered after the main and weight-gradient streams.
The number of writes per parameter is taken from a first, non-overlapped census
backward (the graph is static, as DDP's ``static_graph``); every rank runs the
same graph, so the buckets complete in the same order everywhere (RCCL needs one
collective order on all ranks).  ``finish()`` makes the current stream wait.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist


def init_from_env(backend=None):
    """Initialise torch.distributed from torchrun's env (RANK/WORLD_SIZE/MASTER_*); no-op at world 1."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world <= 1 or dist.is_initialized():
        return dist.get_rank() if dist.is_initialized() else 0, world
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    dist.init_process_group(backend=backend)
    return dist.get_rank(), dist.get_world_size()


def broadcast_parameters(module: torch.nn.Module, src: int = 0):
    """Same initial weights on every rank (DDP does this at wrap time)."""
    if not (dist.is_initialized() and dist.get_world_size() > 1):
        return
    with torch.no_grad():
        for p in module.parameters():
            dist.broadcast(p.data, src)


class NativeComm:
    """An RCCL communicator owned by libmrg's C-ABI (``mrg_comm_*``, include/mrg.h).

    The 128-byte unique id made by rank 0 travels to the other ranks over torch.distributed
    (any backend: it is host bytes); each rank must have selected its GPU first.  ``allreduce``
    issues the given spans of a flat fp32 buffer as one RCCL group on the caller's current
    stream (op "mean" = ncclAvg, the DDP gradient mean; "sum").
    """

    def __init__(self, rank: int = None, world: int = None):
        import ctypes
        from . import _lib
        self._lib = _lib.load()
        if not self._lib.mrg_comm_available():
            raise RuntimeError("NativeComm: no librccl.so.1 in this process")
        self.rank = dist.get_rank() if rank is None else rank
        self.world = dist.get_world_size() if world is None else world
        nbytes = self._lib.mrg_comm_id_bytes()
        uid = (ctypes.c_char * nbytes)()
        if self.rank == 0:
            _lib.check(self._lib.mrg_comm_unique_id(uid), "mrg_comm_unique_id")
        if self.world > 1:
            obj = [bytes(uid)]
            dist.broadcast_object_list(obj, src=0)
            ctypes.memmove(uid, obj[0], nbytes)
        self._handle = ctypes.c_void_p()
        _lib.check(self._lib.mrg_comm_init(ctypes.byref(self._handle), self.world, uid, self.rank), "mrg_comm_init")

    def allreduce(self, buf: torch.Tensor, spans=None, op: str = "mean"):
        import ctypes
        from . import _lib
        _lib.require_device(buf)
        if buf.dtype != torch.float32 or not buf.is_contiguous():
            raise ValueError("NativeComm.allreduce: contiguous float32 buffer required")
        spans = [(0, buf.numel())] if spans is None else list(spans)
        offs = (ctypes.c_long * len(spans))(*[s for s, _ in spans])
        cnts = (ctypes.c_long * len(spans))(*[e - s for s, e in spans])
        stream = torch.cuda.current_stream(buf.device).cuda_stream
        _lib.check(self._lib.mrg_comm_allreduce_f32(self._handle, ctypes.c_void_p(buf.data_ptr()), offs, cnts,
                                                    len(spans), 1 if op == "mean" else 0,
                                                    ctypes.c_void_p(stream)), "mrg_comm_allreduce_f32")

    def close(self):
        if getattr(self, "_handle", None) is not None and self._handle.value:
            from . import _lib
            _lib.check(self._lib.mrg_comm_destroy(self._handle), "mrg_comm_destroy")
            self._handle = None


class GradReducer:
    """Average a flat gradient buffer across ranks, in buckets, on a side stream.

    ``comm``: None = torch.distributed (backend "nccl" is RCCL), or a ``NativeComm`` (libmrg's
    own RCCL communicator, the ``mrg_comm_*`` C-ABI)."""

    def __init__(self, flat_grad: torch.Tensor, bucket_elems: int = 0, params=None, overlap: bool = False,
                 bucket_bytes: int = 8 << 20, comm: "NativeComm" = None):
        self.flat_grad = flat_grad
        self.comm = comm
        self.world = comm.world if comm is not None else (dist.get_world_size() if dist.is_initialized() else 1)
        self.backend = dist.get_backend() if dist.is_initialized() else None
        n = flat_grad.numel()
        self.overlap = bool(overlap) and params is not None and self.world > 1
        self.stream = torch.cuda.Stream(device=flat_grad.device) if flat_grad.is_cuda else None
        if self.overlap:
            self._init_buckets(list(params), bucket_bytes // flat_grad.element_size())
        else:
            if bucket_elems <= 0:
                bucket_elems = n
            self.buckets = [(s, min(n, s + bucket_elems)) for s in range(0, n, bucket_elems)]

    # ------------------------------------------------------------ overlapped (bucketed) mode
    def _init_buckets(self, params, cap):
        base = self.flat_grad.data_ptr()
        es = self.flat_grad.element_size()
        spans = sorted(((p.grad.data_ptr() - base) // es, p.numel(), p) for p in params)
        self.buckets, self.bucket_of = [], {}
        self._named = [(f"param[{i}] {tuple(p.shape)}", p) for i, p in enumerate(params)]
        cur, start, end = [], None, None
        for off, k, p in reversed(spans):          # reverse registration order = backward order
            if cur and (end - off) > cap:
                self.buckets.append((start, end))
                cur = []
            if not cur:
                end = off + k
            cur.append(p)
            start = off
            self.bucket_of[id(p)] = len(self.buckets)
        if cur:
            self.buckets.append((start, end))
        self.expected = None                        # per-parameter writes per backward (census)
        self.counts = {}
        self.launched = [False] * len(self.buckets)
        self.remaining = None
        self.order = []                             # bucket launch order of the last backward
        self.order_in_backward = []                 # those launched before the end-of-backward callback
        self._task = None
        from . import functional as Fn
        Fn.set_grad_listener(self)

    def touch(self):
        task = torch._C._current_graph_task_id()
        if task != self._task:                       # first gradient write of a new backward pass
            self._task = task
            self.counts = {}
            self.launched = [False] * len(self.buckets)
            self.order = []
            self.order_in_backward = []
            if self.expected is not None:
                self.remaining = [0] * len(self.buckets)
                for pid, c in self.expected.items():
                    self.remaining[self.bucket_of[pid]] += c
            if task >= 0:
                torch.autograd.Variable._execution_engine.queue_callback(self.end_of_backward)

    def ready(self, params):
        for p in params:
            pid = id(p)
            self.counts[pid] = self.counts.get(pid, 0) + 1
            if self.expected is None:
                continue
            b = self.bucket_of[pid]
            if self.launched[b]:
                raise RuntimeError("GradReducer(overlap=True): a parameter received more gradient writes than "
                                   "in the census backward (dynamic graph); use overlap=False")
            self.remaining[b] -= 1
            if self.remaining[b] == 0:
                self._launch(b)

    def end_of_backward(self):
        from . import functional as Fn
        self.order_in_backward = list(self.order)
        Fn._flush_touched()
        if self.expected is None:                    # census pass: remember the structure
            self.expected = dict(self.counts)
            missing = [n for n, p in self._named if id(p) not in self.counts]
            if missing:
                # a gradient written outside libmrg (torch's AccumulateGrad) is invisible to the
                # listener: its bucket could launch before the write lands
                raise RuntimeError("GradReducer(overlap=True): parameters whose gradients do not come "
                                   f"from libmrg ops: {missing[:5]}; use overlap=False")
        for b in range(len(self.buckets)):
            if not self.launched[b]:
                self._launch(b)
        self._task = None

    def _launch(self, b):
        from . import functional as Fn
        s, e = self.buckets[b]
        self.launched[b] = True
        self.order.append(b)
        op, scale = self._op()
        dev = self.flat_grad.device
        if self.stream is not None:
            cur = torch.cuda.current_stream(dev)
            self.stream.wait_stream(cur)
            side = Fn._SIDE.get(dev.index or 0)
            if side is not None:
                self.stream.wait_stream(side)
            with torch.cuda.stream(self.stream):
                if self.comm is not None:
                    self.comm.allreduce(self.flat_grad, [(s, e)], "mean")
                    return
                dist.all_reduce(self.flat_grad[s:e], op=op)
                if scale != 1.0:
                    self.flat_grad[s:e].mul_(scale)
        else:
            dist.all_reduce(self.flat_grad[s:e], op=op)
            if scale != 1.0:
                self.flat_grad[s:e].mul_(scale)

    def _op(self):
        if self.backend == "nccl":
            return dist.ReduceOp.AVG, 1.0
        return dist.ReduceOp.SUM, 1.0 / self.world

    def finish(self):
        """Order the caller's stream after every bucket's all-reduce (call after backward)."""
        if self.world <= 1:
            return
        if not self.overlap:
            return self.allreduce()
        self._agree_error_flag()
        if self.stream is not None:
            torch.cuda.current_stream(self.flat_grad.device).wait_stream(self.stream)

    def _agree_error_flag(self):
        """Sum the device error flag (a persistent recurrence's hand-off timeout, functional._err_flag)
        over the ranks on the comm stream, after the gradient buckets: the faulting rank's gradients
        are already averaged into every rank's buffer, so every rank must skip that AdamW update (the
        kernel skips on a non-zero flag) and raise, not only the rank that saw the timeout."""
        from . import functional as Fn
        dev = self.flat_grad.device
        err = Fn._err_flag(dev)
        if not hasattr(self, "_errf"):
            self._errf = torch.zeros(1, dtype=torch.float32, device=dev)
        cur = torch.cuda.current_stream(dev) if self.stream is not None else None
        ctx = torch.cuda.stream(self.stream) if self.stream is not None else None
        if cur is not None:
            self.stream.wait_stream(cur)
            ctx.__enter__()
        try:
            self._errf.copy_(err)
            if self.comm is not None:
                self.comm.allreduce(self._errf, None, "sum")
            else:
                dist.all_reduce(self._errf, op=dist.ReduceOp.SUM)
            err.copy_(self._errf)
        finally:
            if ctx is not None:
                ctx.__exit__(None, None, None)

    def close(self):
        if self.overlap:
            from . import functional as Fn
            Fn.set_grad_listener(None)

    # ------------------------------------------------------------ after-backward mode
    def allreduce(self):
        if self.world <= 1:
            return
        if self.overlap:
            return self.finish()
        op, scale = self._op()
        if self.comm is not None:
            cur = torch.cuda.current_stream(self.flat_grad.device)
            self.stream.wait_stream(cur)
            with torch.cuda.stream(self.stream):
                self.comm.allreduce(self.flat_grad, self.buckets, "mean")
            self._agree_error_flag()
            cur.wait_stream(self.stream)
            return
        if self.stream is not None:
            cur = torch.cuda.current_stream(self.flat_grad.device)
            self.stream.wait_stream(cur)
            with torch.cuda.stream(self.stream):
                for s, e in self.buckets:
                    dist.all_reduce(self.flat_grad[s:e], op=op)
            self._agree_error_flag()
            cur.wait_stream(self.stream)
        else:
            for s, e in self.buckets:
                dist.all_reduce(self.flat_grad[s:e], op=op)
            self._agree_error_flag()
        if scale != 1.0:
            self.flat_grad.mul_(scale)
