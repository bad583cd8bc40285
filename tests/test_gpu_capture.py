"""HIP-graph capture invariants the training step relies on (graphs.capture, functional._side).

The replayed step forks weight-gradient work onto a side stream in two ways: ``wait_stream`` (fork at
the current point of the main stream, functional._side) and ``wait_event(mark)`` with a mark recorded
BEFORE the next backward recurrence's launch (functional.flush_beside_recurrence).  Both must keep the
side stream's own order across consecutive forks in the captured graph (later products accumulate into
the same gradient buffers and reuse split-K scratch), whatever the timing: a 20 ms busy kernel makes a
missing edge visible.  The model-level cases replay the whole lstmformer step with one fork per layer
(the default) and with one fork per product (round 3's failing pattern, encoder_stack.SPLIT_FORKS) and
require the replayed gradients to be bitwise the eager ones ("Graph-capture finding").
"""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _busy(ms):
    from multimodalreactiongeneration_amd import _lib
    _lib.check(_lib.load().mrg_debug_busy(1, 64, 256, float(ms) * 1e3, torch.cuda.current_stream().cuda_stream),
               "busy")


@pytest.mark.parametrize("pattern", ["wait_stream", "wait_event_mark"])
def test_capture_keeps_side_stream_order_across_forks(pattern):
    """main: x = 1 | fork -> side: busy 20 ms, y = x + 1 | main: a kernel | fork -> side: z = y + 1 |
    join -> main: w = z + 1.  Replayed, w must be 4 (z waits for y although the second fork only
    names a point of the main stream)."""
    dev = torch.device(DEV)
    side = torch.cuda.Stream(device=dev)
    x = torch.zeros(1 << 16, device=dev)
    y, z, w, v = (torch.zeros_like(x) for _ in range(4))
    g = torch.cuda.CUDAGraph()
    cap = torch.cuda.Stream(device=dev)
    with torch.cuda.stream(cap):
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=cap):
            cur = torch.cuda.current_stream()
            x.fill_(1.0)
            for i in range(2):
                if pattern == "wait_stream":
                    side.wait_stream(cur)
                    v.add_(1.0)                      # main-stream work after the fork point
                else:
                    mark = torch.cuda.Event()
                    mark.record(cur)
                    v.add_(1.0)                      # main-stream work between the mark and the wait
                    side.wait_event(mark)
                with torch.cuda.stream(side):
                    if i == 0:
                        _busy(20)
                        torch.add(x, 1.0, out=y)
                    else:
                        torch.add(y, 1.0, out=z)
            cur.wait_stream(side)
            torch.add(z, 1.0, out=w)
    for t in (x, y, z, w, v):
        t.fill_(-7.0)
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    assert (x[0].item(), y[0].item(), z[0].item(), w[0].item()) == (1.0, 2.0, 3.0, 4.0)


def test_fork_guard_with_side_only_work_between_same_point_forks():
    """functional._fork's capture guard (skip a second wait on a main-stream point the side stream
    already waited on) with side-stream-only work issued OUTSIDE _fork between two forks from the same
    point, and a join that resets the point: main: x = 1 | fork -> side: busy 20 ms,
    y = x + 1 | side only (no fork): u = y * 2 | fork again, same main point (wait skipped) -> side:
    z = u + x | join -> main: w = z + 1 | fork after the join (the point was reset) -> side: q = w + 1.
    Replayed twice, every value must be the eager one (x 1, y 2, u 4, z 5, w 6, q 7)."""
    from multimodalreactiongeneration_amd import functional as Fn
    dev = torch.device(DEV)
    side = torch.cuda.Stream(device=dev)
    x = torch.zeros(1 << 16, device=dev)
    y, u, z, w, q = (torch.zeros_like(x) for _ in range(5))
    key = 99   # a key of its own: the model's side streams are not involved
    g = torch.cuda.CUDAGraph()
    cap = torch.cuda.Stream(device=dev)
    skipped = []
    with torch.cuda.stream(cap):
        torch.cuda.synchronize()
        Fn.reset_fork_point()
        with torch.cuda.graph(g, stream=cap):
            cur = torch.cuda.current_stream()
            x.fill_(1.0)
            Fn._fork(key, side, cur)
            with torch.cuda.stream(side):
                _busy(20)
                torch.add(x, 1.0, out=y)
                torch.mul(y, 2.0, out=u)              # side-only work, not through _fork
            before = Fn._LAST_FORK.get(key)
            Fn._fork(key, side, cur)                  # same main point: the guard skips the wait
            skipped.append(before is not None and Fn._LAST_FORK.get(key) == before)
            with torch.cuda.stream(side):
                torch.add(u, x, out=z)
            cur.wait_stream(side)
            Fn.reset_fork_point(key)                  # what every join in functional does
            torch.add(z, 1.0, out=w)
            Fn._fork(key, side, cur)
            with torch.cuda.stream(side):
                torch.add(w, 1.0, out=q)
            cur.wait_stream(side)
        Fn.reset_fork_point()
    assert skipped == [True]
    for _ in range(2):
        for t in (x, y, u, z, w, q):
            t.fill_(-7.0)
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        assert [t[0].item() for t in (x, y, u, z, w, q)] == [1.0, 2.0, 4.0, 5.0, 6.0, 7.0]


@pytest.mark.parametrize("split,defer", [(False, True), (True, True), (True, False), (False, False)])
def test_replayed_step_bitwise_eager_fork_patterns(split, defer):
    """The lstmformer step (B = 64, T = 300) captured and replayed twice: every gradient bitwise the
    eager one, with one side-stream fork per encoder layer (default) and with one fork per product
    (encoder_stack.SPLIT_FORKS), weight gradients deferred beside the backward recurrences (default)
    or forked where they are ready.  (True, False) is the pattern whose replay was wrong before the
    fork-point guard (functional._fork: several forks from one main-stream point)."""
    from multimodalreactiongeneration_amd import configs as C
    from multimodalreactiongeneration_amd import encoder_stack as ES
    from multimodalreactiongeneration_amd import functional as Fn
    from multimodalreactiongeneration_amd.graphs import capture
    from multimodalreactiongeneration_amd.model import Metaformer
    from multimodalreactiongeneration_amd.synthetic import make_batch
    mc, oc, me = C.lstmformer_config(ratio=1)
    torch.manual_seed(0)
    m = Metaformer(mc, oc, me).to(DEV)
    opt = m.configure_optimizers()["optimizer"]
    batch = make_batch(B=64, T=300, ratio=1, seed=5, device=DEV)

    def step():
        opt.zero_grad()
        m.training_step(list(batch))["loss"].backward()
    prev = ES.SPLIT_FORKS
    prev_side, prev_defer = Fn.set_wgrad_stream(True), Fn.set_wgrad_defer(defer)
    try:
        ES.SPLIT_FORKS = split
        step()
        torch.cuda.synchronize()
        ref = opt.flat_grad.clone()
        replay = capture(step, 1)
        for _ in range(2):
            opt.flat_grad.fill_(-1.0)
            replay()
            torch.cuda.synchronize()
            Fn.check_errors()
            assert torch.equal(opt.flat_grad, ref)
    finally:
        ES.SPLIT_FORKS = prev
        Fn.set_wgrad_stream(prev_side)
        Fn.set_wgrad_defer(prev_defer)
