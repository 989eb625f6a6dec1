"""GPU, one process: HaloPipeline's overlapped branch (the side stream, async
collectives, per-slice waits, buffer reuse across calls -- grl/dist.py
HaloPipeline.run / .backward), the branch RCCL takes on a multi-GPU node.

RCCL cannot put two ranks on one GPU, and gloo takes the serial branch, so
the P shards of one graph run here as P threads of this process
(ShardedGraph.in_process), and the collective itself is replaced by a
loopback exchange with torch.distributed's async semantics:
  * issuing a slice's exchange records an event on the issuing stream; the
    transfer (device copies from the peers' slice tables) runs on the
    exchange's own stream after EVERY rank's event -- as a collective starts
    only when all ranks have queued their inputs;
  * a spin kernel (torch.cuda._sleep) runs first on that stream, so a missing
    wait in the pipeline reads tables the transfer has not filled yet;
  * the returned handle's .wait() makes the caller's current stream wait for
    every rank's transfer of that slice (a collective completes on all ranks).
Everything else -- packing, slice tables, stream waits, gathers, combine --
is the product code.  Checked: Z and dX bitwise equal to the serial branch,
with the delay on the exchange side and on the compute side, and two
back-to-back calls with different X (buffer reuse)."""
import threading

import pytest
import torch

from grl import DropEdge, TypedGraph
from grl.dist import HaloPipeline, ShardedGraph

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
SPIN = 2_000_000  # spin-kernel cycles: ~1 ms, far longer than a slice's copies or gathers here


class _Work:
    def __init__(self, events):
        self.events = events

    def wait(self):
        cur = torch.cuda.current_stream(DEV)
        for ev in self.events:
            cur.wait_event(ev)


class Loopback:
    """The P virtual ranks' stand-in for the process group."""

    def __init__(self, world, async_op, delay=0):
        self.world, self.async_op, self.delay = world, async_op, delay
        self.barrier = threading.Barrier(world)
        self.pipes = [None] * world
        self.ready, self.done = {}, {}

    def member(self, rank):
        return _Member(self, rank)


class _Member:
    def __init__(self, group, rank):
        self.g, self.rank = group, rank
        self.world, self.async_op = group.world, group.async_op
        self.stream = torch.cuda.Stream(DEV)  # the collective's own stream
        self.seq = 0

    def _collective(self, pipe, copies, async_op):
        g, r = self.g, self.rank
        key = self.seq
        self.seq += 1
        g.pipes[r] = pipe
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(DEV))  # the inputs as queued on the issuing stream
        g.ready[key, r] = ev
        g.barrier.wait()  # every rank has issued this slice's exchange
        for q in range(self.world):
            self.stream.wait_event(g.ready[key, q])
        with torch.cuda.stream(self.stream):
            if g.delay:
                torch.cuda._sleep(g.delay)
            copies(g.pipes)
        done = torch.cuda.Event()
        done.record(self.stream)
        g.done[key, r] = done
        g.barrier.wait()  # every rank's transfer is queued
        work = _Work([g.done[key, q] for q in range(self.world)])
        if not async_op:
            work.wait()
            return None
        return work

    def forward(self, pipe, c, async_op):
        r, p = self.rank, pipe.plan

        def copies(pipes):
            t = pipe.tables[c]
            if p.mode == "dense":  # all-gather of every rank's padded own rows
                for q, pq in enumerate(pipes):
                    t[p.stride * (1 + q): p.stride * (2 + q)].copy_(pq.tables[c][:p.stride])
                return
            off = p.n_loc
            for q, pq in enumerate(pipes):  # all-to-all-v: peer q's send rows for me, owner order
                cnt = p.recv_counts[q]
                if cnt:
                    o = sum(pq.plan.send_counts[:r])
                    t[off:off + cnt].copy_(pq.send[c][o:o + cnt])
                off += cnt

        return self._collective(pipe, copies, async_op)

    def backward(self, pipe, c, async_op):
        r, p = self.rank, pipe.plan

        def copies(pipes):
            back = pipe.gback[c]
            if p.mode == "dense":  # all-to-all of the gathered region: peer q's rows of my slot
                st = p.stride
                for q, pq in enumerate(pipes):
                    back[q * st:(q + 1) * st].copy_(pq.gtables[c][st + r * st: st + (r + 1) * st])
                return
            off = 0
            for q, pq in enumerate(pipes):  # peer q's halo-row gradients of my rows
                cnt = p.send_counts[q]
                if cnt:
                    o = pq.plan.n_loc + sum(pq.plan.recv_counts[:r])
                    back[off:off + cnt].copy_(pq.gtables[c][o:o + cnt])
                off += cnt

        return self._collective(pipe, copies, async_op)


def _run_ranks(fn, world):
    errs = [None] * world

    def body(r):
        try:
            torch.cuda.set_device(DEV)
            with torch.cuda.stream(torch.cuda.Stream(DEV)):  # each rank's own compute stream
                fn(r)
            torch.cuda.synchronize(DEV)
        except BaseException as e:  # reported below; a failed rank must not hang the others
            errs[r] = e
            for grp in _GROUPS:
                grp.barrier.abort()

    ts = [threading.Thread(target=body, args=(r,)) for r in range(world)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=120)
        assert not t.is_alive(), "virtual rank hung"
    for e in errs:
        if e is not None and not isinstance(e, threading.BrokenBarrierError):
            raise e
    for e in errs:
        if e is not None:
            raise e


_GROUPS = []


def _pipes(shards, F, K, async_op, delay):
    grp = Loopback(len(shards), async_op, delay)
    _GROUPS[:] = [grp]
    return [HaloPipeline(sg, F, chunks=K, device=DEV, exchange=grp.member(r)) for r, sg in enumerate(shards)]


def _slow(fn, cycles):
    def wrapped(*a):
        torch.cuda._sleep(cycles)  # a slow gather: on the compute stream, before the real one
        return fn(*a)
    return wrapped


@pytest.mark.parametrize("mode,kind,world,K", [("dense", "er", 2, 2), ("sparse", "er", 2, 2),
                                               ("sparse", "rmat", 3, 4), ("dense", "rmat", 3, 2)])
def test_overlapped_branch_equals_serial(mode, kind, world, K):
    from grl.ops import spmm_backward_slice, spmm_forward_slice

    N, deg, L, F = 8192, 16.0, 6, 128
    g = TypedGraph.synthetic(N, deg, L, kind=kind, seed=5, device=DEV)
    per = -(-N // world)
    bounds = [min(N, r * per) for r in range(world)] + [N]
    shards = ShardedGraph.in_process(g, bounds, halo=mode)
    assert all(sg.plan.mode == mode for sg in shards)
    de = DropEdge(0.3, 4, 1)
    gen = torch.Generator(device=DEV).manual_seed(7)
    Xs = [torch.randn(N, F, generator=gen, device=DEV) for _ in range(2)]
    dZs = [torch.randn(N, (L + 1) * F, generator=gen, device=DEV) for _ in range(2)]

    def rows(t, r):
        return t[bounds[r]:bounds[r + 1]].contiguous()

    # the serial branch (in stream order, no side stream)
    ref_Z = [[None] * world for _ in range(2)]
    ref_dX = [[None] * world for _ in range(2)]
    pipes = _pipes(shards, F, K, async_op=False, delay=0)
    assert all(p.side is None for p in pipes)

    def serial(r):
        for i in range(2):
            Z = torch.empty(bounds[r + 1] - bounds[r], (L + 1) * F, device=DEV)
            ref_Z[i][r] = pipes[r].run(rows(Xs[i], r), Z, de).clone()
            ref_dX[i][r] = pipes[r].backward(rows(dZs[i], r), de).clone()

    _run_ranks(serial, world)
    # the serial branch is the sharded path the gloo / CPU tests pin: Z rows = the one-GPU graph's
    Zg = [torch.cat([ref_Z[i][r] for r in range(world)]) for i in range(2)]
    from grl.ops import spmm_forward

    for i in range(2):
        assert torch.equal(Zg[i], spmm_forward(Xs[i], g.with_dropedge(de)))

    for where in ("exchange", "compute"):
        pipes = _pipes(shards, F, K, async_op=True, delay=SPIN if where == "exchange" else 0)
        assert all(p.side is not None for p in pipes)
        slow = SPIN if where == "compute" else 0
        agg = _slow(lambda t, gg, out, c0: spmm_forward_slice(t, gg, out, c0), slow) if slow else None
        bwd = _slow(spmm_backward_slice, slow) if slow else None
        got_Z = [[None] * world for _ in range(2)]
        got_dX = [[None] * world for _ in range(2)]

        def overlapped(r):
            X_in = torch.empty(bounds[r + 1] - bounds[r], F, device=DEV)
            dZ_in = torch.empty(bounds[r + 1] - bounds[r], (L + 1) * F, device=DEV)
            Zb = [torch.full((bounds[r + 1] - bounds[r], (L + 1) * F), float("nan"), device=DEV) for _ in range(2)]
            dXb = []
            for i in range(2):  # back to back, the same pipeline buffers, different X
                if slow:
                    torch.cuda._sleep(SPIN)  # X_in becomes final late on the compute stream
                X_in.copy_(rows(Xs[i], r))
                pipes[r].run(X_in, Zb[i], de, aggregate_slice=agg)
                if slow:
                    torch.cuda._sleep(SPIN)
                dZ_in.copy_(rows(dZs[i], r))
                dXb.append(pipes[r].backward(dZ_in, de, backward_slice=bwd))
            torch.cuda.synchronize(DEV)
            for i in range(2):
                got_Z[i][r], got_dX[i][r] = Zb[i], dXb[i]

        _run_ranks(overlapped, world)
        for i in range(2):
            for r in range(world):
                assert torch.equal(got_Z[i][r], ref_Z[i][r]), (where, i, r)
                assert torch.equal(got_dX[i][r], ref_dX[i][r]), (where, i, r)


def test_in_process_shards_match_one_graph():
    """ShardedGraph.in_process: each shard's rows aggregate to the one-GPU
    graph's rows through the product's exchange-then-aggregate form."""
    from grl.ops import spmm_forward

    N, L, F = 3000, 6, 64
    g = TypedGraph.synthetic(N, 12.0, L, seed=2, device=DEV)
    X = torch.randn(N, F, device=DEV)
    ref = spmm_forward(X, g)
    bounds = [0, 1000, 2200, N]
    for mode in ("sparse", "dense"):
        for r, sg in enumerate(ShardedGraph.in_process(g, bounds, halo=mode)):
            p = sg.plan
            X_ext = torch.zeros(p.n_loc + p.n_halo, F, device=DEV)
            X_ext[: p.n_loc] = X[bounds[r]:bounds[r + 1]]
            if mode == "dense":
                for q in range(3):
                    X_ext[p.stride * (1 + q): p.stride * (1 + q) + bounds[q + 1] - bounds[q]] = X[bounds[q]:bounds[q + 1]]
            else:
                X_ext[p.n_loc:] = X[p.halo_ids]
            assert torch.equal(spmm_forward(X_ext, sg.graph), ref[bounds[r]:bounds[r + 1]]), (mode, r)
