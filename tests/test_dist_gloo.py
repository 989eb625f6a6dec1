"""Multi-process (gloo, CPU) test of the node-range sharding path in
grl/dist.py: halo plan, all-to-all-v exchange forward and backward, global
DropEdge ids.  Local aggregation inside each rank is the CPU oracle (the HIP
kernels need a GPU); the product's plan/exchange code is what is tested.
Sharded forward must equal the single-process result BITWISE; sharded
dX within 1e-5 (partial sums from different ranks add in peer order)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from grl.dist import build_halo_plan, halo_exchange
from oracle import c_oracle
from oracle import hash as ohash

N, L, F, DEG, SEED = 240, 6, 12, 9.0, 5
DROP = (0.3, 77, 2)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


class _OracleAggregate(torch.autograd.Function):
    """Test-only stand-in for grl.ops.typed_aggregate on CPU tensors."""

    @staticmethod
    def forward(ctx, X, rowptr, colidx, ncols, self_rows, ebase, sbase, d):
        Z = c_oracle.spmm_fwd(rowptr, colidx, X.detach().numpy(), L, True, d=d, edge_base=ebase, self_base=sbase)
        ctx.args = (rowptr, colidx, ncols, self_rows, ebase, sbase, d)
        return torch.from_numpy(Z)

    @staticmethod
    def backward(ctx, dZ):
        rowptr, colidx, ncols, self_rows, ebase, sbase, d = ctx.args
        colptr, zrow, eid, _ = c_oracle.csr_to_csc(rowptr, colidx, L, ncols, True)
        dX = c_oracle.spmm_bwd(colptr, zrow, eid, dZ.contiguous().numpy(), L, F, self_rows, True, d=d,
                               edge_base=ebase, self_base=sbase)
        return (torch.from_numpy(dX),) + (None,) * 7


def _reference():
    rowptr, colidx = ohash.synth_csr(0, L, N, int(N * DEG), SEED)
    X = np.random.default_rng(1).standard_normal((N, F)).astype(np.float32)
    dZ = np.random.default_rng(2).standard_normal((N, (L + 1) * F)).astype(np.float32)
    d = c_oracle.drop(*DROP, True)
    Z = c_oracle.spmm_fwd(rowptr, colidx, X, L, True, d=d)
    colptr, zrow, eid, _ = c_oracle.csr_to_csc(rowptr, colidx, L, N, True)
    dX = c_oracle.spmm_bwd(colptr, zrow, eid, dZ, L, F, N, True, d=d, self_base=int(rowptr[-1]))
    return rowptr, colidx, X, dZ, Z, dX


def _worker(rank, world, port, bounds, mode):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rowptr, colidx, X, dZ, Zref, dXref = _reference()
        rb, re = bounds[rank], bounds[rank + 1]
        lr = rowptr[rb * L:re * L + 1] - rowptr[rb * L]
        lc = colidx[rowptr[rb * L]:rowptr[re * L]]
        plan = build_halo_plan(torch.from_numpy(lc.copy()), rb, re, mode=mode)
        # referenced/remote rows: 99% ([0,120,240]), 93% ([0,50,170,240]), 50% (empty shard) -> auto at 75%
        assert plan.mode == (mode if mode != "auto" else ("sparse" if bounds[1] == 0 else "dense"))
        assert plan.rank == rank
        assert plan.edge_id_base == int(rowptr[rb * L]) and plan.num_edges_total == colidx.size
        # every halo id is remote and referenced; slots are in owner order
        assert not ((plan.halo_ids >= rb) & (plan.halo_ids < re)).any()
        # the in-process builder (every shard's plan in one process, no collective) gives this rank's plan
        from grl.dist import build_halo_plans_local

        cols = [torch.from_numpy(colidx[rowptr[bounds[q] * L]:rowptr[bounds[q + 1] * L]].copy())
                for q in range(world)]
        local = build_halo_plans_local(cols, bounds, mode=mode)[rank]
        for f in ("row_begin", "row_end", "n_loc", "n_halo", "bounds", "send_counts", "recv_counts",
                  "edge_id_base", "num_edges_total", "mode", "stride", "rank"):
            assert getattr(local, f) == getattr(plan, f), f
        for f in ("send_index", "halo_ids", "colidx_local"):
            assert torch.equal(getattr(local, f), getattr(plan, f)), f
        X_loc = torch.from_numpy(X[rb:re].copy()).requires_grad_(True)
        X_ext = halo_exchange(X_loc, plan)
        # every column resolves to the right global feature row, whatever the layout
        np.testing.assert_array_equal(X_ext[plan.colidx_local.long()].detach().numpy(), X[lc])
        if plan.mode == "sparse":
            np.testing.assert_array_equal(X_ext[plan.n_loc:].detach().numpy(), X[plan.halo_ids.numpy()])
        d = c_oracle.drop(*DROP, True)
        Z = _OracleAggregate.apply(X_ext, lr, plan.colidx_local.numpy(), plan.n_loc + plan.n_halo, plan.n_loc,
                                   plan.edge_id_base, plan.num_edges_total + rb, d)
        np.testing.assert_array_equal(Z.detach().numpy(), Zref[rb:re])  # bitwise: same rows, same edge order
        Z.backward(torch.from_numpy(dZ[rb:re].copy()))
        np.testing.assert_allclose(X_loc.grad.numpy(), dXref[rb:re], rtol=0, atol=1e-5)
        _check_pipeline(plan, lr, X[rb:re], Zref[rb:re], rb, d, dZ[rb:re], X_loc.grad)
    finally:
        dist.destroy_process_group()


class _HostGraph:
    """Test double for the TypedGraph a ShardedGraph carries (the real one
    lives on the GPU); HaloPipeline only asks it for with_dropedge."""

    def __init__(self):
        self.device = torch.device("cpu")

    def with_dropedge(self, de):
        return self


def _check_pipeline(plan, lr, X_loc, Zref, rb, d, dZ_loc, dX_sharded):
    """grl.dist.HaloPipeline's slice tables and exchanges (product code),
    each slice aggregated by the oracle: Z bitwise equal to one process; the
    pipelined backward (slice gathers + reverse exchanges + peer-order
    combine) bitwise equal to the unsliced sharded backward."""
    import types

    from grl.dist import HaloPipeline

    sg = types.SimpleNamespace(plan=plan, graph=_HostGraph(), group=None)
    n = plan.n_loc
    for K in (1, 2, 3):
        pipe = HaloPipeline(sg, F, chunks=K, device="cpu")
        assert pipe.side is None and pipe.tables.shape == (K, plan.n_loc + plan.n_halo, F // K)
        Z = torch.full((n, (L + 1) * F), float("nan"))

        def agg(table, graph, out, col0):
            Zc = c_oracle.spmm_fwd(lr, plan.colidx_local.numpy(), table.numpy(), L, True, d=d,
                                   edge_base=plan.edge_id_base, self_base=plan.num_edges_total + rb)
            out.view(n, L + 1, F)[:, :, col0:col0 + table.shape[1]] = torch.from_numpy(Zc).view(n, L + 1, table.shape[1])

        pipe.run(torch.from_numpy(X_loc.copy()), Z, None, aggregate_slice=agg)
        np.testing.assert_array_equal(Z.numpy(), Zref)

        ncols = plan.n_loc + plan.n_halo
        colptr, zrow, eid, _ = c_oracle.csr_to_csc(lr, plan.colidx_local.numpy(), L, ncols, True)

        def bwd(dZ, graph, col0, out):
            Fc = out.shape[1]
            dZc = np.ascontiguousarray(dZ.numpy().reshape(n, L + 1, F)[:, :, col0:col0 + Fc]).reshape(n, (L + 1) * Fc)
            out.copy_(torch.from_numpy(c_oracle.spmm_bwd(colptr, zrow, eid, dZc, L, Fc, n, True, d=d,
                                                         edge_base=plan.edge_id_base,
                                                         self_base=plan.num_edges_total + rb)))

        for _ in range(2):  # the second call reuses the gradient buffers
            dX = pipe.backward(torch.from_numpy(dZ_loc.copy()), None, backward_slice=bwd)
            np.testing.assert_array_equal(dX.numpy(), dX_sharded.numpy())


@pytest.mark.parametrize("mode", ["auto", "sparse", "dense"])
@pytest.mark.parametrize("bounds", [[0, 120, 240], [0, 50, 170, 240], [0, 0, 100, 240], [0, 0, 0, 240]])
def test_sharded_equals_single_process(bounds, mode):
    world = len(bounds) - 1
    mp.spawn(_worker, args=(world, _free_port(), bounds, mode), nprocs=world, join=True)


def _loopback_worker(rank, world, port, mode):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from rccl_loopback import loopback_plan

        rowptr, colidx, X, dZ, Zref, dXref = _reference()
        plan = loopback_plan(torch.from_numpy(colidx.copy()), N, mode)
        X_loc = torch.from_numpy(X.copy()).requires_grad_(True)
        X_ext = halo_exchange(X_loc, plan)  # a one-rank group with halo rows still exchanges them
        assert X_ext.shape[0] == N + plan.n_halo
        np.testing.assert_array_equal(X_ext[plan.colidx_local.long()].detach().numpy(), X[colidx])
        assert (plan.colidx_local >= N).all()  # every source row came through the collective
        d = c_oracle.drop(*DROP, True)
        Z = _OracleAggregate.apply(X_ext, rowptr, plan.colidx_local.numpy(), N + plan.n_halo, N, 0,
                                   int(colidx.size), d)
        np.testing.assert_array_equal(Z.detach().numpy(), Zref)
        Z.backward(torch.from_numpy(dZ.copy()))
        np.testing.assert_allclose(X_loc.grad.numpy(), dXref, rtol=0, atol=1e-5)
        _check_pipeline(plan, rowptr, X, Zref, 0, d, dZ, X_loc.grad)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["dense", "sparse"])
def test_one_rank_loopback_plan_exchanges(mode):
    """The loopback plans of tests/rccl_loopback.py (what the one-GPU box runs
    on real RCCL) through the product's exchange on a one-rank gloo group:
    Z bitwise one process, dX within fp32 rounding (the edge sums come back
    as a peer's partial), the sliced pipeline bitwise the unsliced exchange."""
    mp.spawn(_loopback_worker, args=(1, _free_port(), mode), nprocs=1, join=True)


def test_single_shard_plan_is_identity():
    rowptr, colidx = ohash.synth_csr(0, L, 50, 300, 1)
    plan = build_halo_plan(torch.from_numpy(colidx), 0, 50)
    assert plan.n_halo == 0 and torch.equal(plan.colidx_local, torch.from_numpy(colidx))
    X = torch.randn(50, 4)
    assert torch.equal(halo_exchange(X, plan), X)


def test_edge_balanced_bounds():
    from grl.dist import edge_balanced_bounds

    src, _, _ = ohash.synth_edges(1, 6, 1 << 12, (1 << 12) * 20, 9)
    deg = torch.from_numpy(np.bincount(src, minlength=1 << 12).astype(np.int32))
    for world in (2, 4, 8):
        b = edge_balanced_bounds(deg, world)
        assert b[0] == 0 and b[-1] == deg.numel() and b == sorted(b)
        loads = [int(deg[b[i]:b[i + 1]].sum()) for i in range(world)]
        # every shard within one max-degree row of the ideal E/P
        assert max(loads) - min(loads) <= 2 * int(deg.max()) + 1, loads
    b = edge_balanced_bounds(torch.zeros(5, dtype=torch.int32), 3)  # degenerate: no edges at all
    assert b[0] == 0 and b[-1] == 5 and b == sorted(b) and len(b) == 4


def _allreduce_worker(rank, world, port):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from grl.dist import allreduce_gradients

        ps = [torch.nn.Parameter(torch.zeros(s)) for s in [(7, 3), (5,), (1000,), (2, 2)]]
        for i, p in enumerate(ps):
            p.grad = torch.full_like(p, float(rank + 1) * (i + 1))
        ps[3].grad = None  # parameters without a gradient are skipped
        allreduce_gradients(ps, bucket_bytes=4 * 40)  # forces several buckets
        tot = sum(r + 1 for r in range(world))
        for i, p in enumerate(ps[:3]):
            assert torch.equal(p.grad, torch.full_like(p, float(tot * (i + 1))))
        assert ps[3].grad is None
        q = torch.nn.Parameter(torch.zeros(3))
        q.grad = torch.full((3,), float(rank + 1))
        allreduce_gradients([q], average=True)
        assert torch.allclose(q.grad, torch.full((3,), tot / world))
        from grl.dist import broadcast_module

        m = torch.nn.Linear(3, 2)
        torch.nn.init.constant_(m.weight, float(rank))
        broadcast_module(m, src=0)
        assert torch.equal(m.weight, torch.zeros(2, 3))
    finally:
        dist.destroy_process_group()


def test_allreduce_gradients_buckets():
    mp.spawn(_allreduce_worker, args=(3, _free_port()), nprocs=3, join=True)


def _agree_worker(rank, world, port):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import types

        from grl import dist as gdist
        from grl import ops

        # rows_backward: one rank's block is outside the one-kernel path -> EVERY rank returns None before any
        # point-to-point transfer is posted (they then all run the unpipelined exchange: matching collectives)
        plan = types.SimpleNamespace(bounds=[0, 10, 20, 30], rank=rank, mode="dense", stride=10, n_loc=10,
                                     recv_counts=[0] * 3, send_counts=[0] * 3)
        sg = types.SimpleNamespace(plan=plan, group=None, graph=types.SimpleNamespace(_shared={}))
        sg.halo_blocks = types.MethodType(gdist.ShardedGraph.halo_blocks, sg)
        orig_views, orig_rows = ops.graph_conv_bwd_data_rows_views, ops.graph_conv_bwd_data_rows
        try:
            ops.graph_conv_bwd_data_rows_views = lambda *a, **k: None if rank == 1 else ["eligible"]

            def no_launch(*a, **k):
                raise AssertionError("launched although a peer fell back")

            ops.graph_conv_bwd_data_rows = no_launch
            g = torch.zeros(10, 4)
            assert gdist.ShardedGraph.rows_backward(sg, g, None, 4, types.SimpleNamespace(num_cols=40)) is None
        finally:
            ops.graph_conv_bwd_data_rows_views, ops.graph_conv_bwd_data_rows = orig_views, orig_rows
        assert gdist._all_agree(True, None, None) and not gdist._all_agree(rank != 2, None, None)
        # the dense blocks are every peer's gathered slot in rotation order
        assert [q for q, _, _ in sg.halo_blocks()] == [(rank + 1) % 3, (rank + 2) % 3]
        # point-to-point inside a SUBGROUP: peers are group ranks (global rank q + 1 here)
        sub = dist.new_group([1, 2])
        if rank in (1, 2):
            me = dist.get_rank(sub)
            peer = 1 - me
            send = torch.full((3,), float(rank))
            recv = torch.empty(3)
            works, finish = gdist._p2p_exchange([(send, peer)], [(recv, peer)], sub)
            for w in works:
                w.wait()
            finish()
            assert torch.equal(recv, torch.full((3,), float(3 - rank)))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_rows_backward_fallback_is_collective_and_p2p_uses_group_ranks():
    """rows_backward's choice between the row-pipelined
    point-to-point backward and the unpipelined exchange is agreed by all
    ranks before anything is posted (a rank whose block cannot take the
    one-kernel path makes every rank fall back), and point-to-point peers are
    ranks of the shard's group, also under a subgroup."""
    mp.spawn(_agree_worker, args=(3, _free_port()), nprocs=3, join=True)


def _memo_worker(rank, world, port, mode):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from grl import dist as gdist

        gen = torch.Generator().manual_seed(11)
        N, L = 40, 2
        cols = torch.randint(0, N, (N * L * 3,), generator=gen)
        rowptr_g = torch.arange(0, N * L * 3 + 1, 3, dtype=torch.int64)
        rb, re = (0, 22) if rank == 0 else (22, N)
        e0, e1 = int(rowptr_g[rb * L]), int(rowptr_g[re * L])
        sg = gdist.ShardedGraph.__new__(gdist.ShardedGraph)  # the exchange needs only the plan (no device graph)
        sg.group, sg.plan = None, build_halo_plan(cols[e0:e1], rb, re, None, mode=mode)
        n = re - rb
        g1 = torch.randn(n, 8, generator=torch.Generator().manual_seed(100 + rank))
        g2 = torch.randn(n, 8, generator=torch.Generator().manual_seed(200 + rank))
        calls = {"n": 0}
        orig_ag, orig_a2a = gdist.all_gather_into, gdist.all_to_all_v

        def count_ag(*a, **k):
            calls["n"] += 1
            return orig_ag(*a, **k)

        def count_a2a(*a, **k):
            calls["n"] += 1
            return orig_a2a(*a, **k)

        gdist.all_gather_into, gdist.all_to_all_v = count_ag, count_a2a
        try:
            x3 = torch.cat([g1, g2], dim=-1)
            want = sg.exchange(x3)  # the concat exchanged as itself
            m = sg.with_halo_memo().with_dropedge(None)  # copies share the memo
            m.remember(g1)
            t1 = m.exchange_table(g1.view(1, n, 8))  # a 3-D view is the same tensor
            assert torch.equal(t1, sg.exchange(g1))
            m.note_concat(x3, (g1, g2))
            before = calls["n"]
            t3 = m.exchange_table(x3)
            assert calls["n"] == before + 1  # only g2's rows travelled
            assert torch.equal(t3, want)
            m.clear_halo_memo()
            before = calls["n"]
            assert torch.equal(m.exchange_table(x3), want) and calls["n"] == before + 1  # no memo: x3 itself
            assert sg.halo_memo is None and torch.equal(sg.exchange_table(g1), t1)  # the original has no memo
        finally:
            gdist.all_gather_into, gdist.all_to_all_v = orig_ag, orig_a2a
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["dense", "sparse"])
def test_halo_memo_reuses_concat_parts(mode):
    """GraphCNNDropEdge's gcn3 input cat[g1, g2] on a shard: with the
    per-forward halo memo only g2's rows travel (g1's table came for gcn2),
    and the assembled table equals the concat's own exchange."""
    mp.spawn(_memo_worker, args=(2, _free_port(), mode), nprocs=2, join=True)


@pytest.mark.parametrize("seed", range(6))
def test_stream_chunks_schedule(seed):
    """The streamed inference schedule (grl.dist.stream_chunks): compute
    chunks tile the shard's rows in order, every rank posts the same blocks
    in the same order, a block is posted only after its rows are computed,
    and a chunk takes the whole shard's GEMM path (so the layer's bits do
    not depend on the blocking)."""
    from grl.dist import stream_chunks

    rng = np.random.default_rng(seed)
    for _ in range(200):
        stride = int(rng.integers(1, 400))
        n_loc = int(rng.integers(0, stride + 1))
        nb = int(rng.integers(1, 6))
        thr = int(rng.integers(1, 300))
        ok = lambda m: m >= thr  # noqa: E731  (x6_rows_ok is monotone in the row count)
        sched = stream_chunks(stride, n_loc, nb, ok)
        bs = -(-stride // nb)
        parts = [(j * bs, min((j + 1) * bs, stride)) for j in range(nb) if j * bs < stride]
        assert [b for _, _, posts in sched for b in posts] == parts
        assert sched[0][0] == 0 and sched[-1][1] == n_loc
        assert all(a[1] == b[0] for a, b in zip(sched, sched[1:]))
        for r0, r1, posts in sched:
            assert all(min(a1, n_loc) <= r1 for _, a1 in posts)
            if r1 > r0:
                assert ok(r1 - r0) == ok(n_loc)
        if not ok(n_loc):
            assert sum(1 for r0, r1, _ in sched if r1 > r0) <= 1


def _stream_worker(rank, world, port, mode):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from grl import dist as gdist

        gen = torch.Generator().manual_seed(5)
        N, L, deg = 60, 2, 3
        cols = torch.randint(0, N, (N * L * deg,), generator=gen)
        bounds = [0, 25, 37, N]  # unequal shards: blocks past a short shard's end carry no rows
        rb, re = bounds[rank], bounds[rank + 1]
        e0, e1 = rb * L * deg, re * L * deg
        sg = gdist.ShardedGraph.__new__(gdist.ShardedGraph)  # the posts need only the plan (no device graph)
        sg.group, sg.plan = None, build_halo_plan(cols[e0:e1], rb, re, None, mode=mode)
        assert sg.plan.mode == mode
        X = torch.randn(re - rb, 8, generator=torch.Generator().manual_seed(100 + rank))
        want = halo_exchange(X, sg.plan)
        # K so large that any run of >= 5 rows takes the x6 path: the schedule then cuts into several chunks
        for nb in (1, 2, 3, 5):
            sg.stream_blocks = nb
            T = sg._stream_table(8, X)
            seen = []
            works = sg._stream_fill(T, 8, 200_000_000,
                                    lambda r0, r1: (seen.append((r0, r1)), T[r0:r1].copy_(X[r0:r1])))
            for w in works:
                if w is not None:
                    w.wait()
            assert torch.equal(T, want), (rank, mode, nb)
            assert seen[0][0] == 0 and seen[-1][1] == re - rb and (nb == 1 or rank != 0 or len(seen) > 1), seen
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["dense", "sparse"])
def test_streamed_blocks_fill_the_halo_table(mode):
    """Streamed inference's posts (ShardedGraph._stream_fill / _post_block):
    a layer's output rows sent block by block as they are computed -- an
    all-gather per block (dense halos) or an all-to-all-v of the rows each
    peer asked for (sparse) -- fill the next layer's table exactly as the
    whole-tensor halo exchange does, on unequal shards, for 1..5 blocks."""
    mp.spawn(_stream_worker, args=(3, _free_port(), mode), nprocs=3, join=True)
