"""GPU: the drop-in GraphCNNDropEdge over a node-range-sharded graph
(verdict r3 item 5, r4 items 1-3; drop_robust_gcn.py:61-103,
robust_gcn.py:45-51, 78-96).

Every rank runs model.forward([V_rows_of_this_rank, ShardedGraph]) --
emb1 / emb2 / the random projection / the classifier row-local, every
GraphConv on the shard (halo exchange; training: the one-kernel forms with
the reverse exchange pipelined over row blocks), NodeSelfAtten with the
softmax over every node, feature dropout 0.5 and DropEdge 0.3 on -- then
backward and allreduce_gradients, then the inference forward (streamed by
row blocks and plain).  The ranks run two ways, on the box's one GPU:
  * gloo processes -- the host-staged branches of grl.dist;
  * threads of this process over a grl.dist.LocalGroup -- the device
    branches RCCL takes on a multi-GPU node (async handles, slot views,
    landing copies, the device MIN all-reduce, point-to-point row blocks),
    which RCCL cannot run with two ranks on one device.
Against the one-GPU model on the whole graph with the same weights, the
same DropEdge and feature-dropout masks (hashes of global edge / element
ids): every GraphConv output row, the logits and the inference logits
BITWISE (every row-local op's arithmetic is independent of the row count:
the GEMM paths sum K in fixed chunks and are chosen for the whole graph's
rows, the attention's key split depends on N only); every parameter
gradient within 1e-4 of its scale (the ranks' partial sums are added in
another order).  The two rank drivers agree bitwise on the logits and the
GraphConv rows, and on the gradients (2 ranks; 3 ranks: 1e-6, gloo's
all-reduce order)."""
import copy
import os
import socket
import threading

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
L, FIN, OUT = 6, 96, 7


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _inputs(world, n_per_rank, balance):
    from grl import TypedGraph
    from grl.dist import edge_balanced_bounds

    N = n_per_rank * world
    g = TypedGraph.synthetic(N, 12.0, L, kind="er", seed=4, device=DEV)
    if balance == "edges":
        bounds = edge_balanced_bounds((g.rowptr[L::L] - g.rowptr[:-1:L]).to(torch.int64), world)
    else:
        per = -(-N // world)
        bounds = [min(N, r * per) for r in range(world + 1)]
    gen = torch.Generator().manual_seed(5)
    V = (torch.rand(N, FIN, generator=gen) < 0.1).float().to(DEV)  # bag-of-chars-like rows
    y = torch.randint(0, OUT, (N,), generator=gen).to(DEV)
    return g, bounds, V, y


def _model(net_size):
    from gnn.models import GraphCNNDropEdge

    torch.manual_seed(0)
    m = GraphCNNDropEdge(FIN, OUT, L, net_size=net_size, dropedge_seed=3).to(DEV)
    assert m.dropout.p == 0.5 and m.edge_dropout.p == 0.3  # both dropouts on
    return m


def _run_rank(model, V_rows, A, y_rows, allreduce=None):
    """train forward + backward (+ the gradient all-reduce), then the
    inference forward (a ShardedGraph: plain, streamed in 2 and 3 blocks).
    Returns CPU copies of everything compared."""
    seen = {}

    def record(name, orig):  # the model calls GraphConv.propagate (module hooks do not see it)
        def fn(*a, **k):
            out = orig(*a, **k)
            seen.setdefault(name, out.detach().reshape(-1, out.shape[-1]).clone())
            return out
        return fn

    for name in ("gcn1", "gcn2", "gcn3"):
        mod = getattr(model, name)
        mod.propagate = record(name, mod.propagate)
    model.train()
    model.zero_grad(set_to_none=True)
    model.edge_dropout.reset_calls()
    model.dropout.reset_calls()
    logits = model.forward([V_rows, A]).reshape(-1, OUT)
    loss = torch.nn.functional.cross_entropy(logits, y_rows, reduction="sum")
    loss.backward()
    if allreduce is not None:
        allreduce([p for p in model.parameters() if p.requires_grad])
    res = {"logits": logits.detach().cpu(), "gcn": {k: v.cpu() for k, v in seen.items()},
           "grads": {k: p.grad.detach().cpu() for k, p in model.named_parameters() if p.grad is not None}}
    from grl.dist import ShardedGraph

    if isinstance(A, ShardedGraph):  # the training forward without streaming its layers' rows: the same bits
        model.edge_dropout.reset_calls()
        model.dropout.reset_calls()
        A.stream_rows = False
        res["logits_unstreamed"] = model.forward([V_rows, A]).reshape(-1, OUT).detach().cpu()
        A.stream_rows = True
    model.eval()
    with torch.no_grad():
        from grl.dist import ShardedGraph

        if isinstance(A, ShardedGraph):
            for tag, on, nb in (("plain", False, 2), ("streamed2", True, 2), ("streamed3", True, 3)):
                A.stream_rows, A.stream_blocks = on, nb
                res["eval_" + tag] = model.forward([V_rows, A]).reshape(-1, OUT).cpu()
            A.stream_rows, A.stream_blocks = True, 2
        else:
            res["eval_plain"] = model.forward([V_rows, A]).reshape(-1, OUT).cpu()
    torch.cuda.synchronize()
    return res


def _gloo_worker(rank, world, port, mode, net_size, n_per_rank, balance, out_dir):
    import torch.distributed as dist

    from grl.dist import ShardedGraph, allreduce_gradients

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        g, bounds, V, y = _inputs(world, n_per_rank, balance)
        sg = ShardedGraph.from_graph(g, balance=balance, halo=mode)
        assert [sg.plan.row_begin, sg.plan.row_end] == bounds[rank:rank + 2]
        rb, re = bounds[rank], bounds[rank + 1]
        res = _run_rank(_model(net_size), V[rb:re], sg, y[rb:re], allreduce_gradients)
        torch.save(res, os.path.join(out_dir, f"gloo{rank}.pt"))
    finally:
        dist.destroy_process_group()


def _thread_ranks(world, mode, net_size, n_per_rank, balance):
    """The P ranks as threads over a LocalGroup (each its own compute stream,
    backward on the calling thread)."""
    from grl.dist import LocalGroup, ShardedGraph, allreduce_gradients

    g, bounds, V, y = _inputs(world, n_per_rank, balance)
    grp = LocalGroup(world)
    shards = ShardedGraph.in_process(g, bounds, halo=mode, group=grp)
    base = _model(net_size)
    replicas = [copy.deepcopy(base) for _ in range(world)]
    res, errs = [None] * world, [None] * world

    def body(r):
        try:
            torch.cuda.set_device(DEV)
            rb, re = bounds[r], bounds[r + 1]
            with torch.autograd.set_multithreading_enabled(False), torch.cuda.stream(torch.cuda.Stream(DEV)):
                res[r] = _run_rank(replicas[r], V[rb:re], shards[r], y[rb:re],
                                   lambda ps: allreduce_gradients(ps, group=shards[r].group))
        except BaseException as e:  # reported below; a failed rank must not hang the others
            errs[r] = e
            grp.abort()

    ts = [threading.Thread(target=body, args=(r,)) for r in range(world)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(240)
        assert not t.is_alive(), "virtual rank hung"
    for e in errs:
        if e is not None and not isinstance(e, threading.BrokenBarrierError):
            raise e
    for e in errs:
        if e is not None:
            raise e
    return res, g, bounds, V, y


@pytest.mark.parametrize("world,mode,net_size,n_per_rank,balance", [
    (2, "dense", 64, 3000, "nodes"),      # small shards: the two-kernel layer, unpipelined reverse exchange
    (3, "sparse", 64, 2500, "edges"),
    (3, "dense", 64, 2500, "edges"),
    (3, "sparse", 64, 2500, "nodes"),
    (2, "sparse", 64, 3000, "edges"),
    (2, "dense", 256, 20_000, "nodes"),   # one-kernel forward / data gradient, p2p row blocks in the backward
    (3, "sparse", 256, 20_000, "nodes"),
    (4, "sparse", 64, 2_000, "edges"),      # four ranks: every rank both sends and receives from three peers
])
def test_sharded_model_equals_one_gpu(world, mode, net_size, n_per_rank, balance, tmp_path):
    import torch.multiprocessing as mp

    mp.spawn(_gloo_worker, args=(world, _free_port(), mode, net_size, n_per_rank, balance, str(tmp_path)),
             nprocs=world, join=True)
    gloo = [torch.load(os.path.join(tmp_path, f"gloo{r}.pt"), weights_only=True) for r in range(world)]
    threads, g, bounds, V, y = _thread_ranks(world, mode, net_size, n_per_rank, balance)
    one = _run_rank(_model(net_size), V[None], g, y)
    bad = []
    for r in range(world):
        rb, re = bounds[r], bounds[r + 1]
        for tag, got in (("threads", threads[r]), ("gloo", gloo[r])):
            for k in ("gcn1", "gcn2", "gcn3"):
                if not torch.equal(got["gcn"][k], one["gcn"][k][rb:re]):
                    bad.append((r, tag, k, float((got["gcn"][k] - one["gcn"][k][rb:re]).abs().max())))
            for k in ("logits", "logits_unstreamed", "eval_plain", "eval_streamed2", "eval_streamed3"):
                want = one["logits" if k.startswith("logits") else "eval_plain"][rb:re]
                if not torch.equal(got[k], want):
                    bad.append((r, tag, k, float((got[k] - want).abs().max())))
            for k, ga in one["grads"].items():
                gb = got["grads"][k]
                err, lim = float((ga - gb).abs().max()), 1e-4 * max(1.0, float(ga.abs().max()))
                if not err <= lim:
                    bad.append((r, tag, "grad " + k, err, lim))
        for k, ga in gloo[r]["grads"].items():  # the two rank drivers: the same collectives' results
            gb = threads[r]["grads"][k]
            ok = torch.equal(ga, gb) if world == 2 else \
                float((ga - gb).abs().max()) <= 1e-6 * max(1.0, float(ga.abs().max()))
            if not ok:
                bad.append((r, "threads vs gloo", "grad " + k, float((ga - gb).abs().max())))
    assert not bad, bad


def _attn_worker(rank, world, port, N, dk, dv, bounds):
    import torch.distributed as dist

    from grl.dist import ShardedGraph, sharded_node_attention
    from grl.ops import node_self_attention

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import types

        g = torch.Generator().manual_seed(N)
        Q = torch.relu(torch.randn(N, dk, generator=g)).to(DEV)
        K = torch.relu(torch.randn(N, dk, generator=g)).to(DEV)
        H = torch.relu(torch.randn(N, dv, generator=g)).to(DEV)
        V = torch.randn(N, dv, generator=g).to(DEV)
        gm = torch.randn(dv, generator=g).to(DEV)
        dout = torch.randn(N, dv, generator=g).to(DEV)
        one = [t.clone().requires_grad_(True) for t in (Q, K, H, V, gm)]
        out1 = node_self_attention(one[0][None], one[1][None], one[2][None], one[3][None], one[4])[0]
        out1.backward(dout)
        rb, re = bounds[rank], bounds[rank + 1]
        sg = ShardedGraph.__new__(ShardedGraph)  # the attention needs only the row ranges and the group
        sg.group = None
        sg.plan = types.SimpleNamespace(bounds=bounds, row_begin=rb, row_end=re, n_loc=re - rb, rank=rank)
        loc = [t[rb:re].clone().requires_grad_(True) for t in (Q, K, H, V)] + [gm.clone().requires_grad_(True)]
        out2 = sharded_node_attention(*loc, sg)
        out2.backward(dout[rb:re])
        assert float((out2 - out1[rb:re]).abs().max()) <= 1e-5 * max(1.0, float(out1.abs().max())), rank
        for name, a, b in zip("QKHV", one[:4], loc[:4]):
            ga, gb = a.grad[rb:re], b.grad
            err = float((ga - gb).abs().max())
            assert err <= 2e-5 * (float(ga.abs().max()) + 1.0), (rank, name, err, float(ga.abs().max()))
        dgam = loc[4].grad.clone()
        dist.all_reduce(dgam)
        assert float((dgam - one[4].grad).abs().max()) <= 1e-4 * (float(one[4].grad.abs().max()) + 1.0), rank
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,N,dk,dv,bounds", [(3, 7500, 4, 32, [0, 2500, 5000, 7500]),
                                                   (3, 7500, 4, 32, [0, 2491, 5003, 7500]),
                                                   (2, 6000, 16, 128, [0, 3000, 6000])])
def test_sharded_attention_equals_one_gpu(world, N, dk, dv, bounds):
    """NodeSelfAtten over node-range shards (grl.dist.sharded_node_attention:
    all-gathered K / H, ranged kernels, rank-ordered dK / dH reduction)
    against the one-GPU op on the same rows: out, dQ, dK, dH, dV per row and
    the summed dgamma."""
    import torch.multiprocessing as mp

    mp.spawn(_attn_worker, args=(world, _free_port(), N, dk, dv, bounds), nprocs=world, join=True)


def _stream_chain_worker(rank, world, port, mode, nb):
    import torch.distributed as dist

    from gnn.models.networks.robust_gcn import GraphConv
    from grl import DropEdge, TypedGraph
    from grl.dist import ShardedGraph
    from grl.ops import graph_conv_infer

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        N, deg, L, d = 60_000 * world, 12.0, 6, 256
        g = TypedGraph.synthetic(N, deg, L, kind="er", seed=8, device=DEV)
        sg = ShardedGraph.from_graph(g, halo=mode)
        rb, re = sg.plan.row_begin, sg.plan.row_end
        X = torch.randn(N, d, generator=torch.Generator().manual_seed(6)).to(DEV)
        torch.manual_seed(1)
        layers = [GraphConv(d, d, L).to(DEV) for _ in range(3)]
        de = [DropEdge(0.3, 11, c) for c in range(3)]
        with torch.no_grad():
            ref = X  # the one-GPU chain (one-kernel layers over the whole graph)
            for lay, e in zip(layers, de):
                ref = graph_conv_infer(ref, g.with_dropedge(e), lay.h_weights, lay.bias, True)
            got = {}
            for tag, on in (("streamed", True), ("plain", False)):
                m = sg.with_halo_memo()
                m.stream_rows, m.stream_blocks = on, nb
                h = X[rb:re]
                for lay, e in zip(layers, de):
                    h = m.graphconv(h, lay, e, relu=True)
                got[tag] = h.clone()
                m.clear_halo_memo()
        views = sg.graph._shared.get("fwd_row_views", {})
        assert sum(1 for r0, _ in views if r0 > 0) >= nb - 1, sorted(views)  # the layers ran in row blocks
        assert torch.equal(got["streamed"], got["plain"]), (rank, float((got["streamed"] - got["plain"]).abs().max()))
        assert torch.equal(got["streamed"], ref[rb:re]), (rank, float((got["streamed"] - ref[rb:re]).abs().max()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("mode,nb", [("dense", 2), ("dense", 3), ("sparse", 2)])
def test_streamed_layer_chain_equals_one_gpu(mode, nb):
    """Three inference GraphConv layers over 2 shards of 60k rows (one-kernel
    blocks of >= 17.5k rows: the blocks really split): each layer's rows
    streamed to the peers by blocks as they are written (dense all-gather /
    sparse all-to-all-v per block) and the next layer reading the filled
    table -- bitwise the unstreamed sharded chain and the one-GPU chain."""
    import torch.multiprocessing as mp

    mp.spawn(_stream_chain_worker, args=(2, _free_port(), mode, nb), nprocs=2, join=True)


def test_sharded_model_surfaces_a_poisoned_kernel(monkeypatch, grl_option):
    """Stream-ordered failures of the persistent GraphConv kernel reach the
    caller of the sharded model with no procedure around it: the inference
    forward checks once at its end, and allreduce_gradients (the training
    step's sync point, before any optimizer step) checks the step's kernels
    -- both raise GrlError naming the entry point instead of returning NaN."""
    import grl
    from grl import _lib
    from grl.dist import LocalGroup, ShardedGraph, allreduce_gradients

    g, bounds, V, y = _inputs(1, 20_000, "nodes")
    sg = ShardedGraph.in_process(g, bounds, halo="dense", group=LocalGroup(1))[0]
    m = _model(256)
    grl.check()
    grl_option("ws_spin", 1)
    m.eval()
    with torch.no_grad(), pytest.raises(_lib.GrlError, match="grl_graphconv"):
        m.forward([V, sg])
    m.train()
    logits = m.forward([V, sg]).reshape(-1, OUT)
    torch.nn.functional.cross_entropy(logits, y, reduction="sum").backward()
    with pytest.raises(_lib.GrlError, match="grl_graphconv"):
        allreduce_gradients([p for p in m.parameters() if p.requires_grad], group=sg.group)
    grl_option("ws_spin", 0)
    torch.cuda.synchronize()
    grl.check()
