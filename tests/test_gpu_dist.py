"""GPU, single process: the sharded path degenerates to the plain one at
world size 1 (no process group), through the same code the N-GPU bench runs."""
import pytest
import torch

from grl import DropEdge, TypedGraph
from grl.dist import ShardedGraph, halo_exchange_into
from grl.ops import spmm_forward, typed_aggregate

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def test_world1_shard_equals_plain_graph():
    sg = ShardedGraph.synthetic(5000, 12.0, 6, seed=3, device=DEV)
    g = TypedGraph.synthetic(5000, 12.0, 6, seed=3, device=DEV)
    assert sg.halo_rows == 0 and torch.equal(sg.graph.colidx, g.colidx)
    X = torch.randn(5000, 64, device=DEV, requires_grad=True)
    de = DropEdge(0.3, 9, 1)
    Z1 = sg.aggregate(X, de)
    Z2 = typed_aggregate(X, g.with_dropedge(de))
    assert torch.equal(Z1, Z2)
    (dx1,) = torch.autograd.grad(Z1, X, torch.ones_like(Z1))
    (dx2,) = torch.autograd.grad(Z2, X, torch.ones_like(Z2))
    assert torch.equal(dx1, dx2)
    out = torch.empty_like(Z2)
    halo_exchange_into(X.detach(), X.detach(), torch.empty(0, 64, device=DEV), sg.plan)
    spmm_forward(X.detach(), sg.graph.with_dropedge(de), out=out)
    assert torch.equal(out, Z2)


@pytest.mark.parametrize("kind,F,slices", [("er", 256, (128, 128)), ("er", 256, (64, 64, 128)),
                                           ("rmat", 512, (128, 256, 128)), ("er", 100, (52, 48)),
                                           ("er", 100, (50, 50))])
def test_column_slices_equal_whole_aggregation(kind, F, slices):
    """grl_typed_spmm_fwd_slice: each column slice of Z from its own slice
    table (row stride = slice width), self rows at an offset, bitwise equal
    to the whole-width aggregation -- DropEdge on, R-MAT hub rows split."""
    from grl.ops import spmm_forward_slice

    N = 1 << 13
    g = TypedGraph.synthetic(N, 48.0, 6, kind=kind, seed=8, device=DEV)
    g.split_threshold, g.split_chunk = 256, 128  # force the hub-chunk path at this size
    de = DropEdge(0.3, 4, 2)
    X = torch.randn(N, F, device=DEV)
    Zw = spmm_forward(X, g.with_dropedge(de))
    Zs = torch.full_like(Zw, float("nan"))
    c0 = 0
    for w in slices:
        table = torch.zeros(N + 7, w, device=DEV)  # self rows at offset 7 (a gathered table's own slot)
        table[7:] = X[:, c0:c0 + w]
        gs = TypedGraph(g.rowptr, (g.colidx + 7).to(torch.int32), 6, num_cols=N + 7, edge_id_base=g.edge_id_base,
                        self_id_base=g.self_id_base, self_rows=N)
        gs.split_threshold, gs.split_chunk = 256, 128
        spmm_forward_slice(table, gs.with_dropedge(de), Zs, c0, self_col0=7)
        c0 += w
    assert c0 == F
    assert torch.equal(Zs, Zw)


@pytest.mark.parametrize("kind,F,slices", [("er", 256, (128, 128)), ("er", 256, (64, 64, 128)),
                                           ("rmat", 512, (128, 256, 128)), ("er", 100, (52, 48))])
def test_column_slices_backward_equal_whole(kind, F, slices):
    """grl_typed_spmm_bwd_slice: each column slice of dX (into its own table,
    and into a strided, unaligned view) bitwise equal to the whole-width
    backward -- DropEdge on, R-MAT hub columns split."""
    from grl.ops import spmm_backward, spmm_backward_slice

    N = 1 << 13
    g = TypedGraph.synthetic(N, 48.0, 6, kind=kind, seed=8, device=DEV)
    g.split_threshold, g.split_chunk = 256, 128  # force the hub-chunk path at this size
    gd = g.with_dropedge(DropEdge(0.3, 4, 2))
    dZ = torch.randn(N, 7 * F, device=DEV)
    dXw = spmm_backward(dZ, gd, F)
    c0 = 0
    for w in slices:
        table = torch.full((N, w), float("nan"), device=DEV)
        spmm_backward_slice(dZ, gd, c0, table)
        assert torch.equal(table, dXw[:, c0:c0 + w]), (c0, w)
        buf = torch.full((N, w + 5), float("nan"), device=DEV)
        spmm_backward_slice(dZ, gd, c0, buf[:, 3:3 + w])  # row stride w + 5, 12-B offset: scalar path
        assert torch.equal(buf[:, 3:3 + w], dXw[:, c0:c0 + w]), (c0, w)
        c0 += w
    assert c0 == F


def _free_port():
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _shard_worker(rank, world, port, mode, kind):
    """One rank of a 2-rank gloo world on the box's single GPU: the sharded
    HIP path (halo plan, exchange, typed SpMM fwd+bwd) against the plain
    one-GPU graph, which each rank also builds."""
    import os

    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        N, deg, L, F = 1 << 14, 24.0, 6, 64
        sg = ShardedGraph.synthetic(N, deg, L, kind=kind, seed=4, device=DEV, halo=mode)
        assert sg.plan.mode == mode
        g = TypedGraph.synthetic(N, deg, L, kind=kind, seed=4, device=DEV)
        rb, re = sg.plan.row_begin, sg.plan.row_end
        X = torch.randn(N, F, generator=torch.Generator().manual_seed(11)).to(DEV)
        dZ = torch.randn(N, (L + 1) * F, generator=torch.Generator().manual_seed(12)).to(DEV)
        de = DropEdge(0.25, 5, 3)
        Xg = X.clone().requires_grad_(True)
        Zg = typed_aggregate(Xg, g.with_dropedge(de))
        Zg.backward(dZ)
        X_loc = X[rb:re].clone().requires_grad_(True)
        Z = sg.aggregate(X_loc, de)
        assert torch.equal(Z, Zg[rb:re])  # bitwise: same values, same edge order
        Z.backward(dZ[rb:re])
        # dX: partials from the two ranks add in peer order rather than CSC order; R-MAT hub
        # columns sum thousands of terms, so use the north-star fp32 tolerance (1e-4)
        torch.testing.assert_close(X_loc.grad, Xg.grad[rb:re], rtol=1e-5, atol=1e-4)
        # the no-allocation bench form gives the same Z
        p = sg.plan
        X_ext = torch.zeros(p.n_loc + p.n_halo, F, device=DEV)
        X_ext[: p.n_loc] = X[rb:re]
        send = torch.empty(p.send_index.numel(), F, device=DEV)
        halo_exchange_into(X_ext[: p.n_loc], X_ext, send, p)
        out = torch.empty_like(Z)
        spmm_forward(X_ext, sg.graph.with_dropedge(de), out=out)
        assert torch.equal(out, Zg[rb:re].detach())
        # the pipelined exchange (column slices in flight while the previous slice aggregates)
        from grl.dist import HaloPipeline

        for K in (1, 2, 4):
            pipe = HaloPipeline(sg, F, chunks=K, device=DEV)
            outp = torch.full_like(out, float("nan"))
            pipe.run(X[rb:re].contiguous(), outp, de)
            torch.cuda.synchronize()
            assert torch.equal(outp, Zg[rb:re].detach()), K
        # both exchanges pipelined with the gathers (autograd): same Z, and dX bitwise equal to the
        # unsliced sharded backward (the same partials, added in the same peer order)
        for K in (1, 2, 4):
            X_p = X[rb:re].clone().requires_grad_(True)
            Zp = sg.aggregate(X_p, de, chunks=K)
            assert torch.equal(Zp, Zg[rb:re].detach()), K
            Zp.backward(dZ[rb:re])
            assert torch.equal(X_p.grad, X_loc.grad), K
        # a whole sharded GraphConv layer: weight grads summed over ranks equal one GPU's
        from gnn.models import GraphConv
        from grl.dist import allreduce_gradients

        torch.manual_seed(21)
        layer = GraphConv(F, 48, L).to(DEV)
        torch.manual_seed(21)
        layer1 = GraphConv(F, 48, L).to(DEV)
        R = torch.randn(N, 48, generator=torch.Generator().manual_seed(13)).to(DEV)
        (layer1.propagate(X[None], g.with_dropedge(de), relu=True)[0] * R).sum().backward()
        out_loc = sg.graphconv(X[rb:re], layer, de, relu=True)
        (out_loc * R[rb:re]).sum().backward()
        allreduce_gradients(layer.parameters())
        torch.testing.assert_close(layer.h_weights.grad, layer1.h_weights.grad, rtol=1e-4, atol=1e-4)
        torch.testing.assert_close(layer.bias.grad, layer1.bias.grad, rtol=1e-4, atol=1e-4)
        # the same layer with the pipelined exchanges: bitwise the unpipelined layer's grads
        grads = [t.grad.clone() for t in (layer.h_weights, layer.bias)]
        layer.zero_grad()
        X_a, X_b = X[rb:re].clone().requires_grad_(True), X[rb:re].clone().requires_grad_(True)
        out_c = sg.graphconv(X_a, layer, de, relu=True, chunks=2)
        # the chunked layer's linear takes the whole graph's GEMM path (path_rows): the same rows' bits
        assert torch.equal(out_c, out_loc)
        (out_c * R[rb:re]).sum().backward()
        allreduce_gradients(layer.parameters())
        assert all(torch.equal(t.grad, g0) for t, g0 in zip((layer.h_weights, layer.bias), grads))
        (sg.graphconv(X_b, layer, de, relu=True) * R[rb:re]).sum().backward()
        assert torch.equal(X_a.grad, X_b.grad)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("mode,kind", [("sparse", "er"), ("dense", "er"), ("sparse", "rmat"), ("dense", "rmat")])
def test_two_ranks_on_one_gpu_match_single_gpu(mode, kind):
    """The N>1 path on real kernels (gloo moves the halo through host memory
    here; the bench and product use RCCL)."""
    import torch.multiprocessing as mp

    mp.spawn(_shard_worker, args=(2, _free_port(), mode, kind), nprocs=2, join=True)


def _bench_two_ranks(extra, nproc=2):
    import json
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(nproc),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", str(nproc),
           "--dist-backend", "gloo", "--steps", "2", "--warmup", "1", "--cpu-seconds", "0"] + extra
    r = subprocess.run(cmd, cwd=root, capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    out = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "halo"):
        assert k in out, k
    assert out["n_gpus"] == nproc and out["value"] > 0
    return out


def test_bench_spawns_its_ranks_without_a_launcher():
    """`python bench.py --gpus 2` with no torchrun: bench.py starts the two
    rank processes itself (the parent never touches the GPU) and prints
    rank 0's one line with n_gpus 2."""
    import json
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    cmd = [sys.executable, "bench.py", "--gpus", "2", "--dist-backend", "gloo", "--workload", "weak",
           "--nodes-per-gpu", "20000", "--steps", "2", "--warmup", "1", "--cpu-seconds", "0"]
    r = subprocess.run(cmd, cwd=root, env=env, capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["config"]["nodes_total"] == 40000 and out["value"] > 0


def test_bench_two_ranks_contract():
    """The driver's N>1 launch (torch.distributed.run, one rank per GPU) of
    bench.py, rehearsed with two gloo ranks sharing the box's GPU: exactly
    one JSON line from rank 0 with the contract's fields; with no workload
    flag N>1 is BASELINE's C4 (a fixed 4M-node graph, strong scaling)."""
    out = _bench_two_ranks([])
    assert out["config"]["workload"] == "C4" and out["config"]["nodes_total"] == 4_000_000
    assert out["scaling"] == "strong" and out["config"]["d"] == 256
    assert out["halo"]["mode"] == "dense" and out["halo"]["chunks"] == 2
    bwd = out["halo"]["backward"]
    assert "error" not in bwd, bwd
    assert bwd["pipelined_ms"] > 0 and bwd["gather_only_ms"] > 0 and bwd["exchange_only_ms"] > 0


def test_bench_two_ranks_weak_and_c5_shape():
    """The weak-scaling extra and a small R-MAT d=512 DropEdge shard pair."""
    out = _bench_two_ranks(["--workload", "weak", "--nodes-per-gpu", "20000"])
    assert out["scaling"] == "weak" and out["config"]["nodes_total"] == 40000
    out = _bench_two_ranks(["--workload", "C5", "--nodes-per-gpu", "65536", "--chunks", "4"])
    assert out["config"]["graph"] == "rmat" and out["config"]["d"] == 512 and out["config"]["dropedge_p"] == 0.2
    assert out["config"]["nodes_total"] == 131072 and out["halo"]["chunks"] == 4


def test_bench_four_ranks_c4_shape():
    """World 4 (the driver's N=4 launch shape): a C4-style ER graph at 20k
    nodes cut into 4 node-range shards, dense halo pipelined over 2 slices;
    one JSON line, the halo breakdown in both directions.  (The full 4M-node
    C4 at P=4 ran the same way: tools/rehearse_p4.sh,
    profiles/r02_rehearse_p4_c4_line.json.)"""
    out = _bench_two_ranks(["--workload", "weak", "--nodes-per-gpu", "20000"], nproc=4)
    assert out["config"]["nodes_total"] == 80000 and out["halo"]["chunks"] == 2
    assert "error" not in out["halo"]["backward"]


def _fused_shard_worker(rank, world, port, mode):
    """One rank of a 2-rank gloo world: the one-kernel GraphConv on this
    rank's shard (local rows + halo slots, shard-offset DropEdge ids) equals
    the one-GPU graph's rows, bitwise, and the two-kernel path on the shard."""
    import os

    import torch.distributed as dist

    from grl.ops import graph_conv_infer

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        N, deg, L, F, C = 40_000, 16.0, 6, 256, 256  # shards of 20k rows: the x6 (hence fused) shape
        sg = ShardedGraph.synthetic(N, deg, L, kind="er", seed=6, device=DEV, halo=mode)
        g = TypedGraph.synthetic(N, deg, L, kind="er", seed=6, device=DEV)
        rb, re = sg.plan.row_begin, sg.plan.row_end
        gen = torch.Generator().manual_seed(31)
        X = torch.randn(N, F, generator=gen).to(DEV)
        W = (torch.randn(7 * F, C, generator=gen) / 40).to(DEV)
        b = torch.randn(C, generator=gen).to(DEV)
        de = DropEdge(0.3, 8, 1, True)
        p = sg.plan
        X_ext = torch.zeros(p.n_loc + p.n_halo, F, device=DEV)
        X_ext[: p.n_loc] = X[rb:re]
        send = torch.empty(p.send_index.numel(), F, device=DEV)
        halo_exchange_into(X_ext[: p.n_loc], X_ext, send, p)
        local = sg.graph.with_dropedge(de)
        full = graph_conv_infer(X, g.with_dropedge(de), W, b, True)
        out = graph_conv_infer(X_ext, local, W, b, True)
        assert torch.equal(out, full[rb:re])
        import grl

        with grl.options(graphconv_fused=0):
            assert torch.equal(graph_conv_infer(X_ext, local, W, b, True), out)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["sparse", "dense"])
def test_two_ranks_fused_graphconv_on_shards(mode):
    import torch.multiprocessing as mp

    mp.spawn(_fused_shard_worker, args=(2, _free_port(), mode), nprocs=2, join=True)


def _fused_train_shard_worker(rank, world, port, mode):
    """One rank of a 2-rank gloo world, a training GraphConv on shards big
    enough for the one-kernel paths: forward one kernel on [own | halo] rows
    (out bitwise the one-GPU rows), data gradient one kernel over the shard's
    typed transpose whose halo rows go home in the exchange's backward (dX
    and the all-reduced dW / db within fp32 tolerance of one GPU)."""
    import os

    import torch.distributed as dist

    from gnn.models import GraphConv
    from grl.dist import allreduce_gradients

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        N, deg, L, F, C = 40_000, 16.0, 6, 256, 256
        sg = ShardedGraph.synthetic(N, deg, L, kind="er", seed=6, device=DEV, halo=mode)
        g = TypedGraph.synthetic(N, deg, L, kind="er", seed=6, device=DEV)
        rb, re = sg.plan.row_begin, sg.plan.row_end
        gen = torch.Generator().manual_seed(41)
        X = torch.randn(N, F, generator=gen).to(DEV)
        R = torch.randn(N, C, generator=gen).to(DEV)
        de = DropEdge(0.3, 8, 1, True)
        torch.manual_seed(21)
        layer = GraphConv(F, C, L).to(DEV)
        torch.manual_seed(21)
        layer1 = GraphConv(F, C, L).to(DEV)
        Xg = X.clone().requires_grad_(True)
        out1 = layer1.propagate(Xg[None], g.with_dropedge(de), relu=True)[0]
        (out1 * R).sum().backward()
        X_loc = X[rb:re].clone().requires_grad_(True)
        out = sg.graphconv(X_loc, layer, de, relu=True)
        assert torch.equal(out, out1[rb:re].detach())
        (out * R[rb:re]).sum().backward()
        assert "typed_transpose" in sg.graph._shared  # the shard's dX took the one-kernel path
        allreduce_gradients(layer.parameters())
        torch.testing.assert_close(X_loc.grad, Xg.grad[rb:re], rtol=1e-4, atol=1e-4)
        torch.testing.assert_close(layer.h_weights.grad, layer1.h_weights.grad, rtol=1e-4, atol=1e-3)
        torch.testing.assert_close(layer.bias.grad, layer1.bias.grad, rtol=1e-4, atol=1e-3)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["sparse", "dense"])
def test_two_ranks_one_kernel_training_layer_on_shards(mode):
    import torch.multiprocessing as mp

    mp.spawn(_fused_train_shard_worker, args=(2, _free_port(), mode), nprocs=2, join=True)


def _rows_pipeline_worker(rank, world, port, mode):
    """One rank of a gloo world on the GPU: ShardedGraph.graphconv(pipeline=
    "rows") -- one-kernel forward on [own | halo] rows, one-kernel data
    gradient in row blocks with each peer's halo block sent as soon as it is
    computed -- against the unpipelined one-kernel sharded layer: out, dX,
    dW and db bitwise; out bitwise the one-GPU rows."""
    import os

    import torch.distributed as dist

    from gnn.models import GraphConv

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        N, deg, L, F, C = 30_000 * world, 16.0, 6, 256, 256  # shards large enough for the one-kernel paths
        sg = ShardedGraph.synthetic(N, deg, L, kind="er", seed=6, device=DEV, halo=mode)
        assert sg.plan.mode == mode
        g = TypedGraph.synthetic(N, deg, L, kind="er", seed=6, device=DEV)
        rb, re = sg.plan.row_begin, sg.plan.row_end
        gen = torch.Generator().manual_seed(43)
        X = torch.randn(N, F, generator=gen).to(DEV)
        R = torch.randn(N, C, generator=gen).to(DEV)
        de = DropEdge(0.3, 8, 1, True)
        torch.manual_seed(21)
        layer = GraphConv(F, C, L).to(DEV)
        res = {}
        for pipe in ("rows", None):
            layer.zero_grad()
            X_loc = X[rb:re].clone().requires_grad_(True)
            out = sg.graphconv(X_loc, layer, de, relu=True, pipeline=pipe)
            (out * R[rb:re]).sum().backward()
            res[pipe] = (out.detach(), X_loc.grad, layer.h_weights.grad.clone(), layer.bias.grad.clone())
        bad = [(name, float((a - b).abs().max()), float(b.abs().max()))
               for name, a, b in zip(("out", "dX", "dW", "db"), res["rows"], res[None]) if not torch.equal(a, b)]
        if bad:
            raise AssertionError(f"rank {rank}: not bitwise {bad}")
        # the forward is the one-GPU rows
        from grl.ops import graph_conv_infer

        full = graph_conv_infer(X, g.with_dropedge(de), layer.h_weights.detach(), layer.bias.detach(), True)
        assert torch.equal(res["rows"][0], full[rb:re])
        assert "typed_transpose" in sg.graph._shared
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,mode", [(2, "dense"), (2, "sparse"), (3, "dense"), (3, "sparse")])
def test_rows_pipelined_graphconv_on_shards(world, mode):
    import torch.multiprocessing as mp

    mp.spawn(_rows_pipeline_worker, args=(world, _free_port(), mode), nprocs=world, join=True)
