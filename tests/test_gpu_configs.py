"""GPU parity at BASELINE.json's full configuration sizes:
the HIP path on the device-built C2 / C3 / C4 / C5 graphs against the CPU
oracle (oracle/grl_oracle.c), bitwise.

  C2  ER N=100k, avg_deg 16, d=256                 whole Z vs oracle
  C3  ER N=1M, avg_deg 32, d=256, p=0 and p=0.3    100k sampled rows of Z;
                                                   backward dX (whole) vs oracle
  C4  ER N=4M, avg_deg 32, d=256, two node-range   each shard's Z through the
      shards (gloo ranks on the one GPU)           pipelined halo exchange vs the
                                                   one-GPU graph (whole shard) and
                                                   the oracle (sampled rows)
  C5  R-MAT scale 23, avg_deg 64, d=512, p=0.2     real hub rows (split into
                                                   chunks at the default
                                                   threshold) + random rows, the
                                                   whole-row wide path (X > 12 GB)

The device graphs are also checked against the oracle's generator on the
sampled row ranges.  Reference math: robust_gcn.py:45-47 (aggregation),
drop_robust_gcn.py:76-85 (DropEdge before each GraphConv).
"""
import os
import socket

import numpy as np
import pytest
import torch

from grl import DropEdge, TypedGraph
from grl.ops import spmm_backward, spmm_forward
from oracle import c_oracle

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
L = 6


def _say(msg):
    print(f"  [{msg}]", flush=True)


def _ranges(num_rows, count, width, seed, extra=()):
    """`count` row ranges of `width` rows spread over the graph (+ extra
    ranges), clipped and sorted."""
    rng = np.random.default_rng(seed)
    starts = np.sort(rng.choice(max(1, num_rows - width), size=count, replace=False))
    out = [(int(s), int(min(num_rows, s + width))) for s in starts] + list(extra)
    return sorted(set(out))


def _check_rows(g, X_host, Z, ranges, d, kind, N, avg_deg, seed=0, synth_ranges=None, verbose=False):
    """Z rows of each range bitwise vs the oracle restatement (same edge
    order, same DropEdge ids, the engine's chunked order on heavy rows); the
    device CSR rows of the first `synth_ranges` ranges (all by default) vs
    the oracle's generator (each such check scans every candidate edge)."""
    rowptr_d = g.rowptr
    split = (g.split_threshold, g.split_chunk)
    rows = 0
    for i, (r0, r1) in enumerate(ranges):
        rp = rowptr_d[r0 * L: r1 * L + 1].cpu().numpy()
        e0 = int(rp[0])
        rp = rp - e0
        ci = g.colidx[e0: e0 + int(rp[-1])].cpu().numpy()
        if synth_ranges is None or i < synth_ranges:
            orp, oci, _ = c_oracle.synth({"er": 0, "rmat": 1}[kind], L, N, int(round(avg_deg * N)), seed, r0, r1)
            np.testing.assert_array_equal(rp, orp)
            np.testing.assert_array_equal(ci, oci)
        Zc = c_oracle.spmm_fwd(rp, ci, X_host, L, True, d=d, split=split, edge_base=g.edge_id_base + e0,
                               self_base=g.self_id_base + r0, X_self=X_host[r0:])
        Zg = Z[r0:r1].cpu().numpy()
        if not np.array_equal(Zg, Zc):
            bad = np.argwhere(Zg != Zc)
            raise AssertionError(f"rows [{r0},{r1}): {len(bad)} elements differ, first {bad[:3].tolist()}, "
                                 f"max |d| {np.abs(Zg.astype(np.float64) - Zc).max():.3e}")
        rows += r1 - r0
        if verbose:
            _say(f"rows [{r0}, {r1}) bitwise ({int(rp[-1])} edges)")
    return rows


@pytest.fixture(scope="module")
def c3():
    N = 1_000_000
    g = TypedGraph.synthetic(N, 32.0, L, seed=0, device=DEV)
    assert g.nnz == 31_999_916  # C3 after dedupe (bench config.edges_total)
    X = torch.randn(N, 256, generator=torch.Generator(device=DEV).manual_seed(1), device=DEV)
    yield g, X, X.cpu().numpy()
    del g, X
    torch.cuda.empty_cache()


def test_c2_full_graph_forward_vs_oracle():
    N = 100_000
    g = TypedGraph.synthetic(N, 16.0, L, seed=0, device=DEV)
    X = torch.randn(N, 256, generator=torch.Generator(device=DEV).manual_seed(1), device=DEV)
    Z = spmm_forward(X, g)
    rows = _check_rows(g, X.cpu().numpy(), Z, [(0, N)], None, "er", N, 16.0)
    assert rows == N


@pytest.mark.parametrize("p", [0.0, 0.3])
def test_c3_full_graph_forward_vs_oracle(c3, p):
    g, X, Xh = c3
    N = g.num_rows
    de = DropEdge(p, 2, 0, True) if p else None
    Z = spmm_forward(X, g.with_dropedge(de))
    d = c_oracle.drop(p, 2, 0, True) if p else None
    rows = _check_rows(g, Xh, Z, _ranges(N, 10, 10_000, 3, extra=[(0, 64), (N - 64, N)]), d, "er", N, 32.0)
    assert rows >= 100_000
    _say(f"C3 p={p}: {rows} rows bitwise")
    del Z


def test_c3_full_graph_backward_vs_oracle(c3):
    """dX = A_drop^T dZ over the whole C3 graph (CSC gather, DropEdge p=0.3)
    against the oracle's CSC restatement, every element."""
    g, X, Xh = c3
    N, F = g.num_rows, 256
    gd = g.with_dropedge(DropEdge(0.3, 2, 5, True))
    dZ = torch.randn(N, 7 * F, generator=torch.Generator(device=DEV).manual_seed(9), device=DEV)
    dX = spmm_backward(dZ, gd, F).cpu().numpy()
    rp, ci = g.rowptr.cpu().numpy(), g.colidx.cpu().numpy()
    colptr, zrow, eid, _ = c_oracle.csr_to_csc(rp, ci, L, N, True)
    np.testing.assert_array_equal(colptr, g.csc()["colptr"].cpu().numpy())
    ref = c_oracle.spmm_bwd(colptr, zrow, eid, dZ.cpu().numpy(), L, F, N, True, d=c_oracle.drop(0.3, 2, 5, True),
                            self_base=g.self_id_base, split=(g.split_threshold, g.split_chunk))
    if not np.array_equal(dX, ref):
        raise AssertionError(f"dX differs in {(dX != ref).sum()} elements, max |d| "
                             f"{np.abs(dX.astype(np.float64) - ref).max():.3e}")
    _say("C3 backward: whole dX bitwise")


def test_c3_full_graph_layer_data_gradient_one_kernel(c3):
    """The layer's dX at C3 through the one-kernel reassociated backward
    (grl_graphconv_bwd_data over the typed transpose, DropEdge p=0.3) against
    the oracle in float64 on 2,048 sampled rows: dX[m] = w_self(m) G[m] W_0^T
    + sum over the oracle CSC's entries (n, t) -> m of w_e G[n] W_{1+t}^T,
    with the oracle's mask; within 1e-5 of the same sum over |terms|."""
    from grl.ops import graph_conv_bwd_data
    from oracle import hash as ohash

    g, X, Xh = c3
    N, F, C = g.num_rows, 256, 256
    p, seed, call = 0.3, 2, 6
    gd = g.with_dropedge(DropEdge(p, seed, call, True))
    gen = torch.Generator(device=DEV).manual_seed(13)
    G = torch.randn(N, C, generator=gen, device=DEV)
    W = torch.randn(7 * F, C, generator=gen, device=DEV) / (7 * F) ** 0.5
    dX = graph_conv_bwd_data(G, gd, W, F)
    assert dX is not None
    rows = np.unique(np.r_[0:64, N - 64:N, np.random.default_rng(4).integers(0, N, 1920)])
    c = g.csc()
    colptr, zrow, eid = (c[k].cpu().numpy() for k in ("colptr", "zrow", "eid"))
    Gh, Wh = G.cpu().numpy().astype(np.float64), W.cpu().numpy().astype(np.float64)
    Wt = Wh.reshape(7, F, C)  # W_s = rows [s F, (s+1) F)
    _, _, scale = ohash.dropedge_params(p)
    got = dX.cpu().numpy()[rows]
    ref = np.zeros((len(rows), F))
    mag = np.zeros((len(rows), F))
    for i, m in enumerate(rows):
        ids = [g.self_id_base + int(m)]
        ns, ss = [int(m)], [0]
        for e in range(colptr[m], colptr[m + 1]):
            ns.append(int(zrow[e]) // 7)
            ss.append(int(zrow[e]) % 7)
            ids.append(int(eid[e]))
        keep = ohash.dropedge_keep(p, seed, call, np.array(ids, dtype=np.uint64)).astype(np.float64) * float(scale)
        for w, n, s_ in zip(keep, ns, ss):
            if w:
                ref[i] += w * (Wt[s_] @ Gh[n])
                mag[i] += w * (np.abs(Wt[s_]) @ np.abs(Gh[n]))
    err = np.abs(got - ref)
    assert np.all(err <= 1e-5 * mag + 1e-6), float((err / (mag + 1e-30)).max())
    _say(f"C3 one-kernel dX: {len(rows)} rows within {float((err / (mag + 1e-30)).max()):.2e} of sum|terms|")


def test_c5_rmat_scale23_forward_vs_oracle():
    """C5 on one GPU: 2^23 nodes, ~528M typed edges, d=512, DropEdge p=0.2.
    Hub rows run as chunk items (default split threshold) and the table
    (17 GB) takes the whole-row wide path; hub ranges + random ranges are
    compared bitwise with the oracle's chunked order."""
    N, deg, F = 1 << 23, 64.0, 512
    g = TypedGraph.synthetic(N, deg, L, kind="rmat", seed=0, device=DEV)
    _say(f"C5 graph: {g.nnz} edges")
    assert g.nnz > 500_000_000
    X = torch.randn(N, F, generator=torch.Generator(device=DEV).manual_seed(1), device=DEV)
    de = DropEdge(0.2, 2, 0, True)
    Z = spmm_forward(X, g.with_dropedge(de))
    torch.cuda.synchronize()
    stats = g.split_stats()["csr"]
    assert stats["chunks"] > 100_000 and stats["heavy_segments"] > 0, stats  # real hubs, split at default
    deg_rows = (g.rowptr[L::L] - g.rowptr[:-1:L])
    hubs = torch.topk(deg_rows.float(), 4).indices.cpu().tolist()
    assert int(deg_rows.max()) > 100 * g.split_threshold
    _say(f"C5 split: {stats}; max row {int(deg_rows.max())} edges; hubs {hubs}")
    Xh = X.cpu().numpy()
    _say("C5: X on host")
    extra = [(h, h + 1) for h in hubs] + [(0, 2048)]  # low ids: R-MAT's densest rows
    rows = _check_rows(g, Xh, Z, _ranges(N, 8, 2048, 5, extra=extra), c_oracle.drop(0.2, 2, 0, True), "rmat", N, deg,
                       synth_ranges=2, verbose=True)
    _say(f"C5: {rows} rows bitwise (incl. {len(hubs)} hub rows)")
    del Z, X, g
    torch.cuda.empty_cache()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _c4_worker(rank, world, port):
    import torch.distributed as dist

    from grl.dist import HaloPipeline, ShardedGraph

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        N, F = 4_000_000, 256
        sg = ShardedGraph.synthetic(N, 32.0, L, seed=0, device=DEV)
        rb, re = sg.plan.row_begin, sg.plan.row_end
        X = torch.randn(N, F, generator=torch.Generator(device=DEV).manual_seed(1), device=DEV)
        de = DropEdge(0.3, 2, 0, True)
        Zs = torch.empty(re - rb, 7 * F, device=DEV)
        HaloPipeline(sg, F, chunks=2, device=DEV).run(X[rb:re].contiguous(), Zs, de)
        g = TypedGraph.synthetic(N, 32.0, L, seed=0, device=DEV)
        Zf = torch.empty(N, 7 * F, device=DEV)
        spmm_forward(X, g.with_dropedge(de), out=Zf)
        assert torch.equal(Zs, Zf[rb:re]), f"rank {rank}: shard Z differs from the one-GPU graph"
        del Zf
        torch.cuda.empty_cache()
        # and the one-GPU rows against the oracle on sampled ranges of this shard
        n = re - rb
        rel = _ranges(n, 4, 4096, 11 + rank)
        Xh = X.cpu().numpy()
        for a, b in rel:
            r0, r1 = rb + a, rb + b
            rp = g.rowptr[r0 * L: r1 * L + 1].cpu().numpy()
            e0 = int(rp[0])
            ci = g.colidx[e0: int(rp[-1])].cpu().numpy()
            Zc = c_oracle.spmm_fwd(rp - e0, ci, Xh, L, True, d=c_oracle.drop(0.3, 2, 0, True), edge_base=e0,
                                   self_base=g.self_id_base + r0, X_self=Xh[r0:])
            assert np.array_equal(Zs[a:b].cpu().numpy(), Zc), (rank, a, b)
        print(f"  [C4 rank {rank}: shard rows [{rb},{re}) bitwise vs one GPU and oracle]", flush=True)
    finally:
        dist.destroy_process_group()


def test_c4_two_shards_pipelined_halo_vs_one_gpu_and_oracle():
    """C4 (N=4M) as two node-range shards on the box's GPU (gloo moves the
    halo through host memory; the bench uses RCCL): the pipelined exchange +
    column-slice aggregation equals the one-GPU aggregation bitwise."""
    import torch.multiprocessing as mp

    mp.spawn(_c4_worker, args=(2, _free_port()), nprocs=2, join=True)
