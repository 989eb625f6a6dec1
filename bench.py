#!/usr/bin/env python
"""Benchmark: typed-CSR SpMM (GraphConv aggregation, robust_gcn.py:45-47) on
MI355X -- BASELINE.json metric "aggregated edges/sec + SpMM HBM GB/s vs
roofline, d=256, 1/2/4/8 GPU".

    python bench.py [--gpus N --steps K --warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU)

Workload: per GPU a node-range shard of 1M nodes of a
seeded Erdos-Renyi typed graph (avg total out-degree 32 over L=6 edge
types, dedupe), d=256 fp32 features -- config C3 at N=1, the C4 shape
(4M nodes) at N=4.  A step = one GraphConv aggregation forward over the
rank's rows (N>1: preceded by the halo exchange -- RCCL all-to-all-v of the
remote feature rows the shard's edges reference, grl/dist.py).  Inputs are resident in HBM before timing.
Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "graph-representation-learning_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "aggregated edges/sec + SpMM HBM GB/s vs roofline, d=256, 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0     # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
F32_MFMA_PEAK_TFS = 157.3  # dense fp32 MFMA (v_mfma_f32_32x32x2_f32)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--nodes-per-gpu", type=int, default=1_000_000)
    ap.add_argument("--avg-deg", type=float, default=32.0)
    ap.add_argument("--types", type=int, default=6)
    ap.add_argument("--dim", type=int, default=256)
    ap.add_argument("--p", type=float, default=0.0, help="DropEdge rate inside the timed step (0 = eval)")
    ap.add_argument("--graph", choices=["er", "rmat"], default="er")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline budget (0 disables)")
    ap.add_argument("--extras", action="store_true",
                    help="also time fused-DropEdge fwd, backward, MFMA linear and a full layer (not the headline)")
    ap.add_argument("--dist-backend", default="nccl",
                    help="process-group backend for N>1 (nccl = RCCL; gloo only to smoke-test the N>1 path "
                         "with several ranks on one GPU)")
    ap.add_argument("--halo", choices=["auto", "sparse", "dense"], default="auto",
                    help="halo exchange layout for N>1 (grl/dist.py): sparse all-to-all-v of the referenced rows, "
                         "dense all-gather of every shard; auto picks dense when >=75%% of remote rows are referenced")
    ap.add_argument("--only", choices=["fwd", "bwd", "linear", "layer", "c1", "model"], default=None,
                    help="profiling aid: run just that kernel K times (no JSON line); c1: print the C1 "
                         "(debug.json model) timings alone")
    return ap.parse_args()


def spmm_bytes(E, N, L, F, p, idx_bytes=4, ptr_bytes=4):
    """Algorithmic HBM bytes of one unfused typed-SpMM forward."""
    keep = 1.0 - p
    return keep * E * F * 4 + idx_bytes * E + ptr_bytes * (N * L + 1) + keep * N * F * 4 + N * (L + 1) * F * 4


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    ndev = torch.cuda.device_count()
    if args.dist_backend == "nccl" and world > 1 and local_rank >= ndev:
        raise SystemExit(f"rank {rank}: LOCAL_RANK {local_rank} but only {ndev} GPU(s) visible")
    dev = torch.device("cuda", local_rank % ndev)
    torch.cuda.set_device(dev)
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(args.dist_backend)

    if args.only == "c1":
        print(json.dumps({"c1_debug_json": c1_extras(dev, max(3, args.steps))}), flush=True)
        return
    if args.only == "model":
        print(json.dumps({"model_one_graph_100k": model_extras(dev),
                          "model_dense_A_mid_n": model_mid_extras(dev)}), flush=True)
        return

    from grl import DropEdge
    from grl.dist import ShardedGraph, halo_exchange_into
    from grl.ops import spmm_forward

    L, F = args.types, args.dim
    n_loc = args.nodes_per_gpu
    N = n_loc * world
    if args.graph == "rmat":
        N = 1 << (N - 1).bit_length()
        n_loc = N // world
    t0 = time.time()
    sg = ShardedGraph.synthetic(N, args.avg_deg, L, kind=args.graph, seed=0, device=dev, halo=args.halo)
    graph, plan = sg.graph, sg.plan
    n_loc = plan.n_loc
    E_loc, E_tot = graph.nnz, plan.num_edges_total
    gen = torch.Generator(device=dev)
    gen.manual_seed(1 + rank)
    # [own rows | halo rows]: own rows are written once, halo rows by the exchange
    X_full = torch.empty(plan.n_loc + plan.n_halo, F, device=dev)
    X_full[n_loc:plan.stride].zero_()  # dense plans: shard padding rows (never read by the kernel)
    X_loc = X_full[:n_loc]
    X_loc.copy_(torch.randn(n_loc, F, generator=gen, device=dev, dtype=torch.float32))
    send_buf = torch.empty(plan.send_index.numel(), F, device=dev)
    build_s = time.time() - t0

    de = DropEdge(args.p, 2, 0, True) if args.p > 0 else None
    g_step = graph.with_dropedge(de)
    stream = torch.cuda.current_stream(dev)
    Z = torch.empty(graph.num_rows, graph.segments * F, device=dev)  # preallocated: no allocation in the step

    def gather():
        halo_exchange_into(X_loc, X_full, send_buf, plan)

    def spmm():
        return spmm_forward(X_full, g_step, out=Z)

    if args.only is not None:
        run_only(args, graph, X_full, gather, spmm, L, F)
        return

    for _ in range(args.warmup):
        gather()
        spmm()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    ev_h = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    for i in range(args.steps):
        ev_h[i].record(stream)
        gather()
        ev[i][0].record(stream)
        spmm()
        ev[i][1].record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    wall = time.perf_counter() - t_start
    per_step = [a.elapsed_time(b) for a, b in ev]
    kern_ms = float(np.mean(per_step))
    halo_ms = float(np.mean([h.elapsed_time(a) for h, (a, _) in zip(ev_h, ev)]))
    if world > 1:
        tt = torch.tensor([wall, kern_ms, halo_ms], dtype=torch.float64,
                          device=dev if args.dist_backend == "nccl" else "cpu")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        wall, kern_ms, halo_ms = float(tt[0]), float(tt[1]), float(tt[2])
    ms_step = wall / args.steps * 1e3
    value = E_tot / (wall / args.steps)

    bytes_launch = spmm_bytes(E_loc, n_loc, L, F, args.p)
    achieved = bytes_launch / (kern_ms * 1e-3) / 1e9
    traffic = load_traffic(args, n_loc, world)
    out = {
        "metric": METRIC, "value": value, "unit": "edges/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": ms_step, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f32",
        "data": f"synthetic: seeded {'Erdos-Renyi' if args.graph == 'er' else 'R-MAT'} typed graph (graph seed 0), "
                "X ~ N(0,1) fp32 (seed 1+rank)",
        "config": {"workload": workload_name(args, world, n_loc) + f": {args.graph.upper()} typed graph, "
                   f"{n_loc} nodes/GPU, avg_deg {args.avg_deg:g} over L={L} edge types, d={F}, typed-SpMM "
                   f"forward (GraphConv aggregation){' + DropEdge p=%g' % args.p if args.p else ''}",
                   "nodes_total": N, "edges_total": E_tot, "nodes_per_gpu": n_loc, "avg_deg": args.avg_deg,
                   "num_types": L, "d": F, "dropedge_p": args.p, "graph": args.graph,
                   "parallelism": "single GPU" if world == 1 else
                   f"node-range shards x{world}, "
                   + ("RCCL" if args.dist_backend == "nccl" else f"{args.dist_backend} (host-staged)") + " "
                   + ("all-gather (dense halo)" if plan.mode == "dense" else "all-to-all-v (sparse halo)")
                   + f", rank {rank} references {plan.referenced_halo_rows} of {N - n_loc} remote rows"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "kernel": "spmm_kernel<4,1,8,false,false> (grl_typed_spmm_fwd)",
                     "kernel_ms": kern_ms, "kernel_ms_min_max": [min(per_step), max(per_step)],
                     "algorithmic_bytes_per_launch": bytes_launch},
        "build_s": build_s,
    }
    if world > 1:
        rows_in = (world - 1) * plan.stride if plan.mode == "dense" else sum(plan.recv_counts)
        out["halo"] = {"mode": plan.mode, "ms_max_over_ranks": halo_ms, "rows_received_rank0": rows_in,
                       "GB_received_rank0": rows_in * F * 4 / 1e9,
                       "GBps_rank0": rows_in * F * 4 / 1e9 / (halo_ms * 1e-3) if halo_ms > 0 else None}
    if args.graph == "rmat":
        out["config"]["split"] = graph.split_stats()
        out["config"]["max_row_edges"] = int((graph.rowptr[L::L] - graph.rowptr[:-1:L]).max())
    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        out["cpu_baseline"], out["parity"] = cpu_baseline(args, g_step, X_loc, Z, L, F)
    if args.extras:
        out["extras"] = extras(args, graph, X_full, gather, L, F, dev, E_loc, n_loc)
        if rank == 0:
            del X_full, Z
            torch.cuda.empty_cache()  # C1 is a small-graph workload: time it without C3's 8 GB resident
            out["extras"]["c1_debug_json"] = c1_extras(dev)
            out["extras"]["model_one_graph_100k"] = model_extras(dev)
            out["extras"]["model_dense_A_mid_n"] = model_mid_extras(dev)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def workload_name(args, world, n_loc):
    """Which SURVEY.md §8(d) config this run is (or is shaped like)."""
    if args.graph == "rmat":
        return "C5" if (n_loc * world == 1 << 23 and args.dim == 512) else "C5-shape"
    if args.dim == 256 and args.avg_deg == 32 and n_loc == 1_000_000:
        return {1: "C3", 4: "C4"}.get(world, "C4-shape (1M nodes/GPU)")
    if args.dim == 256 and args.avg_deg == 32 and n_loc * world == 4_000_000:
        return "C4"
    if args.dim == 256 and args.avg_deg == 16 and n_loc * world == 100_000:
        return "C2"
    return "custom"


def load_traffic(args, n_loc, world):
    """HBM bytes per launch from a committed rocprofv3 PMC summary of the same
    workload (profiles/pmc_traffic.json, written by tools/pmc_traffic.py),
    or None."""
    path = os.path.join(HERE, "profiles", "pmc_traffic.json")
    if not os.path.exists(path):
        return None
    try:
        d = json.load(open(path))
        key = f"{args.graph}_n{n_loc}_deg{args.avg_deg:g}_L{args.types}_d{args.dim}_p{args.p:g}"
        return d.get(key, {}).get("hbm_bytes_per_launch")
    except (OSError, ValueError):  # unreadable summary: report traffic as unmeasured
        return None


def cpu_baseline(args, graph, X, Z, L, F):
    """Oracle (grl_oracle.c, OpenMP) on a bounded row sample of the SAME
    graph and features; also checks the GPU rows of that sample bitwise."""
    from oracle import c_oracle

    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
    # a contiguous row range from the middle of the graph holding ~3.2M edges
    # (= 100k rows of C3; on R-MAT the bulk of rows, not the hub head)
    node_ptr = graph.rowptr[::L].contiguous()
    r0 = graph.num_rows // 2
    target = torch.tensor([int(node_ptr[r0]) + 3_200_000], dtype=torch.int32, device=node_ptr.device)
    r1 = max(r0 + 1, min(graph.num_rows, int(torch.searchsorted(node_ptr, target))))
    rows = r1 - r0
    e0 = int(node_ptr[r0])
    rowptr = (graph.rowptr[r0 * L: r1 * L + 1] - e0).cpu().numpy()
    colidx = graph.colidx[e0: e0 + int(rowptr[-1])].cpu().numpy()
    Xh = X.cpu().numpy()
    E = int(rowptr[-1])
    d = None if args.p <= 0 else c_oracle.drop(args.p, 2, 0, True)  # the timed step's DropEdge stream
    split = (graph.split_threshold, graph.split_chunk)  # the engine's chunked order on heavy rows
    t0 = time.perf_counter()
    passes = 0
    while True:
        Zc = c_oracle.spmm_fwd(rowptr, colidx, Xh, L, True, d=d, nthreads=threads, split=split,
                               edge_base=graph.edge_id_base + e0, self_base=graph.self_id_base + r0,
                               X_self=Xh[r0:])
        passes += 1
        if time.perf_counter() - t0 >= args.cpu_seconds:
            break
    dt = time.perf_counter() - t0
    Zg = Z[r0:r1].cpu().numpy()
    diff = float(np.abs(Zg.astype(np.float64) - Zc).max())
    cpu = {"value": E * passes / dt, "unit": "edges/s", "cores": threads, "kind": "port",
           "sample": f"nodes [{r0}, {r1}) ({E} typed edges) of the same graph and X, {passes} passes in {dt:.1f}s; "
                     f"oracle/grl_oracle.c OpenMP typed-CSR SpMM"}
    parity = {"rows_checked": rows, "max_abs_diff": diff, "bitwise_equal": bool(np.array_equal(Zg, Zc)),
              "tolerance": 1e-4}
    return cpu, parity


def _time(fn, iters, warm=1):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def extras(args, graph, X_full, gather, L, F, dev, E_loc, n_loc):
    """Secondary numbers (not the headline): fused DropEdge forward, backward
    (transposed gather), MFMA linear, full GraphConv layer fwd+bwd."""
    from grl import DropEdge
    from grl.ops import graph_conv, graph_linear, linear_fwd, typed_aggregate

    res = {}
    iters = max(3, min(10, args.steps))
    gd = graph.with_dropedge(DropEdge(0.3, 2, 0, True))
    ms = _time(lambda: typed_aggregate(X_full, gd), iters)
    res["spmm_fwd_dropedge_p0.3"] = {"ms": ms, "edges_per_s": E_loc / (ms * 1e-3),
                                     "alg_GBps": spmm_bytes(E_loc, n_loc, L, F, 0.3) / (ms * 1e-3) / 1e9}
    Xg = X_full.detach().clone().requires_grad_(True)
    Z = typed_aggregate(Xg, graph)
    dZ = torch.randn_like(Z)
    graph.csc()  # one-time CSC build (cached per graph), not part of the step
    ms = _time(lambda: torch.autograd.grad(Z, Xg, dZ, retain_graph=True), iters)
    # no DropEdge on this graph: the CSC edge ids are not read, only the row indices (4 B/edge)
    bwd_bytes = E_loc * F * 4 + 4 * E_loc + 4 * (graph.num_cols + 1) + graph.num_cols * F * 4 * 2
    res["spmm_bwd"] = {"ms": ms, "edges_per_s": E_loc / (ms * 1e-3), "alg_GBps": bwd_bytes / (ms * 1e-3) / 1e9}
    torch.manual_seed(3)
    W = torch.randn((L + 1) * F, F, device=dev) / np.sqrt((L + 1) * F)
    b = torch.randn(F, device=dev)
    Zd = Z.detach()
    ms = _time(lambda: linear_fwd(Zd, W, b, True), iters)
    flops = 2.0 * Zd.shape[0] * Zd.shape[1] * F
    path = ("x6: fp32 split into 3 bf16 parts, 6 products on v_mfma_f32_32x32x16_bf16 (DESIGN 4.2)"
            if os.environ.get("GRL_GEMM_X6", "1") != "0" else "fp32 MFMA v_mfma_f32_32x32x2_f32")
    res["linear_mfma_fwd"] = {"ms": ms, "TFLOPs_fp32_equivalent": flops / (ms * 1e-3) / 1e12,
                              "vs_f32_mfma_peak": flops / (ms * 1e-3) / 1e12 / F32_MFMA_PEAK_TFS, "path": path}
    from grl.ops import linear_bwd_data, linear_bwd_weight, relu_grad

    out_l = linear_fwd(Zd, W, b, True)
    g_l = torch.randn_like(out_l)
    gm, mask = relu_grad(g_l, out_l)  # the layer backward's ReLU handling
    for name, fn in (("linear_mfma_bwd_data", lambda: linear_bwd_data(gm, mask, W)),
                     ("linear_mfma_bwd_weight", lambda: linear_bwd_weight(Zd, gm, mask, True))):
        ms = _time(fn, iters)
        res[name] = {"ms": ms, "TFLOPs_fp32_equivalent": flops / (ms * 1e-3) / 1e12,
                     "vs_f32_mfma_peak": flops / (ms * 1e-3) / 1e12 / F32_MFMA_PEAK_TFS, "path": path}
    del out_l, g_l, gm
    Wp = W.clone().requires_grad_(True)
    bp = b.clone().requires_grad_(True)
    Xl = X_full.detach()[: graph.num_cols].clone().requires_grad_(True)
    gl = graph.with_dropedge(DropEdge(0.3, 2, 1, True))

    def layer():  # the model's path: one autograd node
        graph_conv(Xl, gl, Wp, bp, relu=True).sum().backward()

    def layer_two_ops():
        graph_linear(typed_aggregate(Xl, gl), Wp, bp, relu=True).sum().backward()

    # 3 warm calls: the first builds the CSC and grows the caching allocator's pool
    res["graphconv_layer_fwd_bwd_p0.3"] = {"ms": _time(layer, max(3, iters // 2), warm=3)}
    res["graphconv_layer_fwd_bwd_p0.3_two_ops"] = {"ms": _time(layer_two_ops, max(3, iters // 2), warm=2)}
    del Z, dZ, Zd
    # inference: one grl_graphconv_fwd call, Z whole (7.2 GB) or in 1 GiB row chunks
    from grl.ops import graph_conv_infer
    Xe = X_full.detach()[: graph.num_cols]
    res["graphconv_infer_fwd"] = {"ms": _time(lambda: graph_conv_infer(Xe, graph, W, b, True), iters, warm=2)}
    res["graphconv_infer_fwd_z_chunks_1GiB"] = {
        "ms": _time(lambda: graph_conv_infer(Xe, graph, W, b, True, max_workspace_bytes=1 << 30), iters, warm=2)}
    return res


def c1_extras(dev, iters=20):
    """GraphCNNDropEdge(4369, 53, 6, 256) on the
    real debug.json page (N=74, 216 typed edges) built by the drop-in data
    pipeline; eval latency (B=1) three ways, one Adam train step (B=4), and
    the oracle's float64 numpy model (oracle/dense_ref.py) timed on the host
    as the CPU baseline, with a logits parity check."""
    from gnn.data_generator.data_process import HeuristicGraphBuilder, TextlineEncoding
    from gnn.models import GraphCNNDropEdge
    from oracle import dense_ref

    assets = os.path.join(HERE, "tests", "golden", "assets")
    with open(os.path.join(assets, "master_charset.json"), encoding="utf-8-sig") as f:
        char_to_id = {c: i for i, c in enumerate(json.load(f)["charset"])}
    with open(os.path.join(assets, "debug.json"), encoding="utf-8-sig") as f:
        regions = json.load(f)
    s = {"label": {i: dict(r, polygon=r["location"]) for i, r in enumerate(regions)}, "char_to_id": char_to_id}
    s = HeuristicGraphBuilder(6, "normal_binary")(TextlineEncoding(True)(s))
    V = torch.from_numpy(s["textline_encoding"])[None].to(dev)
    A = torch.from_numpy(s["adjacency_matrix"].astype(np.float32))[None].to(dev)  # collate layout (B,N,L,N)
    torch.manual_seed(0)
    model = GraphCNNDropEdge(4369, 53, 6, 256).to(dev).eval()
    res = {"nodes": int(V.shape[1]), "typed_edges": int((A != 0).sum())}
    with torch.no_grad():
        res["eval_ms_dense_A_in"] = _time(lambda: model([V, A]), iters)
        graph = model.to_graph(A)
        res["eval_ms_graph_prebuilt"] = _time(lambda: model([V, graph]), iters)
        logits = model([V, graph]).double().cpu().numpy()
        try:  # launch-bound at N=74: replay the whole forward as one HIP graph
            side = torch.cuda.Stream(dev)
            side.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(side):
                for _ in range(3):
                    model([V, graph])
            torch.cuda.current_stream(dev).wait_stream(side)
            hg = torch.cuda.CUDAGraph()
            with torch.cuda.graph(hg):
                out_static = model([V, graph])
            hg.replay()
            torch.cuda.synchronize()
            res["eval_ms_hip_graph"] = _time(hg.replay, iters)
            res["hip_graph_matches_eager"] = bool(torch.equal(out_static, model([V, graph])))
        except Exception as err:  # report, never fall back silently
            res["eval_ms_hip_graph"] = None
            res["hip_graph_error"] = repr(err)[:200]
    # CPU baseline (before the train steps below change the weights): the oracle's float64 restatement of the same forward
    P = {k: v.detach().double().cpu().numpy() for k, v in model.state_dict().items()}
    Vh, Ah = V.cpu().numpy(), A.cpu().numpy()
    ref = dense_ref.graph_cnn_dropedge_forward(P, Vh, Ah)
    t0, n = time.perf_counter(), 0
    while time.perf_counter() - t0 < 2.0 or n < 3:
        dense_ref.graph_cnn_dropedge_forward(P, Vh, Ah)
        n += 1
    res["cpu_eval_ms"] = (time.perf_counter() - t0) / n * 1e3
    # train step, B=4 (the reference's training batch), Adam as BuitlinOptimizer builds it
    model.train()
    V4, A4 = V.expand(4, -1, -1).contiguous(), A.expand(4, -1, -1, -1).contiguous()
    y4 = torch.randint(0, 53, (4, V.shape[1]), generator=torch.Generator().manual_seed(5)).to(dev)
    opt = torch.optim.Adam(model.parameters(), lr=1e-3)
    lossf = torch.nn.CrossEntropyLoss()

    def step():
        opt.zero_grad(set_to_none=True)
        loss = lossf(model.forward([V4, A4]).reshape(-1, 53), y4.reshape(-1))
        loss.backward()
        opt.step()

    res["train_step_ms_B4"] = _time(step, iters)
    res["cpu_kind"] = "port: oracle/dense_ref.py float64 numpy dense model (A_pre materialised like the reference)"
    res["logits_max_abs_diff_vs_oracle"] = float(np.abs(logits - ref).max())
    res["tolerance"] = 1e-4
    return res


def model_extras(dev, N=100_000, avg_deg=16.0, iters=3):
    """The whole GraphCNNDropEdge(4369, 53, 6, 256) on ONE synthetic graph of
    N nodes (C2's ER graph, bag-of-characters rows ~7 nonzeros of 4369):
    eval forward and one Adam train step (DropEdge p=0.3 x3, fused
    attention over all N nodes).  The reference's dense path cannot run this
    (A_pre alone would be (L+1)*N^2*4 B = 280 GB at N=100k)."""
    from gnn.models import GraphCNNDropEdge
    from grl import TypedGraph

    g = TypedGraph.synthetic(N, avg_deg, 6, seed=0, device=dev)
    gen = torch.Generator(device=dev).manual_seed(1)
    V = torch.zeros(1, N, 4369, device=dev)
    cols = torch.randint(0, 4365, (N, 7), generator=gen, device=dev)
    V[0].scatter_(1, cols, 1.0)
    V[0, :, -4:] = torch.rand(N, 4, generator=gen, device=dev)
    torch.manual_seed(0)
    model = GraphCNNDropEdge(4369, 53, 6, 256).to(dev)
    y = torch.randint(0, 53, (1, N), generator=gen, device=dev)
    opt = torch.optim.Adam(model.parameters(), lr=1e-3)
    lossf = torch.nn.CrossEntropyLoss()
    model.eval()
    with torch.no_grad():
        ev = _time(lambda: model([V, g]), iters)

    def step():
        opt.zero_grad(set_to_none=True)
        lossf(model.forward([V, g]).reshape(-1, 53), y.reshape(-1)).backward()
        opt.step()

    model.train()
    tr = _time(step, iters)
    return {"nodes": N, "typed_edges": g.nnz, "eval_ms": ev, "train_step_ms": tr,
            "note": "one graph, B=1; reference dense A_pre would need 280 GB"}


def model_mid_extras(dev, sizes=(512, 2048, 4096), iters=5):
    """BASELINE.md §2's orientation row "train fwd+bwd, B=1, random A (~3
    edges/node), N = 512 / 2048 / 4096" -- 0.16 s / 1.7-3.0 s / 9.2 s for the
    reference on an 8-core CPU -- through the drop-in: the same dense
    (B, N, 6, N) A the collate produces, GraphCNNDropEdge(4369, 53, 6, 256) in
    train mode (DropEdge and dropout active), cross-entropy, backward."""
    from gnn.models import GraphCNNDropEdge

    out = {}
    torch.manual_seed(0)
    model = GraphCNNDropEdge(4369, 53, 6, 256).to(dev)
    model.train()
    lossf = torch.nn.CrossEntropyLoss()
    ref = {512: "0.16 s", 2048: "1.7-3.0 s", 4096: "9.2 s"}
    for N in sizes:
        gen = torch.Generator(device=dev).manual_seed(N)
        A = (torch.rand(1, N, 6, N, generator=gen, device=dev) < 3.0 / (6 * N)).float()
        V = torch.zeros(1, N, 4369, device=dev)
        V[0].scatter_(1, torch.randint(0, 4365, (N, 7), generator=gen, device=dev), 1.0)
        y = torch.randint(0, 53, (1, N), generator=gen, device=dev)

        def step():
            model.zero_grad(set_to_none=True)
            lossf(model.forward([V, A]).reshape(-1, 53), y.reshape(-1)).backward()

        out[f"N{N}"] = {"train_fwd_bwd_ms": _time(step, iters, warm=2), "typed_edges": int(A.sum()),
                        "reference_cpu_orientation": ref.get(N)}
        del A, V
    return out


def run_only(args, graph, X_full, gather, spmm, L, F):
    """Kernel-isolated loop for rocprofv3 (kernel trace / PMC passes)."""
    from grl.ops import linear_fwd, typed_aggregate

    if args.only == "fwd":
        fn = spmm
    elif args.only == "bwd":
        Xg = X_full.detach().clone().requires_grad_(True)
        Z = typed_aggregate(Xg, graph)
        dZ = torch.randn_like(Z)
        graph.csc()
        fn = lambda: torch.autograd.grad(Z, Xg, dZ, retain_graph=True)  # noqa: E731
    elif args.only == "linear":
        Z = typed_aggregate(X_full, graph)
        W = torch.randn((L + 1) * F, F, device=X_full.device) / np.sqrt((L + 1) * F)
        fn = lambda: linear_fwd(Z, W, None, False)  # noqa: E731
    else:
        from grl.ops import graph_linear

        Xl = X_full.detach().clone().requires_grad_(True)
        W = (torch.randn((L + 1) * F, F, device=X_full.device) / np.sqrt((L + 1) * F)).requires_grad_(True)
        fn = lambda: graph_linear(typed_aggregate(Xl, graph), W, None, True).sum().backward()  # noqa: E731
    for _ in range(args.warmup):
        fn()
    torch.cuda.synchronize()
    for _ in range(args.steps):
        fn()
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
