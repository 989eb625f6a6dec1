#!/usr/bin/env python
"""Benchmark: typed-CSR SpMM (GraphConv aggregation, robust_gcn.py:45-47) on
MI355X -- BASELINE.json metric "aggregated edges/sec + SpMM HBM GB/s vs
roofline, d=256, 1/2/4/8 GPU".

    python bench.py [--gpus N --steps K --warmup W] [--workload C3|C4|C5|C2|weak]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU)
With --gpus N > 1 and no launcher (WORLD_SIZE unset) bench.py starts the N
rank processes itself (spawn_ranks); under a launcher WORLD_SIZE must equal N.

Workloads (BASELINE.json configs):
  C3 (default at N=1)  seeded Erdos-Renyi typed graph, N=1M, avg total
                       out-degree 32 over L=6 edge types (dedupe), d=256.
  C4 (default at N>1)  the same generator at a FIXED N=4M, node-range shards
                       over the N ranks (strong scaling), halo over RCCL.
  C5                   R-MAT scale 23 (N=8,388,608), avg_deg 64, d=512,
                       DropEdge p=0.2 fused, edge-balanced shards.
  C2                   ER N=100k, avg_deg 16, d=256.
  weak                 1M nodes per GPU (weak scaling; the round-1 N>1 line).
A step = one GraphConv aggregation forward over the rank's rows; at N>1 it
includes the halo exchange, pipelined with the aggregation over column slices
(grl.dist.HaloPipeline: slice c's rows travel while slice c-1 is
aggregated; bitwise equal to the unsliced result).  Inputs are resident in HBM
before timing.  Prints ONE JSON line on rank 0.
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


WORKLOADS = {  # name: (graph, nodes_total (None: per GPU), avg_deg, d, dropedge p)
    "C2": ("er", 100_000, 16.0, 256, 0.0),
    "C3": ("er", 1_000_000, 32.0, 256, 0.0),
    "C4": ("er", 4_000_000, 32.0, 256, 0.0),
    "C5": ("rmat", 1 << 23, 64.0, 512, 0.2),
    "weak": ("er", None, 32.0, 256, 0.0),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--option", action="append", default=[], metavar="NAME=VALUE",
                    help="a libgrl path option (grl_set_option) for this run, e.g. spmm_blocks_per_cu=16 (A/B aid)")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--workload", choices=["auto"] + list(WORKLOADS), default="auto",
                    help="auto: C3 on one GPU, C4 (fixed 4M nodes, strong scaling) on several")
    ap.add_argument("--nodes-per-gpu", type=int, default=None,
                    help="custom workload: nodes per GPU (overrides --workload's node count)")
    ap.add_argument("--avg-deg", type=float, default=None)
    ap.add_argument("--types", type=int, default=6)
    ap.add_argument("--dim", type=int, default=None)
    ap.add_argument("--p", type=float, default=None, help="DropEdge rate inside the timed step (0 = eval)")
    ap.add_argument("--graph", choices=["er", "rmat"], default=None)
    ap.add_argument("--node-order", choices=["auto", "given", "degree"], default="auto",
                    help="one GPU: relabel nodes by descending in-degree before timing (grl.graph.degree_order, a "
                         "one-time preprocessing of the graph); auto = degree for R-MAT, given for ER")
    ap.add_argument("--chunks", type=int, default=0,
                    help="N>1: column slices of the pipelined halo exchange (0 = d/128; 1 = serial)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline budget (0 disables)")
    ap.add_argument("--c4-reference", action="store_true",
                    help="N=1 C3 line: also time BASELINE's C4 graph whole on the one GPU (the N>1 lines' per-GPU "
                         "baseline; off by default: its launches are the headline kernel's and would skew the "
                         "rocprofv3 average of that kernel)")
    ap.add_argument("--extras", action="store_true",
                    help="also time fused-DropEdge fwd, backward, MFMA linear and a full layer (not the headline)")
    ap.add_argument("--dist-backend", default="nccl",
                    help="process-group backend for N>1 (nccl = RCCL; gloo only to smoke-test the N>1 path "
                         "with several ranks on one GPU)")
    ap.add_argument("--halo", choices=["auto", "sparse", "dense"], default="auto",
                    help="halo exchange layout for N>1 (grl/dist.py): sparse all-to-all-v of the referenced rows, "
                         "dense all-gather of every shard; auto picks dense when >=75%% of remote rows are referenced")
    ap.add_argument("--only", choices=["fwd", "bwd", "linear", "layer", "infer", "c1", "model"], default=None,
                    help="profiling aid: run just that kernel K times (no JSON line); c1: print the C1 "
                         "(debug.json model) timings alone")
    return ap.parse_args()


def resolve_workload(args, world):
    """Fill graph / nodes / avg_deg / dim / p from --workload, then apply the
    explicit overrides.  Returns (name, nodes_total, scaling)."""
    name = args.workload if args.workload != "auto" else ("C3" if world == 1 else "C4")
    graph, nodes, deg, dim, p = WORKLOADS[name]
    if nodes is None:
        nodes = 1_000_000 * world
    custom = args.nodes_per_gpu is not None or any(
        v is not None and v != d for v, d in ((args.avg_deg, deg), (args.dim, dim), (args.p, p), (args.graph, graph)))
    args.graph = args.graph or graph
    args.avg_deg = deg if args.avg_deg is None else args.avg_deg
    args.dim = dim if args.dim is None else args.dim
    args.p = p if args.p is None else args.p
    if args.nodes_per_gpu is not None:
        nodes = args.nodes_per_gpu * world
    if args.graph == "rmat":
        nodes = 1 << (nodes - 1).bit_length()
    scaling = "weak" if (name == "weak" or args.nodes_per_gpu is not None) else "strong"
    if world == 1:
        scaling = "weak"  # one GPU: nothing to scale; the driver's N=1 line
    return (name if not custom else name + "-shape (custom)"), nodes, scaling


def spmm_bytes(E, N, L, F, p, idx_bytes=4, ptr_bytes=4):
    """Algorithmic HBM bytes of one unfused typed-SpMM forward."""
    keep = 1.0 - p
    return keep * E * F * 4 + idx_bytes * E + ptr_bytes * (N * L + 1) + keep * N * F * 4 + N * (L + 1) * F * 4


def _grl_option(name):
    from grl import get_option

    return get_option(name)


def _grl_options(**kw):
    """grl.options: path options for a block (the chain forms the extras compare against)."""
    from grl import options

    return options(**kw)


def _events(n):
    return [torch.cuda.Event(enable_timing=True) for _ in range(n)]


def surface(what: str, dev) -> None:
    """grl.check() after a timed region: a persistent GraphConv kernel that
    gave up waiting on its LDS ring poisons its outputs (NaN) and sets a
    sticky word instead of raising at the call (stream-ordered, no host
    sync); a poisoned run must not be reported as a timing.  Exits non-zero
    naming the section and the entry point."""
    from grl import GrlError, device_check

    try:
        device_check(dev)
    except GrlError as err:
        raise SystemExit(f"bench.py: {what}: {err}")


def _free_port():
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_ranks(nproc):
    """`python bench.py --gpus N` (N > 1) without a launcher: start N rank
    processes of this same command (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_*
    as torch.distributed.run sets them, rendezvous on 127.0.0.1) and relay
    rank 0's output.  This parent never touches a GPU and never execs: it
    waits for the children, stops the rest when one fails, and exits with
    the first failing status."""
    import signal
    import subprocess
    import threading

    port = str(_free_port())
    procs = []
    signal.signal(signal.SIGTERM, lambda *_: (_ for _ in ()).throw(KeyboardInterrupt()))
    for r in range(nproc):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(nproc), LOCAL_WORLD_SIZE=str(nproc),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      stdout=subprocess.PIPE if r == 0 else None, text=True, start_new_session=True))

    def relay():  # rank 0's stdout (the JSON line), as it comes
        for line in procs[0].stdout:
            sys.stdout.write(line)
            sys.stdout.flush()

    t = threading.Thread(target=relay, daemon=True)
    t.start()
    status = 0
    live = set(range(nproc))

    def stop(ranks):
        for q in ranks:
            try:
                os.killpg(procs[q].pid, signal.SIGTERM)  # the exact process group this parent started
            except ProcessLookupError:
                pass

    try:
        while live:
            for r in sorted(live):
                rc = procs[r].poll()
                if rc is None:
                    continue
                live.discard(r)
                if rc != 0 and status == 0:
                    status = rc if rc > 0 else 128 - rc
                    print(f"bench.py: rank {r} exited with status {rc}; stopping the other ranks", file=sys.stderr,
                          flush=True)
                    stop(live)
            time.sleep(0.2)
    finally:  # Ctrl-C / SIGTERM of this parent: no rank keeps its GPU
        stop([q for q in live if procs[q].poll() is None])
    t.join(timeout=10)
    return status


def main():
    args = parse()
    if args.gpus < 1:
        raise SystemExit(f"--gpus must be >= 1 (got {args.gpus})")
    if "WORLD_SIZE" not in os.environ:
        if args.gpus > 1:
            raise SystemExit(spawn_ranks(args.gpus))
    elif int(os.environ["WORLD_SIZE"]) != args.gpus:
        raise SystemExit(f"bench.py: WORLD_SIZE={os.environ['WORLD_SIZE']} from the launcher but --gpus {args.gpus}: "
                         "launch one rank per GPU with --gpus equal to the number of ranks")
    if args.option:  # (each rank, after the spawn) before any kernel: a workspace query and its call see the same
        from grl import set_option

        for kv in args.option:
            name, _, value = kv.partition("=")
            set_option(name.strip(), int(value))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    ndev = torch.cuda.device_count()
    if ndev == 0:
        raise SystemExit(f"bench.py rank {rank}: no ROCm GPU visible (the path runs on MI355X only)")
    # one visible GPU per rank (a launcher that isolates devices) -> cuda:0; otherwise LOCAL_RANK picks it
    if args.dist_backend == "nccl" and world > 1 and ndev > 1 and local_rank >= ndev:
        raise SystemExit(f"rank {rank}: LOCAL_RANK {local_rank} but only {ndev} GPU(s) visible")
    dev = torch.device("cuda", local_rank % ndev)
    torch.cuda.set_device(dev)
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(args.dist_backend)

    if args.only == "c1":
        res = {"c1_debug_json": c1_extras(dev, max(3, args.steps))}
        surface("c1", dev)
        print(json.dumps(res), flush=True)
        return
    if args.only == "model":
        res = {"model_one_graph_100k": model_extras(dev), "model_dense_A_mid_n": model_mid_extras(dev)}
        surface("model", dev)
        print(json.dumps(res), flush=True)
        return

    from grl import DropEdge
    from grl.dist import HaloPipeline, ShardedGraph
    from grl.ops import spmm_forward

    wname, N, scaling = resolve_workload(args, world)
    L, F = args.types, args.dim
    node_order = args.node_order if args.node_order != "auto" else ("degree" if args.graph == "rmat" else "given")
    t0 = time.time()
    if world > 1 and node_order == "degree":
        # every rank builds the whole (deterministic) graph, relabels it and keeps its row range:
        # the CSR is small next to the features (C5: 2.3 GB vs 17 GB)
        from grl import TypedGraph
        from grl.graph import degree_order

        g_all, _ = degree_order(TypedGraph.synthetic(N, args.avg_deg, L, kind=args.graph, seed=0, device=dev))
        sg = ShardedGraph.from_graph(g_all, halo=args.halo)
        del g_all
    else:
        sg = ShardedGraph.synthetic(N, args.avg_deg, L, kind=args.graph, seed=0, device=dev, halo=args.halo)
    graph, plan = sg.graph, sg.plan
    n_loc = plan.n_loc
    E_loc, E_tot = graph.nnz, plan.num_edges_total
    gen = torch.Generator(device=dev)
    gen.manual_seed(1 + rank)
    X_loc = torch.randn(n_loc, F, generator=gen, device=dev, dtype=torch.float32)
    order_ab = None
    de = DropEdge(args.p, 2, 0, True) if args.p > 0 else None
    if node_order == "degree" and world == 1:
        from grl.graph import degree_order

        if args.only is None:  # (a profiled run keeps only the timed kernel's launches)
            order_ab = {"given_ms": _time(lambda: spmm_forward(X_loc, graph.with_dropedge(de)), 3)}
        t1 = time.time()
        graph, perm = degree_order(graph)
        X_loc = X_loc[perm].contiguous()  # features enter the relabelled graph once
        if order_ab is not None:
            order_ab["relabel_s"] = time.time() - t1
        del perm
    g_step = graph.with_dropedge(de)
    stream = torch.cuda.current_stream(dev)
    Z = torch.empty(graph.num_rows, graph.segments * F, device=dev)  # preallocated: no allocation in the step
    chunks = args.chunks or max(1, F // 128)
    pipe = X_full = None
    if world > 1:
        pipe = HaloPipeline(sg, F, chunks=chunks, device=dev)

        def step():
            pipe.run(X_loc, Z, de)
    else:
        X_full = X_loc

        def step():
            spmm_forward(X_full, g_step, out=Z)
    build_s = time.time() - t0

    if args.only is not None:
        if world > 1:
            raise SystemExit("--only profiles one GPU")
        run_only(args, graph, X_full, step, L, F)
        return

    for _ in range(args.warmup):
        step()
    ev_s, ev_e = _events(args.steps), _events(args.steps)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    for i in range(args.steps):
        ev_s[i].record(stream)
        step()
        ev_e[i].record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    wall = time.perf_counter() - t_start
    surface("timed region", dev)
    per_step = [a.elapsed_time(b) for a, b in zip(ev_s, ev_e)]
    step_ev_ms = float(np.mean(per_step))
    halo = None
    if world > 1:
        halo = halo_breakdown(args, pipe, X_loc, Z, de, g_step, dev)
        kern_ms = halo["spmm_only_ms"]
        tt = torch.tensor([wall, kern_ms, step_ev_ms], dtype=torch.float64,
                          device=dev if args.dist_backend == "nccl" else "cpu")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        wall, kern_ms, step_ev_ms = float(tt[0]), float(tt[1]), float(tt[2])
    else:
        kern_ms = step_ev_ms
    ms_step = wall / args.steps * 1e3
    value = E_tot / (wall / args.steps)

    bytes_launch = spmm_bytes(E_loc, n_loc, L, F, args.p)
    achieved = bytes_launch / (kern_ms * 1e-3) / 1e9
    wide = F > 256 and graph.num_cols * F * 4 > (12 << 30)
    kernel = (f"spmm_kernel<4,{2 if wide else 1},{4 if wide else 8},false,false> (grl_typed_spmm_fwd)" if world == 1
              else f"spmm_kernel / spmm_pair_kernel (grl_typed_spmm_fwd_slice, {chunks} slices of {F // chunks} "
                   "columns)")
    traffic = load_traffic(args, wname, n_loc, world, kernel)
    # achieved counts algorithmic bytes.  On a degree-ordered R-MAT graph hot rows are re-read from
    # the Infinity Cache / L2, so it can exceed what HBM delivers ("cache-amplified"); the PMC
    # traffic rate (L2-miss reads + writes per launch over the same kernel time) is the HBM figure.
    amplified = node_order == "degree"
    traffic_rate = traffic / (kern_ms * 1e-3) / 1e9 if traffic else None
    gname = "Erdos-Renyi" if args.graph == "er" else "R-MAT (a,b,c,d = 0.57,0.19,0.19,0.05)"
    out = {
        "metric": METRIC, "value": value, "unit": "edges/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": ms_step, "higher_is_better": True, "scaling": scaling,
        "vs_baseline": None, "dtype": "f32",
        "data": f"synthetic: seeded {gname} typed graph (graph seed 0), X ~ N(0,1) fp32 (seed 1+rank)",
        "config": {"workload": wname, "description": f"{args.graph.upper()} typed graph, {N} nodes "
                   f"({'one GPU' if world == 1 else f'{world} node-range shards'}), avg_deg {args.avg_deg:g} over "
                   f"L={L} edge types, d={F}, typed-SpMM forward (GraphConv aggregation)"
                   f"{' + DropEdge p=%g' % args.p if args.p else ''}",
                   "nodes_total": N, "edges_total": E_tot, "nodes_per_gpu_rank0": n_loc, "avg_deg": args.avg_deg,
                   "num_types": L, "d": F, "dropedge_p": args.p, "graph": args.graph,
                   "parallelism": "single GPU" if world == 1 else
                   f"node-range shards x{world}, "
                   + ("RCCL" if args.dist_backend == "nccl" else f"{args.dist_backend} (host-staged)") + " "
                   + ("all-gather (dense halo)" if plan.mode == "dense" else "all-to-all-v (sparse halo)")
                   + f" pipelined over {chunks} column slices, rank 0 references {plan.referenced_halo_rows} of "
                   f"{N - n_loc} remote rows"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "achieved_basis": ("algorithmic bytes, cache-amplified: hot rows of the degree-ordered graph "
                                        "are re-read from the Infinity Cache / L2; traffic_GBps is the HBM figure")
                     if amplified else "algorithmic bytes (SURVEY.md §8(d))",
                     "traffic_GBps": traffic_rate,
                     "traffic_frac": traffic_rate / HBM_PEAK_GBS if traffic_rate else None,
                     "kernel": kernel,
                     "traffic_note": None if traffic else
                     ("no PMC record of this kernel for this workload and world size (a shard's slice kernels over "
                      "its [own | halo] table were never profiled): traffic unmeasured" if world > 1 else
                      "no PMC record for this workload: traffic unmeasured"),
                     "kernel_ms": kern_ms, "kernel_ms_min_max": [min(per_step), max(per_step)] if world == 1 else None,
                     "launches": {"timed": args.steps, "warmup": args.warmup,
                                  "other": 5 if wname.startswith("C3") else 0,
                                  "note": "warmup + timed launches of this kernel, plus `other` launches of it for "
                                          "dropedge_train_p0.3's forward (p=0.3, fewer bytes, faster): a rocprofv3 "
                                          "average over the process reads that much lower"}
                     if world == 1 else None,
                     "algorithmic_bytes_per_launch": bytes_launch},
        "build_s": build_s,
    }
    if halo is not None:
        out["halo"] = halo
    out["config"]["node_order"] = ("degree-sorted node ids (one-time relabel of the same graph, "
                                   "grl.graph.degree_order)" if node_order == "degree" else "as generated")
    if order_ab is not None:
        order_ab["degree_ms"] = kern_ms
        out["node_order_ab"] = order_ab
    if args.graph == "rmat":
        out["config"]["split"] = graph.split_stats()
        out["config"]["max_row_edges"] = int((graph.rowptr[L::L] - graph.rowptr[:-1:L]).max())
    if rank == 0 and args.cpu_seconds > 0:
        if world == 1:
            out["cpu_baseline"], out["parity"] = cpu_baseline(args, g_step, X_loc, Z, L, F)
        else:  # rank 0's node-range shard on the host cores: the same rows, the same [own | halo] table
            out["cpu_baseline"], out["parity"] = cpu_baseline_shard(args, g_step, pipe, Z, L, F, world)
    if world > 1:
        dist.barrier()  # the other ranks wait while rank 0 times the host baseline
    # C3 and C3-sized custom shapes (a second Z of a d = 512, 8M-node graph would not fit beside the first)
    if world == 1 and wname.startswith("C3") and Z.numel() * 4 <= (64 << 30):
        out["dropedge_train_p0.3"] = dropedge_train(graph, X_loc, E_loc, 3)
        surface("dropedge_train_p0.3", dev)
        if args.c4_reference:
            out["C4_one_gpu"] = c4_one_gpu(dev, max(3, min(10, args.steps)))
            surface("C4_one_gpu", dev)
    if args.extras and world == 1:
        out["extras"] = extras(args, graph, X_loc, L, F, dev, E_loc, n_loc)
        surface("extras (layers)", dev)
        del X_loc, X_full, Z
        torch.cuda.empty_cache()  # C1 is a small-graph workload: time it without C3's 8 GB resident
        out["extras"]["c1_debug_json"] = c1_extras(dev)
        surface("extras c1_debug_json", dev)
        out["extras"]["model_one_graph_100k"] = model_extras(dev)
        surface("extras model_one_graph_100k", dev)
        out["extras"]["model_dense_A_mid_n"] = model_mid_extras(dev)
        surface("extras model_dense_A_mid_n", dev)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def halo_breakdown(args, pipe, X_loc, Z, de, g_step, dev, iters=None):
    """Where an N>1 step goes (this rank; the caller takes the max over ranks
    of the aggregation alone): the exchange alone, the aggregation alone (all
    slices, tables resident), and the serial sum -- next to the pipelined step
    the headline times."""
    from grl.ops import spmm_forward_slice

    iters = iters or max(3, min(10, args.steps))
    g = g_step

    def exchange_only():
        pipe._pack(X_loc)
        for c in range(pipe.K):
            pipe._exchange(c) if pipe.side is None else _wait(pipe._exchange(c))

    def aggregate_only():
        for c in range(pipe.K):
            spmm_forward_slice(pipe.tables[c], g, Z, c * pipe.Fc)

    def _wait(w):
        if w is not None:
            w.wait()

    ex = _time(exchange_only, iters)
    ag = _time(aggregate_only, iters)
    plan = pipe.plan
    world = len(plan.bounds) - 1
    rows_in = (world - 1) * plan.stride if plan.mode == "dense" else sum(plan.recv_counts)
    out = {"mode": plan.mode, "chunks": pipe.K, "exchange_only_ms": ex, "spmm_only_ms": ag,
           "serial_sum_ms": ex + ag, "rows_received_rank0": rows_in,
           "GB_received_rank0": rows_in * pipe.F * 4 / 1e9,
           "GBps_received_rank0": rows_in * pipe.F * 4 / 1e9 / (ex * 1e-3) if ex > 0 else None}
    try:
        out["backward"] = halo_backward_breakdown(pipe, g, dev, iters)
    except Exception as err:  # reported, never hidden; the forward line stands on its own
        out["backward"] = {"error": repr(err)[:300]}
    return out


def halo_backward_breakdown(pipe, g, dev, iters):
    """The training-mode counterpart (not the headline): dX of the shard with
    the reverse exchange pipelined with the column-slice gathers
    (HaloPipeline.backward), next to its parts -- the slice gathers alone and
    the reverse exchanges alone (CSC built once per graph, outside)."""
    from grl.ops import spmm_backward_slice

    F, K = pipe.F, pipe.K
    g.csc()
    dZ = torch.randn(pipe.plan.n_loc, g.segments * F, generator=torch.Generator(device=dev).manual_seed(5),
                     device=dev)
    gt, _ = pipe._grad_buffers(dev)
    dX = pipe.backward(dZ, g.dropedge)  # warm: buffers, split plans
    pipelined = _time(lambda: pipe.backward(dZ, g.dropedge), iters)

    def gathers():
        for c in range(K):
            spmm_backward_slice(dZ, g, c * pipe.Fc, gt[c])

    def exchanges():
        for c in range(K):
            w = pipe._exchange_back(c, async_op=pipe.side is not None)
            if w is not None:
                w.wait()

    ga, ex = _time(gathers, iters), _time(exchanges, iters)
    del dX, dZ
    return {"pipelined_ms": pipelined, "gather_only_ms": ga, "exchange_only_ms": ex, "serial_sum_ms": ga + ex,
            "note": "dX = A_drop^T dZ of the shard: grl_typed_spmm_bwd_slice per column slice, reverse halo "
                    "all-to-all per slice in flight under the next gather, peer-order combine"}


def c4_one_gpu(dev, iters):
    """BASELINE's C4 graph (ER, N=4M, avg_deg 32, d=256) aggregated on ONE
    GPU, next to the N=1 headline: the per-GPU reference the driver's N>1
    lines (C4 sharded 2/4/8 ways, strong scaling) are measured against."""
    from grl import TypedGraph
    from grl.ops import spmm_forward

    N, deg, L, F = WORKLOADS["C4"][1], WORKLOADS["C4"][2], 6, WORKLOADS["C4"][3]
    g = TypedGraph.synthetic(N, deg, L, kind="er", seed=0, device=dev)
    X = torch.randn(N, F, generator=torch.Generator(device=dev).manual_seed(1), device=dev)
    Z = torch.empty(N, 7 * F, device=dev)
    ms = _time(lambda: spmm_forward(X, g, out=Z), iters)
    alg = spmm_bytes(g.nnz, N, L, F, 0.0)
    res = {"nodes": N, "edges": g.nnz, "ms": ms, "edges_per_s": g.nnz / (ms * 1e-3),
           "alg_GBps": alg / (ms * 1e-3) / 1e9, "frac_of_8TBps": alg / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
           "note": "C4's whole 4M-node graph on one GPU (same kernel as the headline); the N>1 lines shard it"}
    del g, X, Z
    torch.cuda.empty_cache()
    return res


def dropedge_train(graph, X, E, iters):
    """The training-mode aggregation next to the headline: fused DropEdge
    p=0.3 forward and its backward (CSC gather, same regenerated mask)."""
    from grl import DropEdge
    from grl.ops import spmm_backward, spmm_forward

    g = graph.with_dropedge(DropEdge(0.3, 2, 7, True))
    graph.csc()  # built once per graph, cached (not part of the step)
    Zd = spmm_forward(X, g)
    dZ = torch.randn_like(Zd)
    fwd = _time(lambda: spmm_forward(X, g, out=Zd), iters)
    bwd = _time(lambda: spmm_backward(dZ, g, X.shape[1]), iters)
    del Zd, dZ
    return {"fwd_ms": fwd, "bwd_ms": bwd, "fwd_bwd_edges_per_s": E / ((fwd + bwd) * 1e-3),
            "note": "fused DropEdge p=0.3 (seed 2, call 7): forward SpMM + CSC-gather backward"}


def traffic_key(wname, world, args, n_loc):
    """Key of a PMC record in profiles/pmc_traffic.json: the workload, the
    world size and the shard shape (a record is only ever the kernel it was
    measured on, for that workload at that world size)."""
    return (f"{wname}_w{world}_{args.graph}_n{n_loc}_deg{args.avg_deg:g}_L{args.types}_d{args.dim}"
            f"_p{args.p:g}")


def load_traffic(args, wname, n_loc, world, kernel):
    """HBM bytes per launch of `kernel` from a committed rocprofv3 PMC summary
    of the same workload at the same world size and shard shape, on the same
    kernel family (profiles/pmc_traffic.json, written by tools/pmc_traffic.py
    for one GPU and tools/pmc_rank_traffic.py for a rank's slice kernels over
    its [own | halo] table), or None when no such record exists (one GPU's
    whole-graph bytes are never a shard's traffic)."""
    path = os.path.join(HERE, "profiles", "pmc_traffic.json")
    if not os.path.exists(path):
        return None
    try:
        rec = json.load(open(path)).get(traffic_key(wname, world, args, n_loc))
    except (OSError, ValueError):  # unreadable summary: report traffic as unmeasured
        return None
    family = rec.get("kernel", "").replace(" ", "").split("<")[0].split("(")[0] if rec else ""
    if not family or not str(kernel).replace(" ", "").startswith(family):
        return None
    return rec.get("hbm_bytes_per_launch")


def host_cpu_info():
    """The host the CPU baseline runs on: model name, logical CPUs the OS
    reports, the CPUs this process may run on, and the cgroup CPU quota."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        affinity = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        affinity = os.cpu_count()
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            quota = None if q == "max" else float(q) / float(per)
    except (OSError, ValueError):
        pass
    return {"cpu_model": model, "os_cpu_count": os.cpu_count(), "affinity_cpus": affinity, "cgroup_cpu_quota": quota}


def cpu_threads(info):
    """every core the process can use -- os.cpu_count()
    unless the affinity mask or the cgroup quota grants fewer (threads beyond
    those only time-slice the same cores)."""
    n = info["os_cpu_count"] or 1
    n = min(n, info["affinity_cpus"] or n)
    if info["cgroup_cpu_quota"]:
        n = min(n, max(1, int(info["cgroup_cpu_quota"])))
    return n


def cpu_baseline(args, graph, X, Z, L, F):
    """Oracle (grl_oracle.c, OpenMP) over the WHOLE graph and the same
    features, with every usable host core; also checks every GPU row of Z
    bitwise against it."""
    from oracle import c_oracle

    info = host_cpu_info()
    threads = cpu_threads(info)
    n = graph.num_rows
    # the whole graph, unless Z would not fit the host comfortably twice (C5: 120 GB): then
    # SURVEY.md §8(d)'s 1/8 shard -- the edge-balanced node range rank 3 of 8 would own
    # (grl.dist.edge_balanced_bounds, as the N=8 run shards it: ~E/8 edges; a fixed 1/8 of
    # the rows of a degree-ordered graph would hold almost no edges)
    whole = Z.numel() * 4 <= (16 << 30)
    if whole:
        r0, r1 = 0, n
    else:
        from grl.dist import edge_balanced_bounds

        b8 = edge_balanced_bounds((graph.rowptr[L::L] - graph.rowptr[:-1:L]).to(torch.int64), 8)
        r0, r1 = b8[3], b8[4]
    rp = graph.rowptr[r0 * L: r1 * L + 1].cpu().numpy()
    e0 = int(rp[0])
    rowptr = rp - e0
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
    equal = bool(np.array_equal(Zg, Zc))
    diff = 0.0 if equal else float(np.abs(Zg.astype(np.float64) - Zc).max())
    what = (f"the whole graph ({n} nodes, {E} typed edges)" if whole else
            f"the edge-balanced 1/8 node-range shard rank 3 of 8 would own, rows [{r0}, {r1}) ({E} of {graph.nnz} "
            "typed edges; edges/s of the shard)")
    cpu = {"value": E * passes / dt, "unit": "edges/s", "cores": threads, "kind": "port",
           "sample": f"{what} and X, {passes} pass(es) in {dt:.1f}s; oracle/grl_oracle.c OpenMP typed-CSR SpMM, "
                     f"{threads} threads", **info}
    parity = {"rows_checked": int(r1 - r0), "max_abs_diff": diff, "bitwise_equal": equal, "tolerance": 1e-4}
    return cpu, parity


def cpu_baseline_shard(args, graph, pipe, Z, L, F, world):
    """N>1: the oracle (grl_oracle.c, OpenMP, every usable host core) over
    rank 0's node-range shard -- its typed-CSR rows with the local / halo
    column ids and the exchanged [own | halo] feature table the pipeline
    holds after the timed steps -- and every row of rank 0's Z compared
    bitwise against it.  edges/s of the shard (E_loc per pass); the whole
    graph is P such shards, so the host's whole-graph rate is this rate."""
    from oracle import c_oracle

    info = host_cpu_info()
    threads = cpu_threads(info)
    rowptr = graph.rowptr.cpu().numpy()
    colidx = graph.colidx.cpu().numpy()
    tables = pipe.tables  # [chunks, rows, F / chunks]: slice c = columns [c Fc, (c + 1) Fc)
    X_ext = tables.permute(1, 0, 2).reshape(tables.shape[1], F).cpu().numpy()
    E = int(rowptr[-1])
    d = None if args.p <= 0 else c_oracle.drop(args.p, 2, 0, True)
    split = (graph.split_threshold, graph.split_chunk)
    t0 = time.perf_counter()
    passes = 0
    while True:
        Zc = c_oracle.spmm_fwd(rowptr, colidx, X_ext, L, True, d=d, nthreads=threads, split=split,
                               edge_base=graph.edge_id_base, self_base=graph.self_id_base)
        passes += 1
        if time.perf_counter() - t0 >= args.cpu_seconds:
            break
    dt = time.perf_counter() - t0
    Zg = Z.cpu().numpy()
    equal = bool(np.array_equal(Zg, Zc))
    diff = 0.0 if equal else float(np.abs(Zg.astype(np.float64) - Zc).max())
    cpu = {"value": E * passes / dt, "unit": "edges/s", "cores": threads, "kind": "port",
           "sample": f"rank 0's node-range shard of {world} ({graph.num_rows} rows, {E} typed edges, "
                     f"[own | halo] table of {X_ext.shape[0]} rows), {passes} pass(es) in {dt:.1f}s; "
                     f"oracle/grl_oracle.c OpenMP typed-CSR SpMM, {threads} threads (edges/s of the shard)", **info}
    parity = {"rows_checked": int(graph.num_rows), "scope": "every row of rank 0's shard", "max_abs_diff": diff,
              "bitwise_equal": equal, "tolerance": 1e-4}
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


def extras(args, graph, X_full, L, F, dev, E_loc, n_loc):
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
            if _grl_option("gemm_x6") != 0 else "fp32 MFMA v_mfma_f32_32x32x2_f32")
    res["linear_mfma_fwd"] = {"ms": ms, "TFLOPs_fp32_equivalent": flops / (ms * 1e-3) / 1e12,
                              "vs_f32_mfma_peak": flops / (ms * 1e-3) / 1e12 / F32_MFMA_PEAK_TFS, "path": path}
    from grl.ops import linear_bwd_data, linear_bwd_weight, relu_grad

    out_l = linear_fwd(Zd, W, b, True)
    g_l = torch.randn_like(out_l)
    gm, mask, _ = relu_grad(g_l, out_l)  # the layer backward's ReLU handling
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

    # the layer alone: a fixed upstream gradient (not .sum()'s expanded ones and its reduction) and the
    # parameter grads reset per call, as a training step's zero_grad does (no accumulation adds)
    gout = torch.randn(graph.num_rows, Wp.shape[1], device=dev)

    def run_layer(fn):
        Xl.grad = Wp.grad = bp.grad = None
        fn().backward(gout)

    def layer():  # the model's path: one autograd node
        run_layer(lambda: graph_conv(Xl, gl, Wp, bp, relu=True))

    def layer_two_ops():
        run_layer(lambda: graph_linear(typed_aggregate(Xl, gl), Wp, bp, relu=True))

    # 3 warm calls: the first builds the CSC and grows the caching allocator's pool
    res["graphconv_layer_fwd_bwd_p0.3"] = {"ms": _time(layer, max(3, iters // 2), warm=3),
                                           "path": "fwd: one kernel writing Z; bwd: ReLU mask + db in one pass "
                                                   "(grl_relu_grad), dX one kernel over the typed transpose "
                                                   "(grl_graphconv_bwd_data), dW GEMM",
                                           "harness": "out.backward(fixed upstream gradient), parameter grads reset "
                                                      "per call"}
    res["graphconv_layer_fwd_bwd_p0.3_recompute"] = {
        "ms": _time(lambda: run_layer(lambda: graph_conv(Xl, gl, Wp, bp, relu=True, recompute=True)),
                    max(3, iters // 2), warm=2),
        "path": "keeps X, not Z (7.2 GB less held): fwd one kernel without Z; bwd dX one kernel that also writes "
                "G_s = A_s^T g, dW_s = X^T G_s (no re-aggregation)"}
    with _grl_options(graphconv_fused_bwd=0):
        res["graphconv_layer_fwd_bwd_p0.3_chain_bwd"] = {
            "ms": _time(layer, max(3, iters // 2), warm=2),
            "path": "bwd dX as autograd's chain: dZ = g W^T (x6 GEMM), then the CSC gather"}
    res["graphconv_layer_fwd_bwd_p0.3_two_ops"] = {"ms": _time(layer_two_ops, max(3, iters // 2), warm=2)}
    from grl.ops import graph_conv_bwd_data, linear_bwd_data, spmm_backward

    gC = torch.randn(graph.num_rows, F, device=dev)
    if graph_conv_bwd_data(gC, gl, W, F) is not None:  # builds the typed transpose once (cached per graph)
        res["graphconv_bwd_data_p0.3"] = {
            "one_kernel_ms": _time(lambda: graph_conv_bwd_data(gC, gl, W, F), iters),
            "chain_ms": _time(lambda: spmm_backward(linear_bwd_data(gC, None, W), gl, F), iters)}
    del gC
    del Z, dZ, Zd, gout
    # inference: one grl_graphconv_fwd call -- the one-kernel form (Z stays on
    # chip, graphconv.hip), and the two-kernel form (Z whole, 7.2 GB, or in
    # 1 GiB row chunks) for comparison; all bitwise equal
    from grl.ops import graph_conv_infer
    Xe = X_full.detach()[: graph.num_cols]
    fused = graph_conv_infer(Xe, graph, W, b, True)
    res["graphconv_infer_fwd"] = {"ms": _time(lambda: graph_conv_infer(Xe, graph, W, b, True), iters, warm=2),
                                  "path": "one kernel (graphconv_ws_kernel): gather waves + MFMA waves, Z in LDS"}
    with _grl_options(graphconv_fused=0):
        two = graph_conv_infer(Xe, graph, W, b, True)
        res["graphconv_infer_fwd_two_kernels"] = {
            "ms": _time(lambda: graph_conv_infer(Xe, graph, W, b, True), iters, warm=2),
            "bitwise_equal_to_one_kernel": bool(torch.equal(two, fused))}
        res["graphconv_infer_fwd_two_kernels_z_chunks_1GiB"] = {
            "ms": _time(lambda: graph_conv_infer(Xe, graph, W, b, True, max_workspace_bytes=1 << 30), iters,
                        warm=2)}
    del fused, two, Xe, Xl, Wp, bp
    torch.cuda.empty_cache()
    res["graphconv_wide_layers"] = wide_layers(graph, dev, max(3, iters // 2))
    return res


def wide_layers(graph, dev, iters):
    """The wide GraphConv shapes next to their chains, on the headline graph
    with DropEdge p = 0.3 and ReLU (verdict r3 item 1): gcn3 at d = 256 (F =
    2C = 512 from cat[g1, g2], drop_robust_gcn.py:84-85) and a d = 512 layer
    (C5's width; gcn1/gcn2 at F = C = 512).  Per shape: inference (one
    grl_graphconv_fwd call) and the layer fwd+bwd through graph_conv, one
    kernel vs the graphconv_fused / graphconv_fused_bwd path options at 0 (SpMM writing
    Z + x6 GEMM; dZ GEMM + CSC gather); forward bitwise checked."""
    from grl import DropEdge
    from grl.ops import graph_conv, graph_conv_infer

    gl = graph.with_dropedge(DropEdge(0.3, 2, 1, True))
    gen = torch.Generator(device=dev).manual_seed(11)
    out = {}
    for name, F, C in (("gcn3_d256_F512_C256", 512, 256), ("d512_F512_C512", 512, 512)):
        X = torch.randn(graph.num_cols, F, device=dev, generator=gen)
        W = torch.randn(graph.segments * F, C, device=dev, generator=gen) / (graph.segments * F) ** 0.5
        b = torch.randn(C, device=dev, generator=gen)
        gout = torch.randn(graph.num_rows, C, device=dev, generator=gen)
        Xp, Wp, bp = (t.clone().requires_grad_(True) for t in (X, W, b))

        def layer():
            Xp.grad = Wp.grad = bp.grad = None
            graph_conv(Xp, gl, Wp, bp, relu=True).backward(gout)

        r = {}
        one = graph_conv_infer(X, gl, W, b, True)
        r["infer_one_kernel_ms"] = _time(lambda: graph_conv_infer(X, gl, W, b, True), iters)
        r["layer_fwd_bwd_one_kernel_ms"] = _time(layer, iters, warm=2)
        with _grl_options(graphconv_fused=0, graphconv_fused_bwd=0):
            r["infer_bitwise_equal_to_chain"] = bool(torch.equal(graph_conv_infer(X, gl, W, b, True), one))
            r["infer_chain_ms"] = _time(lambda: graph_conv_infer(X, gl, W, b, True), iters)
            r["layer_fwd_bwd_chain_ms"] = _time(layer, iters, warm=1)
        r["kernel"] = ("graphconv_ws_kernel: two 256-column virtual segments per segment" +
                       (", 4 gather + 8 MFMA waves (C = 512)" if C > 256 else ", 8 gather + 4 MFMA waves"))
        out[name] = r
        del X, W, b, gout, Xp, Wp, bp, one
        torch.cuda.empty_cache()
    return out


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
    # parity (before the train steps below change the weights): the oracle's float64 restatement
    sd = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    P = {k: v.double().numpy() for k, v in sd.items()}
    Vh, Ah = V.cpu().numpy(), A.cpu().numpy()
    ref = dense_ref.graph_cnn_dropedge_forward(P, Vh, Ah)
    # CPU baseline: the reference's own math in fp32 torch on every usable host core
    # (oracle/dense_torch.py: dense A_pre, dense Bernoulli masks in training)
    from oracle import dense_torch

    info = host_cpu_info()
    threads_before = torch.get_num_threads()
    torch.set_num_threads(cpu_threads(info))
    Pf = {k: v.float() for k, v in sd.items()}
    Vc, Ac = V.cpu(), A.cpu()

    def cpu_time(fn, budget=2.0):
        fn()
        t0, n = time.perf_counter(), 0
        while time.perf_counter() - t0 < budget or n < 3:
            fn()
            n += 1
        return (time.perf_counter() - t0) / n * 1e3

    with torch.no_grad():
        res["cpu_eval_ms"] = cpu_time(lambda: dense_torch.forward(Pf, Vc, Ac))
    cpu_step = dense_torch.TrainStep(sd)
    V4c, A4c = Vc.expand(4, -1, -1).contiguous(), Ac.expand(4, -1, -1, -1).contiguous()
    y4c = torch.randint(0, 53, (4, V.shape[1]), generator=torch.Generator().manual_seed(5))
    res["cpu_train_step_ms_B4"] = cpu_time(lambda: cpu_step(V4c, A4c, y4c))
    res["cpu_threads"] = torch.get_num_threads()
    res["cpu_model"] = info["cpu_model"]
    torch.set_num_threads(threads_before)
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
    # the same step with the batch graph prebuilt, eager and as ONE HIP graph (device-seeded DropEdge
    # and feature dropout redraw on every replay; capturable Adam)
    g4 = model.to_graph(A4)
    opt_c = torch.optim.Adam(model.parameters(), lr=1e-3, capturable=True)

    def step_c():
        loss = lossf(model.forward([V4, g4]).reshape(-1, 53), y4.reshape(-1))
        loss.backward()
        opt_c.step()
        return loss

    def step_c_eager():
        opt_c.zero_grad(set_to_none=True)
        step_c()

    res["train_step_ms_B4_graph_prebuilt"] = _time(step_c_eager, iters)
    try:
        side = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            for _ in range(3):
                step_c_eager()
        torch.cuda.current_stream(dev).wait_stream(side)
        hg = torch.cuda.CUDAGraph()
        opt_c.zero_grad(set_to_none=True)
        with torch.cuda.graph(hg):
            step_c()
        res["train_step_ms_B4_hip_graph"] = _time(hg.replay, iters)
    except Exception as err:  # report, never fall back silently
        res["train_step_ms_B4_hip_graph"] = None
        res["train_hip_graph_error"] = repr(err)[:200]
    try:  # the product's own training loop on debug.json pages: KVProcedure._run_train_step per batch
        res["warper_train_step_B4"] = c1_procedure_steps(dev, iters)
    except Exception as err:  # report, never fall back silently
        res["warper_train_step_B4"] = {"error": repr(err)[:300]}
    res["cpu_kind"] = ("port: oracle/dense_torch.py, the reference's dense fp32 torch math on CPU (A_pre "
                       "materialised, Bernoulli masks over it in training, Adam)")
    res["logits_max_abs_diff_vs_oracle"] = float(np.abs(logits - ref).max())
    res["tolerance"] = 1e-4
    return res


def _debug_datapile(root, copies=8, seed=0):
    """`copies` debug.json pages (N=74) as VIA datapile documents with seeded
    random sumi labels: the reference's training input format
    (datapile_dataset.py), one page size, so every B=4 batch has one shape."""
    assets = os.path.join(HERE, "tests", "golden", "assets")
    with open(os.path.join(assets, "debug.json"), encoding="utf-8-sig") as f:
        regions = json.load(f)
    # 26 classes x {key, value} + other = the config-1 model's 53 outputs
    classes = [f"c{i}" for i in range(26)]
    os.makedirs(root, exist_ok=True)
    with open(os.path.join(root, "..", "classes26.json"), "w") as f:
        json.dump({"classes": classes}, f)
    rng = np.random.default_rng(seed)
    for d in range(copies):
        regs = []
        for r in regions:
            fk, kt = ((classes[int(rng.integers(len(classes)))], ["key", "value"][int(rng.integers(2))])
                      if rng.random() < 0.5 else (None, None))
            regs.append({"shape_attributes": {"name": "polygon", "all_points_x": [p[0] for p in r["location"]],
                                              "all_points_y": [p[1] for p in r["location"]]},
                         "region_attributes": {"label": r["text"], "formal_key": fk, "key_type": kt}})
        with open(os.path.join(root, f"page{d}.json"), "w", encoding="utf-8") as f:
            json.dump({"attributes": {"_via_img_metadata": {"regions": regs}}}, f)
    return root


def c1_procedure_steps(dev, iters):
    """SURVEY.md §8(b)'s caller, timed: the drop-in KVProcedure (what
    GNNLearningWarper.train() runs per batch, kv_procedure.py:143-164) on B=4
    batches of debug.json pages -- graph build from the collated dense A,
    forward, CE, backward, clip, Adam, metrics -- eager, and with
    capture_train_step (the step as one HIP graph per batch shape)."""
    import tempfile

    from gnn.models import GraphCNNDropEdge
    from gnn.trainer.training_procedures import KVProcedure
    from gnn.utils.config import AttrDict

    assets = os.path.join(HERE, "tests", "golden", "assets")
    out = {}
    with tempfile.TemporaryDirectory() as tmp:
        root = _debug_datapile(os.path.join(tmp, "pages"))
        split = {"data_path": [root], "class_path": os.path.join(tmp, "classes26.json"),
                 "charset_path": os.path.join(assets, "master_charset.json"), "key_types": ["key", "value"],
                 "batch_size": 4, "num_workers": 0, "shuffle": False, "drop_last": True, "pin_memory": False,
                 "augmentations": [],
                 "data_collate": {"NumpyPadding": {"name_value_pairs": {"textline_encoding": 0.0,
                                                                        "adjacency_matrix": 0.0, "node_label": -100.0},
                                                   "only_selected_items": True}},
                 "data_process": {"TextlineEncoding": {"is_normalized_text": True},
                                  "HeuristicGraphBuilder": {"num_edges": 6, "edge_type": "normal_binary"},
                                  "NodeLabeling": {}}}
        for mode in (None, True):
            cfg = AttrDict({
                "experiment_name": "bench", "seed": 1111, "is_train": True, "output_dir": os.path.join(tmp, "out"),
                "checkpoint_path": None, "num_gpus": 1, "distributed": False, "local_rank": 0, "num_epochs": 1,
                "max_grad_norm": 5.0, "model_dir_name": "models", "capture_train_step": mode,
                "data_config": {"dataset": {"type": "DatapileDataset",
                                            "args": {"node_label_padding_value": -100, "other_class_index": None}},
                                "training": split, "validation": dict(split, batch_size=1)},
                "loss": {"type": "CrossEntropyLoss", "args": {}},
                "lr_scheduler": {"type": "DecayLearningRate", "args": {"lr": 0.001, "factor": 0.9, "num_epochs": 100}},
                "optimizer": {"type": "BuitlinOptimizer", "args": {"type_optimizer": "Adam", "lr": 0.001}}})
            torch.manual_seed(0)
            proc = KVProcedure(GraphCNNDropEdge(4369, 53, 6, 256), cfg)
            batches = list(proc.train_loader)

            def one(i):
                proc._run_train_step(batches[i % len(batches)])
                if proc.step_graph is None:
                    proc.model.zero_grad()

            for i in range(4):  # warm: lazy workspaces; the second sighting of a shape captures it
                one(i)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(iters):
                one(i)
            torch.cuda.synchronize()
            key = "captured" if mode else "eager"
            out[f"{key}_ms"] = (time.perf_counter() - t0) / iters * 1e3
            if mode:
                out["capture_stats"] = proc.step_graph.stats()
            del proc
    out["note"] = ("KVProcedure._run_train_step on B=4 batches of debug.json pages (74 nodes), the drop-in's own "
                   "training loop: dense A -> typed graph, forward, CE, backward, clip, Adam, and the per-batch "
                   "metrics (argmax + sklearn report, host); captured = capture_train_step: true")
    return out


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


def run_only(args, graph, X_full, spmm, L, F):
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
    elif args.only == "infer":  # one-call GraphConv inference (the fused kernel by default)
        from grl.ops import graph_conv_infer

        W = torch.randn((L + 1) * F, F, device=X_full.device) / np.sqrt((L + 1) * F)
        b = torch.randn(F, device=X_full.device)
        Xe = X_full.detach()[: graph.num_cols]
        fn = lambda: graph_conv_infer(Xe, graph, W, b, True)  # noqa: E731
    elif args.only == "linear":
        Z = typed_aggregate(X_full, graph)
        W = torch.randn((L + 1) * F, F, device=X_full.device) / np.sqrt((L + 1) * F)
        fn = lambda: linear_fwd(Z, W, None, False)  # noqa: E731
    else:  # the model's layer (one autograd node, DropEdge 0.3, bias, ReLU), as the extras line times it
        from grl import DropEdge
        from grl.ops import graph_conv

        Xl = X_full.detach().clone().requires_grad_(True)
        W = (torch.randn((L + 1) * F, F, device=X_full.device) / np.sqrt((L + 1) * F)).requires_grad_(True)
        b = torch.zeros(F, device=X_full.device, requires_grad=True)
        gl = graph.with_dropedge(DropEdge(0.3, 2, 1, True))

        def fn():
            Xl.grad = W.grad = b.grad = None
            graph_conv(Xl, gl, W, b, relu=True).sum().backward()
    for _ in range(args.warmup):
        fn()
    torch.cuda.synchronize()
    for _ in range(args.steps):
        fn()
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
