#!/usr/bin/env python
"""Per-rank evidence for the N > 1 bench line, on ONE GPU.

bench.py --gpus N (workload C4: ER, N = 4M, avg_deg 32 over L = 6 types,
d = 256, node-range shards) times each rank's step = the halo exchange
pipelined with grl_typed_spmm_fwd_slice over the rank's [own | halo] table
(grl.dist.HaloPipeline, 2 column slices of 128).  Its roofline.traffic came
out null because no PMC pass had measured those slice kernels over a real
shard's table.  This tool builds rank r's shard of the C4 graph for a world
of P in-process (ShardedGraph.in_process: the same plan and halo mode
from_graph / synthetic build on rank r; node ranges as ShardedGraph.synthetic
gives ER), fills its slice tables exactly as the exchange would (dense:
every rank's padded own rows; sparse: the referenced halo rows in owner
order), and runs ONLY that rank's aggregation -- the K slice launches that
bench's `spmm_only_ms` times -- with HIP events on the launch stream.  Z is
checked bitwise against the one-GPU whole-graph aggregation's rows.

Under rocprofv3 (--kernel-trace --stats, then one --pmc pass each for
FETCH_SIZE and WRITE_SIZE) the same command gives the slice kernels' time
and HBM bytes; tools/pmc_rank_traffic.py folds the passes into
profiles/pmc_traffic.json under bench.traffic_key("C4", P, ..., n_loc of
rank 0), so a C4 --gpus P line carries a measured roofline.traffic.

  python tools/probe_rank_shard.py --world 2 [--rank 0] [--iters 10] [--json out.json]
"""
import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path[:0] = [os.path.join(ROOT, "graph-representation-learning_amd"), ROOT]

import torch  # noqa: E402


class _NoExchange:
    """HaloPipeline's exchange slot: the tables are filled by this tool."""

    async_op = False

    def __init__(self, world):
        self.world = world


def spmm_bytes(E, N, L, F, p):
    from bench import spmm_bytes as sb

    return sb(E, N, L, F, p)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, required=True)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--nodes", type=int, default=4_000_000)
    ap.add_argument("--avg-deg", type=float, default=32.0)
    ap.add_argument("--types", type=int, default=6)
    ap.add_argument("--dim", type=int, default=256)
    ap.add_argument("--chunks", type=int, default=0)
    ap.add_argument("--halo", default="auto")
    ap.add_argument("--json", default=None)
    ap.add_argument("--no-parity", action="store_true",
                    help="skip the whole-graph check (a PMC pass then sees only the slice kernels' SpMM launches)")
    args = ap.parse_args()

    from grl import TypedGraph
    from grl.dist import HaloPipeline, ShardedGraph
    from grl.ops import spmm_forward, spmm_forward_slice

    dev = torch.device("cuda:0")
    P, r, N, L, F = args.world, args.rank, args.nodes, args.types, args.dim
    K = args.chunks or max(1, F // 128)  # bench.py's default slices
    t0 = time.time()
    g = TypedGraph.synthetic(N, args.avg_deg, L, kind="er", seed=0, device=dev)
    per = -(-N // P)
    bounds = [min(N, q * per) for q in range(P + 1)]  # ShardedGraph.synthetic's ER ranges ("nodes")
    shards = ShardedGraph.in_process(g, bounds, halo=args.halo)
    sg = shards[r]
    del shards
    X = torch.randn(N, F, generator=torch.Generator(device=dev).manual_seed(1), device=dev)
    plan = sg.plan
    rb, re = plan.row_begin, plan.row_end
    pipe = HaloPipeline(sg, F, chunks=K, device=dev, exchange=_NoExchange(P))
    # the tables as the exchange leaves them
    xs = pipe._slices(X)  # [K, N, Fc] view
    for c in range(K):
        t = pipe.tables[c]
        t[:plan.n_loc].copy_(xs[c, rb:re])
        if plan.mode == "dense":
            for q in range(P):
                b0, b1 = bounds[q], bounds[q + 1]
                t[plan.stride * (1 + q): plan.stride * (1 + q) + (b1 - b0)].copy_(xs[c, b0:b1])
        else:
            t[plan.n_loc:].copy_(xs[c].index_select(0, plan.halo_ids))
    gs = sg.graph
    Z = torch.empty(plan.n_loc, gs.segments * F, device=dev)
    stream = torch.cuda.current_stream(dev)

    def aggregate():
        for c in range(K):
            spmm_forward_slice(pipe.tables[c], gs, Z, c * pipe.Fc)

    aggregate()
    torch.cuda.synchronize()
    # parity: the shard's rows are bitwise the one-GPU whole-graph rows
    same = None
    if not args.no_parity:
        Zw = spmm_forward(X, g)
        same = bool(torch.equal(Z, Zw[rb:re]))
        del Zw
    torch.cuda.empty_cache()
    build_s = time.time() - t0
    for _ in range(2):
        aggregate()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.iters)]
    torch.cuda.synchronize()
    for a, b in evs:
        a.record(stream)
        aggregate()
        b.record(stream)
    torch.cuda.synchronize()
    ms = [a.elapsed_time(b) for a, b in evs]
    E_loc = gs.nnz
    alg = spmm_bytes(E_loc, plan.n_loc, L, F, 0.0)
    alg_sliced = alg + (K - 1) * (4 * E_loc + 4 * (plan.n_loc * L + 1))  # each slice re-walks colidx / rowptr
    mean = sum(ms) / len(ms)
    out = {
        "workload": "C4", "world": P, "rank": r, "nodes_total": N, "edges_total": g.nnz, "bounds": bounds,
        "n_loc": plan.n_loc, "edges_loc": E_loc, "halo_mode": plan.mode, "halo_rows_referenced":
        plan.referenced_halo_rows, "table_rows": plan.n_loc + plan.n_halo, "chunks": K,
        "aggregate_ms_mean": mean, "aggregate_ms_min_max": [min(ms), max(ms)],
        "alg_bytes_step": alg, "alg_bytes_step_incl_slice_rewalks": alg_sliced,
        "alg_GBps": alg / (mean * 1e-3) / 1e9, "bitwise_vs_one_gpu_rows": same, "build_s": build_s,
        "note": "rank r's K column-slice launches of grl_typed_spmm_fwd_slice over its [own | halo] table "
                "(bench.py halo_breakdown spmm_only_ms), alone on one GPU; tables filled as the exchange "
                "leaves them",
    }
    print(json.dumps(out), flush=True)
    if args.json:
        with open(args.json, "w") as f:
            json.dump(out, f, indent=1)
    if same is False:
        raise SystemExit("shard rows differ from the one-GPU aggregation")


if __name__ == "__main__":
    main()
