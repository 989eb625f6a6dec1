"""Child process of tests/test_gpu_rccl.py: the drop-in GraphCNNDropEdge over
a node-range shard with EVERY collective of grl.dist on REAL RCCL
(torch.distributed "nccl"), on a one-GPU box.

RCCL refuses two ranks on one device, so the group has one rank and the
shard's plan is a loopback (tests/rccl_loopback.py): every source row a
GraphConv reads comes through the exchange.  One training step (feature
dropout 0.5, DropEdge 0.3, forward, backward, allreduce_gradients) and the
inference forward (streamed by row blocks and plain) then run the device
branches the multi-GPU node runs:
  * the halo exchange under autograd (all_gather_into_tensor / all_to_all_single),
  * the row-pipelined one-kernel backward's point-to-point blocks and the
    device MIN all-reduce that agrees on that path (_all_agree),
  * the DropEdge / feature-dropout seed broadcast (broadcast_seed),
  * sharded attention's gather_rows (all-gather) and reduce_rows (all-to-all),
  * streamed inference's async all_gather into slot views (dense) and
    all_to_all_single + _Landing (sparse),
  * the bucketed gradient all-reduce.
The same steps run again with the group replaced by a one-rank
grl.dist.LocalGroup (the in-process rank emulator the multi-rank GPU tests
drive): every output must be BITWISE the RCCL run's -- which pins the
emulator's semantics to RCCL's on the calls it stands in for -- and the
forward bitwise the one-GPU model's (gradients within 1e-4).  Prints one
JSON line; exit 0 iff every check passed.  Test infrastructure only."""
import copy
import json
import os
import socket
import sys

import torch
import torch.distributed as dist

REPO = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(REPO, "graph-representation-learning_amd"))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from grl import TypedGraph  # noqa: E402
from grl import dist as gdist  # noqa: E402
from grl.dist import LocalGroup, ShardedGraph, allreduce_gradients  # noqa: E402
from rccl_loopback import loopback_plan  # noqa: E402

DEV = torch.device("cuda", 0)
L, FIN, OUT = 6, 96, 7


def shard(g: TypedGraph, mode: str, group) -> ShardedGraph:
    sg = ShardedGraph.__new__(ShardedGraph)
    sg._init(g.rowptr, loopback_plan(g.colidx, g.num_rows, mode), g.num_types, g.vals, group)
    return sg


def model(net_size):
    from gnn.models import GraphCNNDropEdge

    torch.manual_seed(0)
    return GraphCNNDropEdge(FIN, OUT, L, net_size=net_size, dropedge_seed=3).to(DEV)


def run(m, V, A, y, group):
    seen = {}

    def record(name, orig):
        def fn(*a, **k):
            out = orig(*a, **k)
            seen.setdefault(name, out.detach().reshape(-1, out.shape[-1]).clone())
            return out
        return fn

    for name in ("gcn1", "gcn2", "gcn3"):
        mod = getattr(m, name)
        mod.propagate = record(name, mod.propagate)
    m.train()
    m.zero_grad(set_to_none=True)
    m.edge_dropout.reset_calls()
    m.dropout.reset_calls()
    logits = m.forward([V, A]).reshape(-1, OUT)
    torch.nn.functional.cross_entropy(logits, y, reduction="sum").backward()
    if group is not None:
        allreduce_gradients([p for p in m.parameters() if p.requires_grad], group=group,
                            bucket_bytes=1 << 16)  # several buckets
    res = {"logits": logits.detach(), **{k: v for k, v in seen.items()},
           **{"grad " + k: p.grad.detach().clone() for k, p in m.named_parameters() if p.grad is not None}}
    # device-drawn DropEdge / feature-dropout seeds (the production default): rank 0's draw is broadcast
    # (ShardedGraph.broadcast_seed); the generator reseeded so both runs draw the same seeds
    m.edge_dropout.seed = m.dropout.seed = None
    torch.manual_seed(11)
    with torch.no_grad():
        res["logits_device_seeds"] = m.forward([V, A]).reshape(-1, OUT)
    m.eval()
    with torch.no_grad():
        if isinstance(A, ShardedGraph):
            for tag, on, nb in (("plain", False, 2), ("streamed2", True, 2), ("streamed3", True, 3)):
                A.stream_rows, A.stream_blocks = on, nb
                res["eval_" + tag] = m.forward([V, A]).reshape(-1, OUT)
        else:
            res["eval_plain"] = m.forward([V, A]).reshape(-1, OUT)
    torch.cuda.synchronize()
    return res


def main():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    torch.cuda.set_device(DEV)
    dist.init_process_group("nccl", device_id=DEV)
    results = {"backend": dist.get_backend(), "checks": {}, "calls": {}}
    ok = True

    def check(name, cond, detail=None):
        nonlocal ok
        results["checks"][name] = bool(cond) if detail is None else {"ok": bool(cond), **detail}
        ok = ok and bool(cond)

    # count the dispatch layer's calls per kind on the RCCL runs (every branch must have run)
    counts = {}
    for fn in ("_c_all_gather", "_c_all_gather_into_tensor", "_c_all_to_all_single", "_c_all_reduce",
               "_c_broadcast", "_c_p2p"):
        orig = getattr(gdist, fn)

        def wrap(*a, _orig=orig, _fn=fn, **k):
            grp = a[-1] if a and not isinstance(a[-1], (bool, int)) else k.get("group")
            if not isinstance(grp, gdist.LocalRank):
                counts[_fn] = counts.get(_fn, 0) + 1
            return _orig(*a, **k)
        setattr(gdist, fn, wrap)

    for N, net in ((5000, 64), (20000, 256)):  # two-kernel layers / one-kernel layers + p2p row blocks
        g = TypedGraph.synthetic(N, 12.0, L, kind="er", seed=4, device=DEV)
        gen = torch.Generator().manual_seed(5)
        V = (torch.rand(N, FIN, generator=gen) < 0.1).float().to(DEV)
        y = torch.randint(0, OUT, (N,), generator=gen).to(DEV)
        one = run(model(net), V[None], g, y, None)
        for mode in ("dense", "sparse"):
            rccl = run(model(net), V, shard(g, mode, dist.group.WORLD), y, dist.group.WORLD)
            lg = LocalGroup(1).member(0)
            loc = run(model(net), V, shard(g, mode, lg), y, lg)
            tag = f"N{N}_{mode}"
            diff = [k for k in rccl if not torch.equal(rccl[k], loc[k])]
            check(f"{tag}_localgroup_bitwise_rccl", not diff, {"differ": diff[:8]})
            for k in ("logits", "gcn1", "gcn2", "gcn3", "eval_plain", "logits_device_seeds"):
                check(f"{tag}_{k}_bitwise_one_gpu", torch.equal(rccl[k], one[k]))
            for k in ("eval_streamed2", "eval_streamed3"):
                check(f"{tag}_{k}_bitwise_one_gpu", torch.equal(rccl[k], one["eval_plain"]))
            worst = 0.0
            for k in one:
                if k.startswith("grad "):
                    err = float((rccl[k] - one[k]).abs().max()) / max(1.0, float(one[k].abs().max()))
                    worst = max(worst, err)
            check(f"{tag}_grads_vs_one_gpu", worst <= 1e-4, {"worst_rel": worst})
    results["calls"] = counts
    for fn in ("_c_all_gather", "_c_all_gather_into_tensor", "_c_all_to_all_single", "_c_all_reduce",
               "_c_broadcast", "_c_p2p"):
        check(f"rccl_ran_{fn}", counts.get(fn, 0) > 0)
    dist.destroy_process_group()
    results["ok"] = ok
    print(json.dumps(results), flush=True)
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
