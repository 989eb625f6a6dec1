"""A/B: row-split count of the sparse emb1 weight gradient (grl_bag_linear_bwd_weight)
at the 100k-node model shape (M = 100k bag rows of 4369, ~7 nonzeros + 4 dense
box features, C = 256), GRL_BAG_DW_SPLITS = S per run; bag_dw_kernel and the
ordered reduce timed together with HIP events."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "graph-representation-learning_amd"))
from grl.ops import bag_linear_bwd_weight  # noqa: E402

dev = torch.device("cuda:0")
M = int(os.environ.get("PROBE_M", 100_000))
gen = torch.Generator(device=dev).manual_seed(1)
V = torch.zeros(M, 4369, device=dev)
V.scatter_(1, torch.randint(0, 4365, (M, 7), generator=gen, device=dev), 1.0)
V[:, -4:] = torch.rand(M, 4, generator=gen, device=dev)
g = torch.randn(M, 256, generator=gen, device=dev)


def t(fn, n=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n


res = {}
ref = None
for S in os.environ.get("PROBE_SPLITS", "0,8,16,28,48,64,96,128,196").split(","):
    if S == "0":
        os.environ.pop("GRL_BAG_DW_SPLITS", None)
    else:
        os.environ["GRL_BAG_DW_SPLITS"] = S
    out = bag_linear_bwd_weight(V, g, None, True)
    if ref is None:
        ref = out
    res[S or "default"] = {"ms": t(lambda: bag_linear_bwd_weight(V, g, None, True)),
                           "max_abs_diff_vs_default": float((out[0] - ref[0]).abs().max())}
print(json.dumps({"M": M, "splits": res}), flush=True)
