"""GPU probe: a GraphConv layer's three GEMMs at document-page sizes (C1: 4 pages x 74
nodes = 296 rows, K = 7 x 256, C = 256; and 1024 / 4096 rows) -- libgrl's fp32 GEMMs
(forward with chunk slabs, masked data gradient, weight gradient) against torch
(hipBLASLt) on the same operands.  Median of timed repetitions, one JSON line per size."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "graph-representation-learning_amd"))
from grl.ops import linear_bwd_data, linear_bwd_weight, linear_fwd  # noqa: E402

DEV = torch.device("cuda:0")


def timed(fn, iters=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(iters):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e) * 1e3)
    ts.sort()
    return round(ts[len(ts) // 2], 1)


def main():
    K, C = 7 * 256, 256
    for M in (296, 1024, 4096):
        g = torch.Generator(device=DEV).manual_seed(M)
        Z = torch.randn(M, K, generator=g, device=DEV)
        W = torch.randn(K, C, generator=g, device=DEV) / K ** 0.5
        b = torch.randn(C, generator=g, device=DEV)
        G = torch.randn(M, C, generator=g, device=DEV)
        out = torch.relu(Z @ W + b)
        res = {"M": M,
               "fwd_grl_us": timed(lambda: linear_fwd(Z, W, b, True)),
               "fwd_torch_us": timed(lambda: torch.relu(torch.addmm(b, Z, W))),
               "dZ_grl_us": timed(lambda: linear_bwd_data(G, out, W)),
               "dZ_torch_us": timed(lambda: torch.where(out > 0, G, 0.0) @ W.t()),
               "dW_grl_us": timed(lambda: linear_bwd_weight(Z, G, out, True)),
               "dW_torch_us": timed(lambda: (Z.t() @ torch.where(out > 0, G, 0.0), G.sum(0)))}
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
