"""A/B: emb1's weight gradient at the 100k-node model shape (M = 100k bag
rows of 4369, ~7 nonzeros + 4 dense box features, C = 256): the dense
grl_linear_bwd_weight GEMM vs the sparse grl_bag_linear_bwd_weight."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "graph-representation-learning_amd"))
from grl.ops import bag_linear_bwd_weight, linear_bwd_weight  # noqa: E402

dev = torch.device("cuda:0")
res = {}
for M in (296, 4096, 20_000, 100_000):
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

    dense = t(lambda: linear_bwd_weight(V, g, None, True))
    sparse = t(lambda: bag_linear_bwd_weight(V, g, None, True))
    a, b = linear_bwd_weight(V, g, None, True), bag_linear_bwd_weight(V, g, None, True)
    scale = float((V.double().abs().T @ g.double().abs()).max())
    res[f"M{M}"] = {"dense_gemm_ms": dense, "sparse_ms": sparse,
                    "max_abs_diff_dW": float((a[0] - b[0]).abs().max()), "sum_abs_terms_max": scale,
                    "max_abs_diff_db": float((a[1] - b[1]).abs().max())}
print(json.dumps(res), flush=True)
