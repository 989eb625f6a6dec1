"""Diagnostic: the small-M GEMMs of the C1 workload (a B=4 batch of 74-node
pages: M = 296 rows; gcn1/gcn2 K = 7 x 256, gcn3 K = 7 x 512; N = 256),
forward / data gradient / weight gradient, at the split count given by
GRL_GEMM_SMALL_SPLITS (or the default)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "graph-representation-learning_amd"))
import torch  # noqa: E402

from grl.ops import linear_bwd_data, linear_bwd_weight, linear_fwd  # noqa: E402


def timeit(fn, n=200):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3


dev = torch.device("cuda:0")
torch.manual_seed(0)
out = []
for M, K, N in ((296, 1792, 256), (296, 3584, 256), (74, 1792, 256)):
    Z = torch.randn(M, K, device=dev)
    W = torch.randn(K, N, device=dev) / K ** 0.5
    b = torch.zeros(N, device=dev)
    g = torch.randn(M, N, device=dev)
    ref = (linear_fwd(Z, W, b, True), linear_bwd_data(g, None, W), linear_bwd_weight(Z, g, None, True)[0])
    t = (timeit(lambda: linear_fwd(Z, W, b, True)), timeit(lambda: linear_bwd_data(g, None, W)),
         timeit(lambda: linear_bwd_weight(Z, g, None, True)))
    out.append(f"M={M} K={K} N={N}: fwd {t[0]:6.1f} us  dZ {t[1]:6.1f} us  dW {t[2]:6.1f} us")
print(os.environ.get("GRL_GEMM_SMALL_SPLITS", "default"), " | ".join(out), flush=True)
