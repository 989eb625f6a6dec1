"""Diagnostic: can the HBM-bound typed SpMM and the MFMA-bound GraphConv GEMM
run concurrently on two HIP streams (C3 shapes)?  Times each alone and both
together; run with grl.set_option("spmm_blocks_per_cu", 16 / 8 / 4) to vary the SpMM's
persistent-grid footprint."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "graph-representation-learning_amd"))
import torch  # noqa: E402

from grl import TypedGraph  # noqa: E402
from grl.ops import linear_fwd, spmm_forward  # noqa: E402


def timeit(fn, n=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n


dev = torch.device("cuda:0")
N, F = 1_000_000, 256
g = TypedGraph.synthetic(N, 32.0, 6, seed=0, device=dev)
X = torch.randn(N, F, device=dev)
Z = torch.empty(N, 7 * F, device=dev)
Zg = torch.randn(N, 7 * F, device=dev)
W = torch.randn(7 * F, F, device=dev) / 42
b = torch.randn(F, device=dev)
s2 = torch.cuda.Stream(dev)


def spmm():
    spmm_forward(X, g, out=Z)


def gemm():
    linear_fwd(Zg, W, b, True)


def both():
    s2.wait_stream(torch.cuda.current_stream(dev))
    spmm()
    with torch.cuda.stream(s2):
        gemm()
    torch.cuda.current_stream(dev).wait_stream(s2)


def both_gemm_first():
    s2.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s2):
        gemm()
    spmm()
    torch.cuda.current_stream(dev).wait_stream(s2)


a, c = timeit(spmm), timeit(gemm)
print(f"blocks/CU={os.environ.get('GRL_SPMM_BLOCKS_PER_CU', '16')}: spmm {a:.3f} ms, gemm {c:.3f} ms, "
      f"sum {a + c:.3f}, concurrent {timeit(both):.3f} ms, gemm launched first {timeit(both_gemm_first):.3f} ms",
      flush=True)
