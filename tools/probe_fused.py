"""Probe: one-kernel GraphConv inference (graphconv.hip) vs the two-kernel
path (typed SpMM, then the x6 GEMM) on C3 (N=1M, avg_deg 32, L=6, d=256,
C=256), p=0 and DropEdge p=0.3; checks the two agree bitwise.  Times with
HIP events over back-to-back calls (same stream)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "graph-representation-learning_amd"))
import torch  # noqa: E402

from grl import DropEdge, TypedGraph, set_option  # noqa: E402
from grl.ops import graph_conv_infer  # noqa: E402


def timeit(fn, n=10, warm=2):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n


def main():
    dev = torch.device("cuda:0")
    N = int(os.environ.get("PROBE_N", 1_000_000))
    F, C = 256, 256
    g0 = TypedGraph.synthetic(N, 32.0, 6, seed=0, device=dev)
    gen = torch.Generator(device=dev).manual_seed(1)
    X = torch.randn(N, F, device=dev, generator=gen)
    W = torch.randn(7 * F, C, device=dev, generator=gen) / 40
    b = torch.randn(C, device=dev, generator=gen)
    lib = os.path.basename(os.environ.get("GRL_LIB_PATH", "libgrl.so"))
    for p in (0.0, 0.3):
        g = g0 if p == 0 else g0.with_dropedge(DropEdge(p, 2, 1, True))
        set_option("graphconv_fused", 1)
        fused = graph_conv_infer(X, g, W, b, True)
        t_f = timeit(lambda: graph_conv_infer(X, g, W, b, True))
        if os.environ.get("PROBE_ONLY_FUSED"):  # profiler runs: the fused kernel only
            print(f"{lib} p={p}: fused {t_f:.3f} ms", flush=True)
            if os.environ.get("PROBE_SIMPLE"):  # the phase-alternating kernel (fg_ws = 0) beside it
                set_option("fg_ws", 0)
                simple = graph_conv_infer(X, g, W, b, True)
                t_s = timeit(lambda: graph_conv_infer(X, g, W, b, True))
                set_option("fg_ws", 1)
                print(f"{lib} p={p}: simple {t_s:.3f} ms, bitwise equal to ws: {bool(torch.equal(simple, fused))}",
                      flush=True)
            continue
        set_option("graphconv_fused", 0)
        two = graph_conv_infer(X, g, W, b, True)
        t_2 = timeit(lambda: graph_conv_infer(X, g, W, b, True))
        set_option("graphconv_fused", 1)
        t_f2 = timeit(lambda: graph_conv_infer(X, g, W, b, True))
        same = bool(torch.equal(fused, two))
        print(f"{lib} p={p}: fused {t_f:.3f} / {t_f2:.3f} ms, two-kernel {t_2:.3f} ms, bitwise equal: {same}", flush=True)
        if not same:
            d = (fused - two).abs()
            print(f"   max|d| {d.max().item():.3e}, rows differing {(d.amax(1) > 0).sum().item()}", flush=True)


if __name__ == "__main__":
    main()
