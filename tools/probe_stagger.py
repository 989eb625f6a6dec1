"""A/B (one box, interleaved): the x6 GEMM with and without the stagger of
the SIMD partner waves (GRL_X6_STAGGER, read per call) on C3's shapes --
forward (M=1M, K=1792, C=256, bias+ReLU), dZ (K=256 -> 1792) -- and the
one-call GraphConv inference.  Outputs must be bitwise equal."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "graph-representation-learning_amd"))
import torch  # noqa: E402

from grl import TypedGraph  # noqa: E402
from grl.ops import graph_conv_infer, linear_bwd_data, linear_fwd  # noqa: E402


def timeit(fn, n=10):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n * 1e3


def main():
    dev = torch.device("cuda:0")
    M, F, C = 1_000_000, 256, 256
    gen = torch.Generator(device=dev).manual_seed(0)
    Z = torch.randn(M, 7 * F, generator=gen, device=dev)
    W = torch.randn(7 * F, C, generator=gen, device=dev) / 40
    b = torch.randn(C, generator=gen, device=dev)
    g = torch.randn(M, C, generator=gen, device=dev)
    graph = TypedGraph.synthetic(M, 32.0, 6, seed=0, device=dev)
    X = torch.randn(M, F, generator=gen, device=dev)
    res = {}
    outs = {}
    for rnd in range(3):
        for st in ("0", "1"):
            os.environ["GRL_X6_STAGGER"] = st
            r = res.setdefault(st, {"fwd": [], "dZ": [], "infer": []})
            r["fwd"].append(timeit(lambda: linear_fwd(Z, W, b, True)))
            r["dZ"].append(timeit(lambda: linear_bwd_data(g, None, W)))
            r["infer"].append(timeit(lambda: graph_conv_infer(X, graph, W, b, True), 5))
            if rnd == 0:
                outs[st] = (linear_fwd(Z, W, b, True), linear_bwd_data(g, None, W))
        print(f"round {rnd}: " + "; ".join(f"stagger={k}: " + ", ".join(f"{n} {v[-1]:.3f}" for n, v in r.items())
                                         for k, r in res.items()), flush=True)
    same = all(torch.equal(a, c) for a, c in zip(outs["0"], outs["1"]))
    print("min ms: " + "; ".join(f"stagger={k}: " + ", ".join(f"{n} {min(v):.3f}" for n, v in r.items())
                                 for k, r in res.items()) + f"; bitwise equal {same}", flush=True)


if __name__ == "__main__":
    main()
