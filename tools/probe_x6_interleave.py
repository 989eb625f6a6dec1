"""A/B of the x6 GEMM's interleaved A split (GRL_X6_INTERLEAVE=1) against the
default schedule on the C3 layer shapes, same process, alternating; checks
the outputs are bitwise equal."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "graph-representation-learning_amd"))
import torch  # noqa: E402

from grl.ops import linear_bwd_data, linear_fwd  # noqa: E402


def t(fn, n=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n


def main():
    M, K, C = 1_000_000, 1792, 256
    dev = torch.device("cuda:0")
    Z = torch.randn(M, K, device=dev)
    W = torch.randn(K, C, device=dev) / K ** 0.5
    b = torch.randn(C, device=dev)
    g = torch.randn(M, C, device=dev)
    fl = 2.0 * M * K * C / 1e12
    outs = {}
    for rep in range(3):
        for mode in ("0", "1"):
            os.environ["GRL_X6_INTERLEAVE"] = mode
            for name, fn in (("fwd", lambda: linear_fwd(Z, W, b, True)), ("dZ", lambda: linear_bwd_data(g, None, W))):
                ms = t(fn)
                if rep == 0:
                    outs[(mode, name)] = fn()
                print(f"interleave={mode} {name}: {ms:.3f} ms ({fl / (ms * 1e-3):.0f} TF)", flush=True)
    for name in ("fwd", "dZ"):
        print(f"{name} bitwise equal: {bool(torch.equal(outs[('0', name)], outs[('1', name)]))}", flush=True)


if __name__ == "__main__":
    main()
