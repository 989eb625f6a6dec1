"""Diagnostic: does gathering X in column slices (so one pass's slice of X
fits the 256 MiB Infinity Cache) beat one full-width pass on the C3 graph?
Times spmm_forward over X[:, c:c+w] (ldx = 256) for w in 256/128/64/32."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "graph-representation-learning_amd"))
import torch  # noqa: E402

from grl import TypedGraph  # noqa: E402
from grl.ops import spmm_forward  # noqa: E402


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


def main():
    N, F = int(os.environ.get("PROBE_N", "1000000")), 256
    dev = torch.device("cuda:0")
    g = TypedGraph.synthetic(N, 32.0, 6, seed=0, device=dev)
    X = torch.randn(N, F, device=dev)
    for w in (256, 128, 64, 32):
        outs = [torch.empty(N, 7 * w, device=dev) for _ in range(F // w)]
        Xc = [X[:, c * w:(c + 1) * w].contiguous() for c in range(F // w)]

        def strided():
            for c in range(F // w):
                spmm_forward(X[:, c * w:(c + 1) * w], g, out=outs[c])

        def packed():
            for c in range(F // w):
                spmm_forward(Xc[c], g, out=outs[c])

        print(f"w={w:3d} passes={F // w}  strided {timeit(strided):7.3f} ms   packed {timeit(packed):7.3f} ms",
              flush=True)
        del outs, Xc
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
