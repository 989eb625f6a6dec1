"""Diagnostic: time the typed-SpMM forward under several conditions on the
C3 graph (used to investigate p=0 vs p>0 and allocation effects)."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "graph-representation-learning_amd"))
import torch  # noqa: E402

from grl import DropEdge, TypedGraph  # noqa: E402
from grl.ops import typed_aggregate  # noqa: E402


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
    N = int(os.environ.get("PROBE_N", "1000000"))
    dev = torch.device("cuda:0")
    g = TypedGraph.synthetic(N, 32.0, 6, seed=0, device=dev)
    X = torch.randn(N, 256, device=dev)
    variants = {
        "p0": g.with_dropedge(None),
        "p0.3": g.with_dropedge(DropEdge(0.3, 2, 0, True)),
        "p1e-9": g.with_dropedge(DropEdge(1e-9, 2, 0, True)),
    }
    keep = []
    for rep in range(2):
        for name, gv in variants.items():
            ms = timeit(lambda: typed_aggregate(X, gv))
            print(f"rep{rep} {name:6s} discard-out {ms:8.3f} ms", flush=True)
            def hold():
                keep.append(typed_aggregate(X, gv))
                if len(keep) > 1:
                    keep.pop(0)
            ms = timeit(hold)
            print(f"rep{rep} {name:6s} hold-out    {ms:8.3f} ms", flush=True)
            keep.clear()
    t0 = time.time()
    torch.cuda.synchronize()
    print("done", time.time() - t0)


if __name__ == "__main__":
    main()
