"""Diagnostic: C3 typed-SpMM forward (p=0, p=0.3) and backward (p=0) times for
A/B of libgrl builds (select the library with GRL_LIB_PATH)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "graph-representation-learning_amd"))
import torch  # noqa: E402

from grl import DropEdge, TypedGraph  # noqa: E402
from grl.ops import typed_aggregate  # noqa: E402


def timeit(fn, n=20):
    for _ in range(3):
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
N = int(os.environ.get("PROBE_N", "1000000"))
F = int(os.environ.get("PROBE_F", "256"))
g = TypedGraph.synthetic(N, 32.0, 6, seed=0, device=dev)
X = torch.randn(N, F, device=dev, generator=torch.Generator(device=dev).manual_seed(1))  # fixed: zbits compare builds
gd = g.with_dropedge(DropEdge(0.3, 2, 0, True))
Xg = X.clone().requires_grad_(True)
Z = typed_aggregate(Xg, g)
dZ = torch.randn_like(Z)
g.csc()
tag = os.path.basename(os.environ.get("GRL_LIB_PATH", "libgrl.so"))
r = {"fwd_p0": timeit(lambda: typed_aggregate(X, g)),
     "fwd_p0.3": timeit(lambda: typed_aggregate(X, gd)),
     "bwd_p0": timeit(lambda: torch.autograd.grad(Z, Xg, dZ, retain_graph=True))}
zc = int(typed_aggregate(X, g).view(torch.int32).to(torch.int64).sum())  # bit checksum: equal across builds iff same bits
print(tag, F, " ".join(f"{k}={v:.3f}ms" for k, v in r.items()), f"zbits={zc}", flush=True)
