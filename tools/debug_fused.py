"""Debug aid: read Z segment s back out of the fused GraphConv kernel with a
selector W (identity block at rows s*F..s*F+F-1: out = Z_s exactly, since
1.0 splits into (1, 0, 0)) and compare with the typed SpMM's Z, reporting
which segments / rows / columns differ."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "graph-representation-learning_amd"))
import torch  # noqa: E402

from grl import TypedGraph  # noqa: E402
from grl.ops import graph_conv_infer, typed_aggregate  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    N, L, F = int(os.environ.get("DBG_N", 20_011)), 6, 256
    g = TypedGraph.synthetic(N, 16.0, L, seed=0, device=dev)
    X = torch.randn(N, F, device=dev)
    Z = typed_aggregate(X, g)
    for s in range(L + 1):
        W = torch.zeros((L + 1) * F, F, device=dev)
        W[s * F:(s + 1) * F] = torch.eye(F, device=dev)
        out = graph_conv_infer(X, g, W, None, False)
        ref = Z[:, s * F:(s + 1) * F]
        d = (out - ref).abs()
        bad = (d.amax(1) > 0).nonzero().flatten()
        print(f"segment {s}: rows differing {bad.numel()} / {N}; first {bad[:8].tolist()}; "
              f"max|d| {d.max().item():.3e}", flush=True)
        if bad.numel():
            r = bad[0].item()
            print("   out", out[r, :6].tolist(), "\n   ref", ref[r, :6].tolist(), flush=True)
            cols = (d[r] > 0).nonzero().flatten()
            print(f"   row {r}: cols differing {cols.numel()} first {cols[:8].tolist()}", flush=True)


if __name__ == "__main__":
    main()
