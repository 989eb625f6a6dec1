"""GPU probe: the model's row-local linears on the libgrl GEMM (grl.ops.row_linear,
M-invariant rows) against torch's nn.Linear (hipBLASLt) at the shapes of
GraphCNNDropEdge(net_size=256): emb2 512->128, f / g 128->16, h 128->128 (and the
three as the one 128->160 GEMM the model runs),
RanPAC 128->1280 (no bias, frozen), classifier 1280->53; rows of a C1 batch
(4 x 74), the 100k-node model and a 1M-node graph.  Forward and
forward+backward, median of timed repetitions.  Prints one JSON line."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "graph-representation-learning_amd"))
from grl.ops import row_linear  # noqa: E402

DEV = torch.device("cuda:0")
SHAPES = {"emb2": (512, 128, True, True), "f": (128, 16, True, True), "h": (128, 128, True, True),
          "fgh_merged": (128, 160, True, True),
          "w_rand": (128, 1280, False, True), "classifier": (1280, 53, True, False)}


def timed(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(iters):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e))
    ts.sort()
    return ts[len(ts) // 2]


def main():
    out = {}
    for M in [int(x) for x in os.environ.get("PROBE_ROWS", "296,100000,1000000").split(",")]:
        for name, (K, C, bias, relu) in SHAPES.items():
            lin = torch.nn.Linear(K, C, bias=bias).to(DEV)
            X = torch.randn(M, K, device=DEV, requires_grad=True)
            G = torch.randn(M, C, device=DEV)

            def t_fwd():
                with torch.no_grad():
                    y = lin(X)
                    return torch.relu(y) if relu else y

            def t_fb():
                y = lin(X)
                y = torch.relu(y) if relu else y
                y.backward(G)

            def g_fwd():
                with torch.no_grad():
                    return row_linear(X, lin.weight, lin.bias, relu=relu)

            def g_fb():
                row_linear(X, lin.weight, lin.bias, relu=relu).backward(G)

            out[f"M{M}_{name}"] = {"torch_fwd_ms": timed(t_fwd), "grl_fwd_ms": timed(g_fwd),
                                   "torch_fwd_bwd_ms": timed(t_fb), "grl_fwd_bwd_ms": timed(g_fb)}
            print(f"M{M}_{name}", out[f"M{M}_{name}"], flush=True)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
