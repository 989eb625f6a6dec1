"""Diagnostic: time the three GraphConv GEMMs (fwd, bwd-data, bwd-weight) at
the C3 layer shape (M=1M nodes, K=(L+1)*256=1792, C=256) for the libgrl
build named by GRL_LIB_PATH, and hipBLASLt (torch.matmul) for reference."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "graph-representation-learning_amd"))
import torch  # noqa: E402

from grl.ops import linear_bwd_data, linear_bwd_weight, linear_fwd  # noqa: E402


def t(fn, n=5):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n


M, K, C = 1_000_000, 1792, 256
dev = torch.device("cuda:0")
Z = torch.randn(M, K, device=dev)
W = torch.randn(K, C, device=dev) / K ** 0.5
b = torch.randn(C, device=dev)
g = torch.randn(M, C, device=dev)
out = torch.randn(M, C, device=dev)
fl = 2.0 * M * K * C / 1e12
tag = os.path.basename(os.environ.get("GRL_LIB_PATH", "libgrl.so"))
gm = torch.where(out > 0, g, 0.0)
for name, fn in [("fwd", lambda: linear_fwd(Z, W, b, True)), ("bwd_data", lambda: linear_bwd_data(g, out, W)),
                 ("bwd_weight", lambda: linear_bwd_weight(Z, g, out, True)),
                 ("bwd_data_pm", lambda: linear_bwd_data(gm, None, W)),
                 ("bwd_wgt_pm", lambda: linear_bwd_weight(Z, gm, None, True)),
                 ("premask", lambda: torch.where(out > 0, g, 0.0)),
                 ("torch_fwd", lambda: torch.addmm(b, Z, W)), ("torch_dZ", lambda: g @ W.t()),
                 ("torch_dW", lambda: Z.t() @ g)]:
    ms = t(fn)
    print(f"{tag:18s} {name:11s} {ms:7.3f} ms  {fl / (ms * 1e-3):6.1f} TFLOP/s", flush=True)
