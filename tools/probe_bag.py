"""Diagnostic: emb1 bag-of-characters linear (grl_bag_linear_fwd) time per
call at the C1 shapes (K=4369, C=256, ~7 nonzeros per row) and at a larger
batch; select the library with GRL_LIB_PATH."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "graph-representation-learning_amd"))
import torch  # noqa: E402

from grl import _lib  # noqa: E402
from grl.graph import current_stream_handle  # noqa: E402

dev = torch.device("cuda:0")


def t(fn, n=200):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3


g = torch.Generator(device=dev).manual_seed(0)
K, C = 4369, 256
Wt = torch.randn(K, C, device=dev, generator=g)
b = torch.randn(C, device=dev, generator=g)
tag = os.path.basename(os.environ.get("GRL_LIB_PATH", "libgrl.so"))
res = []
for M in (74, 296, 100_000):
    V = torch.zeros(M, K, device=dev)
    idx = torch.randint(0, K, (M, 7), device=dev, generator=g)
    V.scatter_(1, idx, torch.rand(M, 7, device=dev, generator=g) + 0.5)
    out = torch.empty(M, C, device=dev)
    st = current_stream_handle(dev)
    fn = lambda: _lib.call("grl_bag_linear_fwd", V.data_ptr(), K, M, K, Wt.data_ptr(), C, b.data_ptr(), 1,  # noqa
                           out.data_ptr(), st)
    res.append(f"M={M}: {t(fn, 200 if M < 1000 else 20):8.1f} us")
    ref = torch.relu(V @ Wt + b)
    res[-1] += f" (max|d| {float((out - ref).abs().max()):.1e})"
print(tag, " | ".join(res), flush=True)
