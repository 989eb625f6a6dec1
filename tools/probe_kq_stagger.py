"""A/B: the fused dK/dQ attention pass with waves 4-7 half a block late
(GRL_ATTN_KQ_STAGGER=1) vs in phase (default), in one process: gradients
compared bitwise, forward + backward timed interleaved (B=1, dk=16, dv=128)."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "graph-representation-learning_amd"))
import torch  # noqa: E402

from grl.ops import node_self_attention  # noqa: E402

dev = torch.device("cuda:0")
res = {}
for N in [int(x) for x in (sys.argv[1:] or ["3000", "33333", "100000", "131072"])]:
    gen = torch.Generator(device=dev).manual_seed(N)
    dk, dv = 16, 128
    Q = torch.relu(torch.randn(1, N, dk, device=dev, generator=gen)).requires_grad_(True)
    K = torch.relu(torch.randn(1, N, dk, device=dev, generator=gen)).requires_grad_(True)
    H = torch.relu(torch.randn(1, N, dv, device=dev, generator=gen)).requires_grad_(True)
    V = torch.randn(1, N, dv, device=dev, generator=gen).requires_grad_(True)
    g = torch.randn(dv, device=dev, generator=gen).requires_grad_(True)
    dout = torch.randn(1, N, dv, device=dev, generator=gen)

    def step():
        for t in (Q, K, H, V, g):
            t.grad = None
        node_self_attention(Q, K, H, V, g).backward(dout)
        return [t.grad.clone() for t in (Q, K, H, V, g)]

    grads, times = {}, {"0": [], "1": []}
    for rep in range(3):
        for mode in ("0", "1"):
            os.environ["GRL_ATTN_KQ_STAGGER"] = mode
            grads[mode] = step()
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            n = 3 if N >= 65536 else 10
            s.record()
            for _ in range(n):
                step()
            e.record()
            torch.cuda.synchronize()
            times[mode].append(s.elapsed_time(e) / n)
    same = all(torch.equal(a, b) for a, b in zip(grads["0"], grads["1"]))
    res[N] = {"fwd_bwd_ms_default": times["0"], "fwd_bwd_ms_stagger": times["1"], "grads_bitwise_equal": same}
    print(json.dumps({N: res[N]}), flush=True)
