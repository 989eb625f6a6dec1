"""Diagnostic: accuracy of the attention backward at the small-model widths
(dk = 4, dv = 32: the fp32-MFMA backward kernels) vs float64, unranged and
over query ranges, for N around the sizes where key / query splits change."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "graph-representation-learning_amd"))
import torch  # noqa: E402

from grl.ops import node_attention_backward, node_attention_forward, node_self_attention  # noqa: E402

dev = torch.device("cuda:0")
for dk, dv in ((4, 32), (16, 128)):
    for N in (3000, 6000, 7500, 8192, 12000):
        g = torch.Generator().manual_seed(N)
        Q = torch.relu(torch.randn(1, N, dk, generator=g)).to(dev)
        K = torch.relu(torch.randn(1, N, dk, generator=g)).to(dev)
        H = torch.relu(torch.randn(1, N, dv, generator=g)).to(dev)
        V = torch.randn(1, N, dv, generator=g).to(dev)
        gm = torch.randn(dv, generator=g).to(dev)
        dout = torch.randn(1, N, dv, generator=g).to(dev)
        leaves = [t.clone().requires_grad_(True) for t in (Q, K, H, V, gm)]
        node_self_attention(*leaves).backward(dout)
        ref = [t.double().clone().requires_grad_(True) for t in (Q, K, H, V, gm)]
        s = torch.softmax(ref[0] @ ref[1].transpose(1, 2), -1)
        (ref[4] * (s @ ref[2]) + ref[3]).backward(dout.double())
        errs = []
        for name, a, r in zip("QKH", leaves, ref):
            sc = float(r.grad.abs().max())
            errs.append(f"d{name} {float((a.grad.double() - r.grad).abs().max()) / sc:.2e}")
        # ranged: 3 equal ranges
        out, on, rm, rs = None, None, None, None
        dQs = torch.zeros_like(Q)
        dKs, dHs = torch.zeros_like(K), torch.zeros_like(H)
        cuts = [0, N // 3, 2 * N // 3, N]
        for q0, q1 in zip(cuts[:-1], cuts[1:]):
            o, on, rm, rs = node_attention_forward(Q, K, H, V, gm, stats=True, q_range=(q0, q1))
            dQ, dK, dH = node_attention_backward(Q, K, H, gm, on, rm, rs, dout, q_range=(q0, q1))
            dQs += dQ
            dKs += dK
            dHs += dH
        for name, a, r in zip("QKH", (dQs, dKs, dHs), ref):
            sc = float(r.grad.abs().max())
            errs.append(f"ranged d{name} {float((a.double() - r.grad).abs().max()) / sc:.2e}")
        print(f"dk {dk} dv {dv} N {N}: " + ", ".join(errs), flush=True)
