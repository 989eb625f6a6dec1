"""Diagnostic: fused NodeSelfAtten throughput at large N (B=1, dk=16, dv=128,
the config-1 model's attention shape) -- forward and forward+backward."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "graph-representation-learning_amd"))
import torch  # noqa: E402

from grl.ops import node_attention_forward, node_self_attention  # noqa: E402


def timeit(fn, n=5):
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
# arguments: N values, and NAME=VALUE path options (grl.set_option) for the whole run
_opts = [a for a in sys.argv[1:] if "=" in a]
if _opts:
    from grl import set_option

    for kv in _opts:
        set_option(kv.split("=")[0], int(kv.split("=")[1]))
for N in ([int(x) for x in sys.argv[1:] if "=" not in x] or (2048, 16384, 65536, 131072)):
    dk, dv = 16, 128
    torch.manual_seed(N)  # the same inputs in every library's run (AB_SAVE bit check)
    Q, K = torch.relu(torch.randn(1, N, dk, device=dev)), torch.relu(torch.randn(1, N, dk, device=dev))
    H, V, g = torch.relu(torch.randn(1, N, dv, device=dev)), torch.randn(1, N, dv, device=dev), torch.randn(dv, device=dev)
    flops = 2.0 * N * N * (dk + dv)
    ms = timeit(lambda: node_attention_forward(Q, K, H, V, g))
    leaves = [t.clone().requires_grad_(True) for t in (Q, K, H, V, g)]
    ms_fb = timeit(lambda: node_self_attention(*leaves).sum().backward(), 3)
    # backward = 2 S recomputes (2*N^2*dk each) + 2 dP (2*N^2*dv each) + dQ, dK (2*N^2*dk each) + dH (2*N^2*dv)
    bflops = 2.0 * N * N * (4 * dk + 3 * dv)
    same = None
    ref_path = os.environ.get("AB_SAVE")
    if ref_path:  # bits of out and every gradient against the first library's (A/B of builds)
        for t in leaves:
            t.grad = None
        out = node_self_attention(*leaves)
        out.backward(torch.ones_like(out))
        got = torch.cat([out.detach().flatten()] + [t.grad.flatten() for t in leaves]).cpu()
        path = f"{ref_path}.{N}"
        if os.path.exists(path):
            same = bool(torch.equal(torch.load(path, weights_only=True), got))
        else:
            torch.save(got, path)
    print(f"{' '.join(_opts)} N={N:7d} fwd {ms:9.3f} ms {flops / ms / 1e9:7.1f} TFLOP/s | fwd+bwd {ms_fb:9.3f} ms "
          f"{(flops + bflops) / ms_fb / 1e9:7.1f} TFLOP/s bitwise_vs_first={same}", flush=True)
