"""Probe: the x6 weight-gradient GEMM at C3 (dW = Z^T g: M = 1M nodes, K =
1792, C = 256; grl_linear_bwd_weight), HIP events over back-to-back calls,
with the library GRL_LIB_PATH names; checks the result against the default
library's bits when AB_REF is set."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "graph-representation-learning_amd"))
import torch  # noqa: E402

from grl.ops import linear_bwd_weight  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    gen = torch.Generator(device=dev).manual_seed(3)
    M, K, C = 1_000_000, 1792, 256
    Z = torch.randn(M, K, device=dev, generator=gen)
    g = torch.randn(M, C, device=dev, generator=gen)
    dW, db = linear_bwd_weight(Z, g, None, True)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(10):
        linear_bwd_weight(Z, g, None, True)
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / 10
    lib = os.path.basename(os.environ.get("GRL_LIB_PATH", "libgrl.so"))
    out = os.environ.get("AB_SAVE")
    same = None
    if out:
        if os.path.exists(out):
            ref = torch.load(out, weights_only=True)
            same = bool(torch.equal(ref, dW.cpu()))
        else:
            torch.save(dW.cpu(), out)
    print(f"{lib}: dW {ms:.3f} ms ({2.0 * M * K * C / ms / 1e9:.1f} TF fp32-eq) bitwise_vs_first={same}", flush=True)


if __name__ == "__main__":
    main()
