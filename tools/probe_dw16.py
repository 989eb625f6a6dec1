"""A/B probe: the x6 weight-gradient GEMM dW = Z^T g at C3 (M = 1M nodes,
K = 1792, C = 256; grl_linear_bwd_weight) on the 16x16x32 kernel
(gemm_x6t16_kernel, GRL_X6T16=1; =2 with the next stage's split interleaved
between the MFMA groups) and the 32x32x16 one (GRL_X6T16=0),
interleaved rounds of 10 back-to-back calls (HIP events), and both results
against float64 on the first 256 rows of dW (error / sum |Z||g|).  Also the
gcn3 shape (K = 3584).  Prints one line per measurement and a JSON summary."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "graph-representation-learning_amd"))
import torch  # noqa: E402

from grl.ops import linear_bwd_weight  # noqa: E402


def timed(fn, n=10):
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
    dev = torch.device("cuda:0")
    out = {}
    for M, K, C in ((1_000_000, 1792, 256), (1_000_000, 3584, 256), (200_000, 1792, 256)):
        gen = torch.Generator(device=dev).manual_seed(3)
        Z = torch.randn(M, K, device=dev, generator=gen)
        g = torch.randn(M, C, device=dev, generator=gen)
        ref = Z[:, :256].double().t() @ g.double()
        bound = Z[:, :256].abs().double().t() @ g.abs().double()
        res = {}
        for rnd in range(3):
            for v in ("2", "1", "0"):
                os.environ["GRL_X6T16"] = v
                ms = timed(lambda: linear_bwd_weight(Z, g, None, True))
                res.setdefault(v, []).append(ms)
                print(f"M={M} K={K} GRL_X6T16={v} round {rnd}: {ms:.3f} ms", flush=True)
        errs = {}
        for v in ("2", "1", "0"):
            os.environ["GRL_X6T16"] = v
            dW, db = linear_bwd_weight(Z, g, None, True)
            errs[v] = float(((dW[:256].double() - ref).abs() / bound).max())
        os.environ.pop("GRL_X6T16")
        out[f"M{M}_K{K}_C{C}"] = {"x6t16_il_ms": sorted(res["2"]), "x6t16_ms": sorted(res["1"]),
                                  "x6t_ms": sorted(res["0"]), "x6t16_il_err_rel_bound": errs["2"],
                                  "x6t16_err_rel_bound": errs["1"], "x6t_err_rel_bound": errs["0"]}
        print(json.dumps(out[f"M{M}_K{K}_C{C}"]), flush=True)
        del Z, g, ref, bound
        torch.cuda.empty_cache()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
