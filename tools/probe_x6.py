"""Diagnostic: split-bf16 ("x6") vs fp32-MFMA GEMMs at the C3 layer shape.
Runs itself twice (path option gemm_x6 = 1 / 0, one child process each)
and prints time, TFLOP/s and the error vs fp64 on sampled rows, relative to
sum |terms| per element (the test suite's criterion)."""
import json
import os
import subprocess
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "graph-representation-learning_amd"))


def child():
    import torch
    from grl import set_option
    from grl.ops import linear_bwd_data, linear_fwd

    set_option("gemm_x6", int(sys.argv[2]))

    def t(fn, n=10):
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
    gen = torch.Generator(device=dev).manual_seed(0)
    Z = torch.randn(M, K, device=dev, generator=gen)
    W = torch.randn(K, C, device=dev, generator=gen) / K ** 0.5
    b = torch.randn(C, device=dev, generator=gen)
    g = torch.randn(M, C, device=dev, generator=gen)
    fl = 2.0 * M * K * C / 1e12
    res = {"x6": os.environ.get("GRL_GEMM_X6", "1")}
    rows = torch.randint(0, M, (4096,), device=dev, generator=gen)
    out = linear_fwd(Z, W, b, False)
    ref = Z[rows].double() @ W.double() + b.double()
    scale = Z[rows].double().abs() @ W.double().abs() + b.double().abs()
    res["fwd_err_rel_max"] = float(((out[rows].double() - ref).abs() / scale).max())
    res["fwd_err_rel_mean"] = float(((out[rows].double() - ref).abs() / scale).mean())
    dZ = linear_bwd_data(g, None, W)
    refz = g[rows].double() @ W.double().t()
    scz = g[rows].double().abs() @ W.double().abs().t()
    res["dZ_err_rel_max"] = float(((dZ[rows].double() - refz).abs() / scz).max())
    res["dZ_err_rel_mean"] = float(((dZ[rows].double() - refz).abs() / scz).mean())
    del out, dZ
    for name, fn in [("fwd", lambda: linear_fwd(Z, W, b, True)), ("dZ", lambda: linear_bwd_data(g, None, W))]:
        ms = t(fn)
        res[name + "_ms"] = ms
        res[name + "_tflops"] = fl / (ms * 1e-3)
    print("RESULT " + json.dumps(res), flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "child":
        child()
    else:
        for v in ("1", "0"):
            r = subprocess.run([sys.executable, __file__, "child", v], capture_output=True, text=True)
            line = [x for x in r.stdout.splitlines() if x.startswith("RESULT ")]
            print(line[0] if line else f"x6={v} failed rc={r.returncode}: {r.stderr[-2000:]}", flush=True)
            if r.returncode:
                sys.exit(r.returncode)
