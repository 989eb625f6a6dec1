"""Probe: GraphConv inference (SpMM -> x6 GEMM) with the two kernels on
disjoint CU sets (hipExtStreamCreateWithCUMask), pipelined over row chunks.

The HBM-bound gather and the MFMA-bound GEMM cannot share CUs (the x6 GEMM
holds 147 KB of LDS and 2 waves/SIMD of 203 VGPRs per CU, leaving the
gather one wave per SIMD), but on separate CUs they can run at
once: chunk i's GEMM on CU set B while chunk i+1 is gathered on set A.
Prints per-mask times of each kernel alone and of the pipeline, on C3.
"""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "graph-representation-learning_amd"))
import torch  # noqa: E402

from grl import TypedGraph  # noqa: E402
from grl.ops import graph_conv_infer, linear_fwd, spmm_forward, spmm_forward_slice  # noqa: E402

hip = ctypes.CDLL("libamdhip64.so")


def masked_stream(cus):
    """A HIP stream restricted to the CU ids in `cus`."""
    words = (ctypes.c_uint32 * 8)()
    for c in cus:
        words[c // 32] |= 1 << (c % 32)
    s = ctypes.c_void_p()
    rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(s), 8, words)
    assert rc == 0, rc
    return torch.cuda.ExternalStream(s.value)


def timeit(fn, n=5):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n * 1e3


def main():
    dev = torch.device("cuda:0")
    N, F, C = 1_000_000, 256, 256
    g = TypedGraph.synthetic(N, 32.0, 6, seed=0, device=dev)
    X = torch.randn(N, F, device=dev)
    W = torch.randn(7 * F, C, device=dev) / 40
    b = torch.randn(C, device=dev)
    Z = torch.empty(N, 7 * F, device=dev)
    out = torch.empty(N, C, device=dev)
    ref = graph_conv_infer(X, g, W, b, True)
    print(f"one call (grl_graphconv_fwd): {timeit(lambda: graph_conv_infer(X, g, W, b, True)):.2f} ms", flush=True)
    print(f"spmm alone {timeit(lambda: spmm_forward(X, g, out=Z)):.2f} ms, "
          f"gemm alone {timeit(lambda: linear_fwd(Z, W, b, True)):.2f} ms", flush=True)
    for split in os.environ.get("PROBE_SPLITS", "12,16,20").split(","):
        k = int(split)  # gather CUs per 32-CU group (XCD-sized)
        A = [c for c in range(256) if c % 32 < k]
        B = [c for c in range(256) if c % 32 >= k]
        sa, sb = masked_stream(A), masked_stream(B)
        with torch.cuda.stream(sa):
            ta = timeit(lambda: spmm_forward(X, g, out=Z))
        with torch.cuda.stream(sb):
            tb = timeit(lambda: linear_fwd(Z, W, b, True))
        for chunks in (4, 8, 16):
            rows = -(-N // chunks)
            sub = [(r, min(N, r + rows)) for r in range(0, N, rows)]
            views = [TypedGraph(g.rowptr[r0 * 6: r1 * 6 + 1], g.colidx, 6, num_cols=N, edge_id_base=g.edge_id_base,
                                self_id_base=g.self_id_base + r0, self_rows=r1 - r0) for r0, r1 in sub]

            def pipeline():
                main = torch.cuda.current_stream(dev)
                sa.wait_stream(main)
                sb.wait_stream(main)
                evs = []
                for (r0, r1), gv in zip(sub, views):
                    with torch.cuda.stream(sa):  # rows [r0, r1): rowptr view, absolute edge positions
                        spmm_forward_slice(X, gv, Z[r0:r1], 0, self_col0=r0)
                        e = torch.cuda.Event()
                        e.record(sa)
                        evs.append(e)
                for (r0, r1), e in zip(sub, evs):
                    with torch.cuda.stream(sb):
                        sb.wait_event(e)
                        out[r0:r1] = linear_fwd(Z[r0:r1], W, b, True)
                main.wait_stream(sa)
                main.wait_stream(sb)

            try:
                tp = timeit(pipeline)
                ok = torch.equal(out, ref)
            except Exception as err:  # probe: report and continue
                tp, ok = float("nan"), repr(err)[:120]
            print(f"gather CUs {len(A)} / gemm CUs {len(B)}: spmm {ta:.2f} ms, gemm {tb:.2f} ms, "
                  f"pipeline x{chunks} {tp:.2f} ms, bitwise {ok}", flush=True)


if __name__ == "__main__":
    main()
