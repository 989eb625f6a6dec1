"""Probe: does a physically contiguous feature table (hipExtMallocWithFlags
hipDeviceMallocContiguous: larger translation fragments) speed up the ER
gather whose cost on big tables is address translation (C4 shape: 3.2 %
UTCL1 misses)?  Times grl_typed_spmm_fwd with X in torch memory vs in a
contiguous allocation (same bytes), C3 and C4 shapes; Z must be equal."""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "graph-representation-learning_amd"))
import torch  # noqa: E402

from grl import TypedGraph, _lib  # noqa: E402
from grl.graph import current_stream_handle  # noqa: E402

hip = ctypes.CDLL("libamdhip64.so")


def timeit(fn, n=10):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n * 1e3


def main():
    dev = torch.device("cuda:0")
    F = 256
    for N in (1_000_000, 4_000_000):
        g = TypedGraph.synthetic(N, 32.0, 6, seed=0, device=dev)
        X = torch.randn(N, F, device=dev)
        Z = torch.empty(N, 7 * F, device=dev)
        Z2 = torch.empty_like(Z)
        nbytes = X.numel() * 4
        res = {}
        for flag, name in ((4, "contiguous"), (0, "hipExtMalloc default")):
            p = ctypes.c_void_p()
            rc = hip.hipExtMallocWithFlags(ctypes.byref(p), ctypes.c_size_t(nbytes), ctypes.c_uint(flag))
            if rc != 0:
                print(f"N={N} {name}: hipExtMallocWithFlags rc={rc}", flush=True)
                continue
            assert hip.hipMemcpy(p, ctypes.c_void_p(X.data_ptr()), ctypes.c_size_t(nbytes), 3) == 0
            csr = g.csr_c(F)

            def run_raw():
                _lib.call("grl_typed_spmm_fwd", ctypes.byref(csr), p.value, F, F, Z2.data_ptr(), None,
                          current_stream_handle(dev))

            def run_torch():
                _lib.call("grl_typed_spmm_fwd", ctypes.byref(csr), X.data_ptr(), F, F, Z.data_ptr(), None,
                          current_stream_handle(dev))

            for _ in range(2):
                res.setdefault("torch", []).append(timeit(run_torch))
                res.setdefault(name, []).append(timeit(run_raw))
            torch.cuda.synchronize()
            print(f"N={N} {name}: bitwise {torch.equal(Z, Z2)}", flush=True)
            hip.hipFree(p)
        print(f"N={N}: " + ", ".join(f"{k} {min(v):.3f} ms" for k, v in res.items()), flush=True)
        del g, X, Z, Z2
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
