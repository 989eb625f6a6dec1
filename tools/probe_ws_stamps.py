"""Diagnostic: wait-time breakdown of the warp-specialized fused GraphConv
kernel (diag build with -DGRL_WS_STAMP=1, via GRL_LIB_PATH): per role, the
fraction of each wave's lifetime spent waiting on the LDS ring."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "graph-representation-learning_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from grl import TypedGraph, _lib  # noqa: E402
from grl.ops import graph_conv_infer  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    N, F, C = 1_000_000, 256, 256
    g = TypedGraph.synthetic(N, 32.0, 6, seed=0, device=dev)
    X = torch.randn(N, F, device=dev)
    W = torch.randn(7 * F, C, device=dev) / 40
    for _ in range(3):
        graph_conv_infer(X, g, W, None, True)
    torch.cuda.synchronize()
    cu = torch.cuda.get_device_properties(dev).multi_processor_count
    buf = (ctypes.c_ulonglong * (1024 * 12 * 2))()
    fn = _lib.lib().grl_debug_ws_stats
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int64]
    assert fn(buf, 1024 * 12 * 2) == 0
    a = np.frombuffer(buf, dtype=np.uint64).reshape(1024, 12, 2)[:cu].astype(np.float64)
    for name, sl in (("gather", slice(0, 8)), ("mfma", slice(8, 12))):
        w, t = a[:, sl, 0], a[:, sl, 1]
        print(f"{name}: waiting {w.sum() / t.sum():.3f} of wave time (min {np.min(w / t):.3f}, max "
              f"{np.max(w / t):.3f}); wave lifetime {t.mean() / 1e6:.2f} M cycles", flush=True)


if __name__ == "__main__":
    main()
