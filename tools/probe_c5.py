"""Probe (C5: R-MAT scale 23, avg_deg 64, d=512, DropEdge p=0.2, one GPU):
what limits the 17 GB-table gather.  Times the forward under
  * GRL_SPMM_WIDE_U = 4 / 8   (whole 2 KB rows issued 4 or 8 at a time),
  * GRL_SPMM_WIDE   = 0       (two 256-column waves per row),
  * a source relabeling by descending in-degree (colidx' = rank[colidx],
    X' = X[perm]): hot rows packed together -- a locality probe only (the
    self term still reads row n of X', so Z is not checked),
interleaved, 3 rounds."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "graph-representation-learning_amd"))
import torch  # noqa: E402

from grl import DropEdge, TypedGraph  # noqa: E402
from grl.ops import spmm_forward  # noqa: E402


def timeit(fn, n=3):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n * 1e3


def main():
    dev = torch.device("cuda:0")
    N, deg, F = 1 << 23, 64.0, 512
    g = TypedGraph.synthetic(N, deg, 6, kind="rmat", seed=0, device=dev).with_dropedge(DropEdge(0.2, 2, 0))
    X = torch.randn(N, F, device=dev)
    Z = torch.empty(N, 7 * F, device=dev)
    indeg = torch.bincount(g.colidx.long(), minlength=N)
    perm = torch.argsort(indeg, descending=True)
    rank = torch.empty_like(perm)
    rank[perm] = torch.arange(N, device=dev)
    top = indeg[perm].cumsum(0).float() / indeg.sum()
    print(f"edges {g.nnz}; sources covering 50/90% of edges: {int((top < 0.5).sum())} / {int((top < 0.9).sum())} "
          f"rows ({int((top < 0.5).sum()) * F * 4 / 2**20:.0f} / {int((top < 0.9).sum()) * F * 4 / 2**20:.0f} MiB)",
          flush=True)
    gr = TypedGraph(g.rowptr, rank[g.colidx.long()].to(torch.int32), 6, num_cols=N).with_dropedge(DropEdge(0.2, 2, 0))
    Xr = X[perm].contiguous()
    variants = {
        "wide U=4": ({"GRL_SPMM_WIDE_U": "4"}, lambda: spmm_forward(X, g, out=Z)),
        "wide U=8": ({"GRL_SPMM_WIDE_U": "8"}, lambda: spmm_forward(X, g, out=Z)),
        "half rows": ({"GRL_SPMM_WIDE": "0"}, lambda: spmm_forward(X, g, out=Z)),
        "relabelled U=4": ({"GRL_SPMM_WIDE_U": "4"}, lambda: spmm_forward(Xr, gr, out=Z)),
        "relabelled U=8": ({"GRL_SPMM_WIDE_U": "8"}, lambda: spmm_forward(Xr, gr, out=Z)),
    }
    res = {k: [] for k in variants}
    for rnd in range(3):
        for name, (env, fn) in variants.items():
            saved = {k: os.environ.get(k) for k in ("GRL_SPMM_WIDE_U", "GRL_SPMM_WIDE")}
            os.environ.pop("GRL_SPMM_WIDE", None)
            os.environ.update(env)
            res[name].append(timeit(fn))
            for k, v in saved.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
        print(f"round {rnd}: " + ", ".join(f"{k} {v[-1]:.1f}" for k, v in res.items()), flush=True)
    print("min ms: " + ", ".join(f"{k} {min(v):.1f}" for k, v in res.items()), flush=True)


if __name__ == "__main__":
    main()
