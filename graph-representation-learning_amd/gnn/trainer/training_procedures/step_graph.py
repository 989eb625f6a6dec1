"""The training step of KVProcedure as one HIP graph (kv_procedure.py:143-164
in the reference: forward, loss, backward, clip, optimizer step).

The reference's document workload is many small pages (74 nodes in
debug.json): an eager step launches ~130 small kernels and is host-bound
(DESIGN.md §4.8).  Captured, the whole step replays with one launch.

What stays outside the graph, every step (host work, or shapes that change):
  * a dense adjacency batch (the collate's (B, N, L, N), B*N*L*N <=
    DENSE_IN_GRAPH_MAX entries): only its copy into the bucket's static A --
    the typed CSR and its CSC are built INSIDE the graph into static buffers
    at the capacity cap = B*N*L*N (grl_dense_to_csr_rowptr / _fill, entries
    past nnz given a sentinel column = B*N that the CSC sort puts last,
    grl_csr_to_csc over cap entries and B*N + 1 columns), so no host sync
    on nnz and no host graph objects per step;
  * otherwise the batch's TypedGraph (dense -> typed CSR, its CSC, or the
    typed edge list) -- then copied into the bucket's STATIC buffers: rowptr
    [B*N*L+1], colidx / CSC arrays at a capacity `cap` (a power of two >=
    nnz).
  Kernels walk rowptr / colptr, so entries past nnz are never read; the
  static graph's self-loop DropEdge ids start at SELF_ID_BASE = 2^31 (any
  fixed id scheme gives i.i.d. masks; eager steps of this procedure use the
  same static graph, so they draw the same masks);
  * V and the labels, copied into static tensors;
  * the DropEdge seed of the step, written into a device word every
    EdgeDropout reads at launch (`seed_source`), call ids 0, 1, 2 per step;
  * metrics (argmax, sklearn report, loss.item()) from the static outputs.

Inside: model.forward([V, graph]), the criterion, backward, the DP gradient
all-reduce (RCCL only: gloo stages through the host), clip_grad_norm_ and
the optimizer step (Adam with capturable=True and a device LR the epoch
schedule fills).  One graph per bucket (B, N, F_in, cap, values), captured
the second time a bucket is seen (the first, eager, step initialises the
optimizer state and every lazy workspace), kept in an LRU of MAX_BUCKETS.

mode "capture" replays; mode "static" runs the same static pipeline eagerly
(the parity reference for replays: same graphs, same seeds, same kernels).
"""
from __future__ import annotations

import ctypes
from collections import OrderedDict
from typing import Any, Dict, Optional, Tuple

import torch
import torch.nn as nn

from grl import TypedGraph
from grl._lib import call
from grl._lib import lib as _grl
from grl.graph import current_stream_handle

MAX_BUCKETS = 32
# DropEdge id of row 0's self loop in every static graph: past any edge id (edge ids are CSR positions < 2^31),
# and the same for a batch whatever its edge capacity, so the dense and the typed-edge form of one batch draw the
# same masks
SELF_ID_BASE = 1 << 31
MAX_ROWS = 1 << 14  # larger batches are not launch-bound: they run the normal eager step
DENSE_IN_GRAPH_MAX = 1 << 22  # B*N*L*N entries: dense batches up to this build their graph inside the replay


def _mix64(x: int) -> int:
    x &= (1 << 64) - 1
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & ((1 << 64) - 1)
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & ((1 << 64) - 1)
    return x ^ (x >> 31)


class _Bucket:
    """Static device buffers of one (B, N, F, cap, vals) bucket and its graph."""

    def __init__(self, B: int, N: int, F: int, L: int, cap: int, vals: bool, device, dense: bool = False):
        rows = B * N
        self.cap = cap
        self.V = torch.zeros(B, N, F, device=device)
        self.y = torch.zeros(B, N, dtype=torch.int64, device=device)
        self.rowptr = torch.zeros(rows * L + 1, dtype=torch.int32, device=device)
        self.colidx = torch.zeros(cap, dtype=torch.int32, device=device)
        self.vals = torch.zeros(cap, device=device) if vals else None
        # dense: one more column, the sentinel B*N of the padding entries (sorted last)
        self.csc = {"colptr": torch.zeros(rows + (2 if dense else 1), dtype=torch.int32, device=device),
                    "zrow": torch.zeros(cap, dtype=torch.int32, device=device),
                    "eid": torch.zeros(cap, dtype=torch.int32, device=device),
                    "cvals": torch.zeros(cap, device=device) if vals else None}
        self.graph = TypedGraph(self.rowptr, self.colidx, L, vals=self.vals, num_cols=rows, batch_shape=(B, N),
                                self_id_base=SELF_ID_BASE)
        # no heavy rows in a bucket (checked on load); the CSC lives in the static buffers.  The arrays are
        # refilled every step and nnz here is the capacity, so no typed transpose may be cached on this graph:
        # static_buffers keeps graph_conv's backward off the one-kernel data gradient (grl.ops)
        self.graph._shared.update({"csc": self.csc, "split_csr": None, "split_csc": None, "static_buffers": True})
        self.hip_graph: Optional[torch.cuda.CUDAGraph] = None
        self.out: Optional[Tuple[torch.Tensor, torch.Tensor]] = None  # static (loss, logits)
        self.failed = False
        self.A = None
        if dense:  # the graph is built from A inside the step (build_graph)
            self.A = torch.zeros(B, N, L, N, device=device)
            self.ws_rowptr = torch.empty(max(1, int(_grl().grl_dense_to_csr_workspace_size(rows * L))),
                                         dtype=torch.uint8, device=device)
            self.ws_csc = torch.empty(int(_grl().grl_csr_to_csc_workspace_size(cap, rows + 1)), dtype=torch.uint8,
                                      device=device)
            self.slot = torch.arange(cap, dtype=torch.int32, device=device)

    def load_dense(self, V: torch.Tensor, A: torch.Tensor, y: torch.Tensor) -> None:
        self.V.copy_(V)
        self.y.copy_(y)
        self.A.copy_(A)

    def build_graph(self) -> None:
        """Dense A -> the static typed CSR and CSC, on the stream (capturable:
        no host sync).  rowptr and the first nnz entries are what
        TypedGraph.from_dense builds; entries past nnz get column B*N, so the
        CSC builder's stable sort (over cap entries, B*N + 1 columns) puts them
        after every real entry and colptr[B*N] = nnz."""
        B, N, L, _ = self.A.shape
        rows = B * N
        st = current_stream_handle(self.A.device)
        strides = (ctypes.c_int64 * 4)(*self.A.stride())
        call("grl_dense_to_csr_rowptr", self.A.data_ptr(), B, N, L, strides, self.rowptr.data_ptr(),
             self.ws_rowptr.data_ptr(), self.ws_rowptr.numel(), st)
        call("grl_dense_to_csr_fill", self.A.data_ptr(), B, N, L, strides, self.rowptr.data_ptr(),
             self.colidx.data_ptr(), self.vals.data_ptr() if self.vals is not None else None, st)
        self.colidx.masked_fill_(self.slot >= self.rowptr[-1], rows)  # device compare: no sync
        c = self.csc
        call("grl_csr_to_csc", ctypes.byref(self.graph.csr_c()), rows + 1, c["colptr"].data_ptr(),
             c["zrow"].data_ptr(), c["eid"].data_ptr(), c["cvals"].data_ptr() if c["cvals"] is not None else None,
             self.ws_csc.data_ptr(), self.ws_csc.numel(), st)

    def load(self, V: torch.Tensor, g: TypedGraph, y: torch.Tensor) -> None:
        n = g.nnz
        self.V.copy_(V)
        self.y.copy_(y)
        self.rowptr.copy_(g.rowptr)
        c = g.csc()
        self.csc["colptr"].copy_(c["colptr"])
        if n:
            self.colidx[:n].copy_(g.colidx)
            self.csc["zrow"][:n].copy_(c["zrow"][:n])
            self.csc["eid"][:n].copy_(c["eid"][:n])
            if self.vals is not None:
                self.vals[:n].copy_(g.vals)
                self.csc["cvals"][:n].copy_(c["cvals"][:n])


class StepGraph:
    def __init__(self, procedure, mode: str = "capture"):
        if mode not in ("capture", "static"):
            raise ValueError(f"capture_train_step must be true/'capture' or 'static', got {mode!r}")
        from gnn.models.networks.drop_robust_gcn import EdgeDropout, FeatureDropout

        self.proc, self.mode = procedure, mode
        dev = procedure.device
        if dev.type != "cuda":
            raise RuntimeError("capture_train_step needs a ROCm device")
        self.device = dev
        self.buckets: "OrderedDict[tuple, _Bucket]" = OrderedDict()
        self.seen: Dict[tuple, int] = {}
        self.seed_t = torch.zeros(1, dtype=torch.int64, device=dev)
        # every hash-masked dropout (DropEdge and the feature dropout) reads the step's seed word
        self.edge_dropouts = [m for m in procedure.model.modules() if isinstance(m, (EdgeDropout, FeatureDropout))]
        for m in self.edge_dropouts:
            m.seed_source = self.seed_t
        fixed = [m.seed for m in self.edge_dropouts if m.seed is not None]
        self.base_seed = fixed[0] if fixed else None
        self.step = 0
        self.replays = 0
        self.captures = 0
        opt = procedure.optimizer
        for group in opt.param_groups:  # a captured step reads the LR and the step count from device memory
            if "capturable" in group:
                group["capturable"] = True
            if "lr" in group and not isinstance(group["lr"], torch.Tensor):
                group["lr"] = torch.tensor(float(group["lr"]), device=dev)
        self.capturable = mode == "capture" and (not procedure.distributed or
                                                 torch.distributed.get_backend() == "nccl")

    # ---------------------------------------------------------------- seeds
    def _step_seed(self) -> int:
        if self.base_seed is not None:
            return _mix64(self.base_seed * 0x9E3779B97F4A7C15 + self.step) & ((1 << 62) - 1)
        return int(torch.randint(0, 2 ** 62, (1,)).item())  # host generator: torch.manual_seed reproduces it

    # ----------------------------------------------------------------- step
    def _key(self, V: torch.Tensor, g: TypedGraph):
        cap = max(1024, 1 << max(0, int(g.nnz - 1).bit_length()))
        return tuple(V.shape) + (cap, g.vals is not None)

    def _dense_in_graph(self, V: torch.Tensor, A: torch.Tensor) -> bool:
        """A dense batch whose graph can be built inside the replay: the
        collate layout, a small capacity, and no row that could be heavy
        (a row segment holds at most N entries)."""
        if V.dim() != 3 or A.dim() != 4 or A.shape[0] != V.shape[0] or A.shape[1] != V.shape[1] \
                or A.shape[3] != A.shape[1] or V.shape[0] * V.shape[1] > MAX_ROWS:
            return False
        from grl.graph import SPLIT_THRESHOLD

        B, N, L, _ = A.shape
        return B * N * L * N <= DENSE_IN_GRAPH_MAX and L * N <= SPLIT_THRESHOLD

    def _bucket(self, key, make) -> _Bucket:
        b = self.buckets.get(key)
        if b is None:
            b = make()
            self.buckets[key] = b
            while len(self.buckets) > MAX_BUCKETS:
                self.buckets.popitem(last=False)
        self.buckets.move_to_end(key)
        return b

    def eligible(self, V: torch.Tensor, g: TypedGraph) -> bool:
        if V.dim() != 3 or V.shape[0] * V.shape[1] > MAX_ROWS or g.nnz >= 2 ** 31:
            return False
        return g._split("csr", 1) is None and g._split("csc", 1) is None

    def _compute(self, b: _Bucket):
        p = self.proc
        if b.A is not None:
            b.build_graph()
        logits = p.model.forward([b.V, b.graph])
        loss = p.criterion(logits, b.y)
        loss.backward()
        p._sync_gradients()
        nn.utils.clip_grad_norm_(p.model.parameters(), p.config.max_grad_norm)
        p.optimizer.step()
        return loss.detach(), logits.detach()

    def run(self, batch: Dict[str, Any]):
        """One training step; None when the batch is not eligible (the caller
        runs the ordinary eager step)."""
        from gnn.trainer.training_procedures.kv_procedure import batch_graph

        p = self.proc
        V = batch["textline_encoding"].float().to(self.device)
        y = batch["node_label"].to(self.device)
        A_src = batch.get("adjacency_matrix") if "typed_edges" not in batch else None
        if A_src is not None and self._dense_in_graph(V, A_src):
            B, N, L, _ = A_src.shape
            # the values are always kept (0/1 graphs then multiply by exact ones: the same bits as without
            # them) -- deciding per batch would cost a host pass over A (~0.13 ms of a 1.7 ms step)
            key = tuple(V.shape) + ("dense", L)
            b = self._bucket(key, lambda: _Bucket(B, N, V.shape[2], L, B * N * L * N, True, self.device, dense=True))
            b.load_dense(V, A_src, y)
        else:
            A = batch_graph(batch, self.device)
            g = A if isinstance(A, TypedGraph) else p.model.to_graph(A)
            if not self.eligible(V, g):
                return None
            key = self._key(V, g)
            b = self._bucket(key, lambda: _Bucket(V.shape[0], V.shape[1], V.shape[2], g.num_types, key[-2],
                                                  g.vals is not None, self.device))
            b.load(V, g, y)
        self.seed_t.fill_(self._step_seed())
        self.step += 1
        p.model.train()
        self.seen[key] = self.seen.get(key, 0) + 1
        if self.capturable and b.hip_graph is None and not b.failed and self.seen[key] >= 2:
            self._capture(b)
        if b.hip_graph is not None:
            b.hip_graph.replay()
            self.replays += 1
            loss, logits = b.out
        else:
            for m in self.edge_dropouts:
                m.reset_calls()
            p.optimizer.zero_grad(set_to_none=True)
            loss, logits = self._compute(b)
        return loss, logits, b.y

    def _capture(self, b: _Bucket) -> None:
        p = self.proc
        for m in self.edge_dropouts:
            m.reset_calls()
        p.optimizer.zero_grad(set_to_none=True)  # the graph's backward assigns every .grad afresh
        torch.cuda.synchronize(self.device)
        hg = torch.cuda.CUDAGraph()
        try:
            with torch.cuda.graph(hg):
                b.out = self._compute(b)
        except Exception as err:  # not capturable here: this bucket keeps the eager static step
            b.failed = True
            b.out = None
            p.logger.warning(f"training-step capture failed for a batch of {tuple(b.V.shape)}: {err!r}; "
                             "running it eagerly")
            torch.cuda.synchronize(self.device)
            p.optimizer.zero_grad(set_to_none=True)
            return
        b.hip_graph = hg
        self.captures += 1

    def stats(self) -> Dict[str, Any]:
        return {"mode": self.mode, "steps": self.step, "replays": self.replays, "captures": self.captures,
                "buckets": len(self.buckets)}


def as_mode(value) -> Optional[str]:
    """Config value of capture_train_step -> None (off), "capture" or "static"."""
    if value in (None, False, 0, "false", "False", "off", ""):
        return None
    if value in (True, 1, "true", "True", "capture"):
        return "capture"
    if value == "static":
        return "static"
    raise ValueError(f"capture_train_step must be true/false/'capture'/'static', got {value!r}")
