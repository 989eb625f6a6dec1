"""Node-range sharding of the GraphConv aggregation over GPUs.

One process per GPU (torch.distributed, backend "nccl" = RCCL over xGMI).
Rank r owns node rows [row_begin_r, row_end_r): their feature rows, their
typed-CSR rows (destination = owned node) and their output rows.  The only
data-path exchange is the halo: before each aggregation every rank receives
the feature rows of the remote sources its edges reference, via one
all-to-all-v (`all_to_all_single` with per-peer split sizes); backward sends
the halo-row gradients back the same way and the owner adds them in peer
order (deterministic, no float atomics).

The plan is static per graph and built once (two small all-to-alls of ids).
Edge ids stay global (edge_id_base = nnz of lower ranks, self ids
E_total + global node), so fused DropEdge masks are identical to the
single-GPU run and the forward is bitwise identical to it.

Two exchange layouts, chosen collectively per graph (HaloPlan.mode):
  "sparse"  X_ext = [own rows | needed remote rows in owner order]; the owner
            packs the rows each peer asked for and one all-to-all-v moves
            them.  Right when a shard references a small part of the rest.
  "dense"   X_ext = [own rows padded to `stride` | every rank's rows, rank q
            at stride*(1+q)], filled by one all_gather (no packing, no
            id lists).  Right when nearly every remote row is referenced --
            Erdos-Renyi graphs at avg_deg 32 need ~98% of each peer's rows,
            where packing would cost two extra HBM passes over the halo for
            nothing.  "auto" picks dense when the referenced remote rows are
            >= DENSE_HALO_FRACTION of all remote rows (summed over ranks).
Both layouts give the same Z bitwise (the kernel reads the same values in the
same edge order) and the same dX values (peer-order sums; a peer's rows that
no edge referenced contribute +0.0).

Communication goes through one dispatch layer (the `_c_*` functions below),
whose `group` is either a torch.distributed group -- RCCL ("nccl"), the
product; gloo, whose device tensors are staged through the host -- or a
LocalGroup member: P virtual ranks driven as threads of one process, with
torch.distributed's asynchronous stream semantics emulated by device copies
(LocalGroup).  Every function above the dispatch layer runs unchanged on
all three, so the code RCCL runs on a multi-GPU node -- async handles, slot
views, landing copies, peer-order combines -- also runs, with P > 1, on a
one-GPU box (RCCL refuses two ranks on one device), and the RCCL calls
themselves run on a one-rank "nccl" group (tests/rccl_loopback.py).
"""
from __future__ import annotations

import threading
from dataclasses import dataclass
from typing import List, Optional

import torch
import torch.distributed as dist

from ._lib import trace
from .graph import DropEdge, TypedGraph
from .ops import graph_conv, graph_linear, typed_aggregate


# ------------------------------------------------------------ virtual ranks
class _LocalWork:
    """A LocalGroup transfer's handle: wait() orders the caller's current
    stream after the transfer on every rank it involves (a collective
    completes on all ranks), as a torch.distributed work handle does."""

    def __init__(self, events=(), ready=None):
        self.events, self.ready = list(events), ready

    def wait(self):
        if self.ready is not None:  # a send: the receiver's copy must have been queued
            self.events += self.ready()
            self.ready = None
        if self.events:
            cur = torch.cuda.current_stream(self.events[0][1])
            for ev, _ in self.events:
                cur.wait_event(ev)
        self.events = []
        return True


class LocalGroup:
    """P virtual ranks in one process: the stand-in for a P-rank process
    group when the ranks are threads (one GPU can hold one RCCL rank only).

    Each member(r) is passed as `group` to the functions of this module.  A
    collective on rank r records an event on r's current stream (its inputs
    as queued); after every rank has issued it, rank r's receive side runs
    on r's own transfer stream once every rank's event has fired, and the
    handle's wait() makes the caller's stream wait for every rank's transfer
    -- torch.distributed's async contract (the transfer starts after the work
    queued before it; inputs must not change until wait()).  Reductions add
    in rank order.  Ranks must issue the same collectives in the same order:
    a mismatch raises instead of hanging.  Point-to-point transfers
    (batch_isend_irecv) match sends and receives per (source, destination)
    in posting order.  Host (CPU) tensors are copied at once."""

    def __init__(self, world: int, timeout: float = 120.0):
        self.world = int(world)
        self.timeout = timeout
        self.barrier = threading.Barrier(self.world, timeout=timeout)
        self.slots = [[None] * self.world for _ in range(2)]  # double-buffered per collective sequence number
        self.done = [[None] * self.world for _ in range(2)]
        self.cond = threading.Condition()
        self.mail = {}

    def member(self, rank: int) -> "LocalRank":
        return LocalRank(self, rank)

    def abort(self) -> None:
        self.barrier.abort()
        with self.cond:
            self.cond.notify_all()


class LocalRank:
    def __init__(self, grp: LocalGroup, rank: int):
        self.g, self.rank, self.world = grp, int(rank), grp.world
        self.seq = 0
        self._stream = {}

    def _side(self, device):
        s = self._stream.get(device)
        if s is None:
            s = self._stream[device] = torch.cuda.Stream(device)
        return s

    @staticmethod
    def _ready_event(t):
        if not t.is_cuda:
            return None
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(t.device))
        return ev, t.device

    def _run(self, kind: str, payload, recv, like, async_op: bool, phases: int = 1):
        """One collective: post `payload`; when every rank has posted, run
        recv(payloads, phase) for phase 0..phases-1 on this rank's transfer
        stream (phase 0 after every rank's inputs are ready, phase p after
        every rank's phase p-1: a later phase may overwrite what an earlier
        one read).  Sequence numbers alternate between two slot sets: a rank
        can post collective n+2 only after every rank has left collective n."""
        g, r = self.g, self.rank
        k = self.seq % 2
        self.seq += 1
        ev = self._ready_event(like)
        g.slots[k][r] = (kind, payload, ev)
        g.done[k][r] = {}
        g.barrier.wait()
        kinds = {g.slots[k][q][0] for q in range(self.world)}
        if len(kinds) != 1:
            g.abort()
            raise RuntimeError(f"LocalGroup: ranks issued different collectives {sorted(kinds)}")
        pays = [g.slots[k][q][1] for q in range(self.world)]
        waits = [g.slots[k][q][2] for q in range(self.world) if g.slots[k][q][2] is not None]
        for ph in range(phases):
            if ev is not None:
                side = self._side(ev[1])
                for e, _ in waits:
                    side.wait_event(e)
                with torch.cuda.stream(side):
                    recv(pays, ph)
                d = torch.cuda.Event()
                d.record(side)
                g.done[k][r][ph] = (d, ev[1])
            else:
                recv(pays, ph)
            g.barrier.wait()  # every rank's phase is queued (its event posted)
            if ev is not None:
                waits = [g.done[k][q][ph] for q in range(self.world)]
        work = _LocalWork(waits if ev is not None else [])
        if not async_op:
            work.wait()
            return None
        return work

    # -- the collectives of torch.distributed this module uses --
    def all_gather(self, outs, inp, async_op=False):
        r = self.rank

        def recv(pays, ph):
            for q in range(self.world):
                outs[q].copy_(pays[q])
                _keep_for_stream(outs[q], pays[q])
        return self._run("all_gather", inp, recv, inp, async_op)

    def all_gather_into_tensor(self, out, inp, async_op=False):
        n = inp.shape[0]

        def recv(pays, ph):
            for q in range(self.world):
                out[q * n:(q + 1) * n].copy_(pays[q])
                _keep_for_stream(pays[q])
            _keep_for_stream(out)
        return self._run("all_gather_into", inp, recv, inp, async_op)

    def all_to_all_single(self, out, inp, out_splits=None, in_splits=None, async_op=False):
        W, r = self.world, self.rank
        osp = list(out_splits) if out_splits is not None else [out.shape[0] // W] * W
        isp = list(in_splits) if in_splits is not None else [inp.shape[0] // W] * W

        def recv(pays, ph):
            off = 0
            for q in range(W):
                t_q, isp_q = pays[q]
                if isp_q[r] != osp[q]:
                    raise RuntimeError(f"LocalGroup all_to_all: rank {q} sends {isp_q[r]} rows, rank {r} expects {osp[q]}")
                o = sum(isp_q[:r])
                if osp[q]:
                    out[off:off + osp[q]].copy_(t_q[o:o + osp[q]])
                _keep_for_stream(t_q)
                off += osp[q]
            _keep_for_stream(out)
        return self._run("all_to_all", (inp, isp), recv, inp, async_op)

    def all_reduce(self, t, op="sum", async_op=False):
        tmp = torch.empty_like(t)
        name = op if isinstance(op, str) else {dist.ReduceOp.SUM: "sum", dist.ReduceOp.MIN: "min",
                                                dist.ReduceOp.MAX: "max"}[op]

        def recv(pays, ph):
            if ph == 0:  # reduce everyone's input in rank order into tmp (inputs untouched)
                tmp.copy_(pays[0])
                for q in range(1, self.world):
                    if name == "sum":
                        tmp.add_(pays[q])
                    elif name == "min":
                        torch.minimum(tmp, pays[q], out=tmp)
                    else:
                        torch.maximum(tmp, pays[q], out=tmp)
                _keep_for_stream(tmp, *pays)
            else:  # every rank has read every input: overwrite mine
                t.copy_(tmp)
                _keep_for_stream(t)
        return self._run("all_reduce_" + name, t, recv, t, async_op, phases=2)

    def broadcast(self, t, src=0, async_op=False):
        r = self.rank

        def recv(pays, ph):
            if r != src:
                t.copy_(pays[src])
                _keep_for_stream(t, pays[src])
        return self._run("broadcast", t, recv, t, async_op)

    def barrier(self):
        self.g.barrier.wait()

    def batch_isend_irecv(self, sends, recvs):
        """sends [(tensor, dst)], recvs [(tensor, src)] -> works."""
        g, r = self.g, self.rank
        works = []
        for t, dst in sends:
            box = {"ev": self._ready_event(t), "t": t, "done": None}
            with g.cond:
                g.mail.setdefault((r, dst), []).append(box)
                g.cond.notify_all()

            def ready(box=box):
                with g.cond:
                    if not g.cond.wait_for(lambda: box["done"] is not None, timeout=g.timeout):
                        raise RuntimeError(f"LocalGroup: rank {r}'s send was never received")
                return [box["done"]] if box["done"][0] is not None else []
            works.append(_LocalWork([], ready))
        for t, src in recvs:
            with g.cond:
                if not g.cond.wait_for(lambda: g.mail.get((src, r)), timeout=g.timeout):
                    raise RuntimeError(f"LocalGroup: rank {r} waited for a send from rank {src} that never came")
                box = g.mail[(src, r)].pop(0)
            if box["t"].shape != t.shape:
                raise RuntimeError(f"LocalGroup p2p: rank {src} sent {tuple(box['t'].shape)}, rank {r} receives "
                                   f"{tuple(t.shape)}")
            if t.is_cuda:
                side = self._side(t.device)
                side.wait_event(box["ev"][0])
                with torch.cuda.stream(side):
                    t.copy_(box["t"])
                    _keep_for_stream(t, box["t"])
                d = torch.cuda.Event()
                d.record(side)
                done = (d, t.device)
                works.append(_LocalWork([done]))
            else:
                t.copy_(box["t"])
                done = (None, None)
            with g.cond:
                box["done"] = done
                g.cond.notify_all()
        return works


def _keep_for_stream(*ts) -> None:
    """The caching allocator must not hand these tensors' memory out again
    before the current (transfer) stream's work on them has run -- what
    ProcessGroupNCCL's recordStream does for RCCL transfers."""
    for t in ts:
        if t is not None and t.is_cuda:
            t.record_stream(torch.cuda.current_stream(t.device))


def _local(group) -> bool:
    return isinstance(group, LocalRank)


def _comm_on(group) -> bool:
    """A group to communicate over: a LocalGroup member or an initialised
    torch.distributed process group (a one-rank group included)."""
    return _local(group) or (dist.is_available() and dist.is_initialized())


def _world(group) -> int:
    if _local(group):
        return group.world
    return dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1


def _rank(group) -> int:
    if _local(group):
        return group.rank
    return dist.get_rank(group) if dist.is_available() and dist.is_initialized() else 0


def _host_staged(group) -> bool:
    """gloo moves device tensors only through host copies (used to smoke-test
    the N>1 path with several ranks on one GPU; production uses RCCL)."""
    return not _local(group) and dist.is_available() and dist.is_initialized() and dist.get_backend(group) == "gloo"


# ---- the dispatch layer: each function is the one place its collective is
# issued (RCCL / gloo through torch.distributed, or the LocalGroup) ----
def _c_all_gather(outs, inp, group, async_op=False):
    if _local(group):
        return group.all_gather(outs, inp, async_op)
    return dist.all_gather(outs, inp, group=group, async_op=async_op)


def _c_all_gather_into_tensor(out, inp, group, async_op=False):
    if _local(group):
        return group.all_gather_into_tensor(out, inp, async_op)
    return dist.all_gather_into_tensor(out, inp, group=group, async_op=async_op)


def _c_all_to_all_single(out, inp, out_splits, in_splits, group, async_op=False):
    if _local(group):
        return group.all_to_all_single(out, inp, out_splits, in_splits, async_op)
    return dist.all_to_all_single(out, inp, out_splits, in_splits, group=group, async_op=async_op)


def _c_all_reduce(t, op, group, async_op=False):
    if _local(group):
        return group.all_reduce(t, op, async_op)
    return dist.all_reduce(t, op=op, group=group, async_op=async_op)


def _c_broadcast(t, src_in_group, group):
    if _local(group):
        return group.broadcast(t, src_in_group)
    src = dist.get_global_rank(group, src_in_group) if group is not None else src_in_group
    return dist.broadcast(t, src, group=group)


def _c_p2p(sends, recvs, group):
    if _local(group):
        return group.batch_isend_irecv(sends, recvs)
    ops = [dist.P2POp(dist.isend, t, group=group, group_peer=dst) for t, dst in sends]
    ops += [dist.P2POp(dist.irecv, t, group=group, group_peer=src) for t, src in recvs]
    return dist.batch_isend_irecv(ops)


def all_to_all_v(out: torch.Tensor, inp: torch.Tensor, out_splits, in_splits, group=None) -> None:
    if _host_staged(group) and (out.is_cuda or inp.is_cuda):
        o = torch.empty(out.shape, dtype=out.dtype)
        dist.all_to_all_single(o, inp.cpu(), out_splits, in_splits, group=group)
        out.copy_(o)
    else:
        _c_all_to_all_single(out, inp, out_splits, in_splits, group)


def all_gather_into(out: torch.Tensor, inp: torch.Tensor, group=None) -> None:
    """out = concat over ranks of inp (equal sizes)."""
    if _host_staged(group) and (out.is_cuda or inp.is_cuda):
        parts = all_gather_list(inp, group)
        out.copy_(torch.cat(parts, 0))
    else:
        _c_all_gather_into_tensor(out, inp, group)


def all_reduce_sum(t: torch.Tensor, group=None) -> torch.Tensor:
    """t summed over the ranks of `group`, in place (host-staged on gloo);
    returns t.  No group: t unchanged."""
    if not _comm_on(group):
        return t
    if _host_staged(group) and t.is_cuda:
        h = t.cpu()
        _c_all_reduce(h, dist.ReduceOp.SUM, group)
        t.copy_(h)
    else:
        _c_all_reduce(t, dist.ReduceOp.SUM, group)
    return t


def all_gather_list(t: torch.Tensor, group=None) -> List[torch.Tensor]:
    src = t.cpu() if _host_staged(group) else t
    outs = [torch.empty_like(src) for _ in range(_world(group))]
    _c_all_gather(outs, src, group)
    return outs


DENSE_HALO_FRACTION = 0.75


@dataclass
class HaloPlan:
    row_begin: int
    row_end: int
    n_loc: int
    n_halo: int                  # rows of X_ext after the own rows (dense: padding + all gathered rows)
    bounds: List[int]            # row ranges of all ranks: [b_0, b_1, ..., b_P]
    send_index: torch.Tensor     # sparse: int64 local rows, concatenated per destination peer
    send_counts: List[int]       # sparse: rows I send to each peer
    recv_counts: List[int]       # sparse: halo rows I receive from each peer (owner order)
    halo_ids: torch.Tensor       # int64 global ids of the remote rows my edges reference, ascending
    colidx_local: torch.Tensor   # int32 column into X_ext (own -> id - row_begin)
    edge_id_base: int
    num_edges_total: int
    mode: str = "sparse"         # "sparse" | "dense" (module docstring)
    stride: int = 0              # dense: max shard rows; rank q's rows sit at X_ext[stride*(1+q):]
    rank: int = 0                # this shard's rank in the group

    @property
    def referenced_halo_rows(self) -> int:
        return int(self.halo_ids.numel())


def build_halo_plan(colidx: torch.Tensor, row_begin: int, row_end: int, group=None,
                    mode: str = "auto") -> HaloPlan:
    """Collective: every rank of `group` calls it with its own shard (and the
    same `mode`)."""
    if mode not in ("auto", "sparse", "dense"):
        raise ValueError(f"halo mode must be auto|sparse|dense, got {mode!r}")
    dev = colidx.device
    world, rank = _world(group), _rank(group)
    c = colidx.long()
    if world > 1:
        rr = torch.tensor([row_begin, row_end, colidx.numel()], dtype=torch.int64, device=dev)
        allr = torch.stack([x.cpu() for x in all_gather_list(rr, group)])
        begins, ends, nnzs = allr[:, 0].tolist(), allr[:, 1].tolist(), allr[:, 2].tolist()
        bounds = _check_bounds(begins, ends)
    else:
        bounds, nnzs = [row_begin, row_end], [colidx.numel()]
    _check_columns(c, bounds, world)
    halo_ids = _halo_ids(c, row_begin, row_end)
    if world > 1 and mode == "auto":
        referenced = sum(int(x) for x in all_gather_list(
            torch.tensor([halo_ids.numel()], dtype=torch.int64, device=dev), group))
        mode = _auto_mode(referenced, bounds)
    asked = None
    if world > 1 and mode != "dense":
        ends_t = torch.tensor(bounds[1:], dtype=torch.int64, device=dev)
        owner = torch.searchsorted(ends_t, halo_ids, right=True)
        need = torch.bincount(owner, minlength=world).to(torch.int64)
        asked_counts = torch.empty_like(need)
        all_to_all_v(asked_counts, need, None, None, group)
        recv_counts = need.cpu().tolist()
        send_counts = asked_counts.cpu().tolist()
        asked_ids = torch.empty(sum(send_counts), dtype=torch.int64, device=dev)
        all_to_all_v(asked_ids, halo_ids.contiguous(), send_counts, recv_counts, group)
        asked = (asked_ids, send_counts, recv_counts)
    return _make_plan(c, row_begin, row_end, bounds, nnzs, rank, "dense" if mode == "dense" else "sparse",
                      halo_ids, asked)


def build_halo_plans_local(colidx_per_rank: List[torch.Tensor], bounds: List[int],
                           mode: str = "auto") -> List[HaloPlan]:
    """Every rank's HaloPlan at once, in one process, without a process group:
    the plans build_halo_plan returns on rank r of a P-rank group when rank r
    holds colidx_per_rank[r] and the rows [bounds[r], bounds[r+1]).  (Used to
    drive several shards from one process, e.g. the one-GPU tests of the
    pipelined exchange.)"""
    if mode not in ("auto", "sparse", "dense"):
        raise ValueError(f"halo mode must be auto|sparse|dense, got {mode!r}")
    world = len(bounds) - 1
    if len(colidx_per_rank) != world:
        raise ValueError(f"{len(colidx_per_rank)} shards for {world} node ranges")
    bounds = _check_bounds(bounds[:-1], bounds[1:])
    nnzs = [int(c.numel()) for c in colidx_per_rank]
    cs = [c.long() for c in colidx_per_rank]
    for c in cs:
        _check_columns(c, bounds, world)
    halo = [_halo_ids(c, bounds[r], bounds[r + 1]) for r, c in enumerate(cs)]
    if mode == "auto":
        mode = _auto_mode(sum(int(h.numel()) for h in halo), bounds) if world > 1 else "sparse"
    plans = []
    for r, c in enumerate(cs):
        asked = None
        if world > 1 and mode != "dense":
            ends_t = torch.tensor(bounds[1:], dtype=torch.int64, device=c.device)
            owners = [torch.searchsorted(ends_t, h, right=True) for h in halo]
            recv_counts = torch.bincount(owners[r], minlength=world).tolist()
            mine = [halo[q][owners[q] == r].to(c.device) for q in range(world)]  # what peer q asks of me
            asked = (torch.cat(mine), [int(m.numel()) for m in mine], recv_counts)
        plans.append(_make_plan(c, bounds[r], bounds[r + 1], bounds, nnzs, r,
                                "dense" if mode == "dense" else "sparse", halo[r], asked))
    return plans


def _check_bounds(begins, ends) -> List[int]:
    begins, ends = [int(b) for b in begins], [int(e) for e in ends]
    if begins != sorted(begins) or any(ends[i] != begins[i + 1] for i in range(len(begins) - 1)):
        raise ValueError(f"node ranges must be contiguous in rank order: {list(zip(begins, ends))}")
    return begins + [ends[-1]]


def _check_columns(c: torch.Tensor, bounds: List[int], world: int) -> None:
    if world > 1 and c.numel() and (int(c.min()) < bounds[0] or int(c.max()) >= bounds[-1]):
        raise ValueError(f"column ids outside the global node range [{bounds[0]}, {bounds[-1]})")


def _halo_ids(c: torch.Tensor, row_begin: int, row_end: int) -> torch.Tensor:
    own = (c >= row_begin) & (c < row_end)
    return torch.unique(c[~own])  # sorted ascending => grouped by owner


def _auto_mode(referenced: int, bounds: List[int]) -> str:
    remote = (len(bounds) - 2) * (bounds[-1] - bounds[0])
    return "dense" if remote and referenced >= DENSE_HALO_FRACTION * remote else "sparse"


def _make_plan(c: torch.Tensor, row_begin: int, row_end: int, bounds: List[int], nnzs: List[int], rank: int,
               mode: str, halo_ids: torch.Tensor, asked) -> HaloPlan:
    """The plan of one shard from what the collective (or the in-process
    builder) learned: the node ranges, every shard's edge count and, for the
    sparse layout, (ids the peers ask of this rank in peer order, send counts,
    receive counts)."""
    dev = c.device
    world = len(bounds) - 1
    n_loc = row_end - row_begin
    edge_id_base, num_edges_total = sum(nnzs[:rank]), sum(nnzs)
    own = (c >= row_begin) & (c < row_end)
    if world > 1 and mode == "dense":
        stride = max(bounds[i + 1] - bounds[i] for i in range(world))
        ends_t = torch.tensor(bounds[1:], dtype=torch.int64, device=dev)
        begins_t = torch.tensor(bounds[:-1], dtype=torch.int64, device=dev)
        owner = torch.searchsorted(ends_t, c, right=True)
        slot = stride * (1 + owner) + (c - begins_t[owner.clamp(max=world - 1)])
        colidx_local = torch.where(own, c - row_begin, slot).to(torch.int32)
        empty = torch.zeros(0, dtype=torch.int64, device=dev)
        return HaloPlan(row_begin, row_end, n_loc, stride * (world + 1) - n_loc, bounds, empty, [0] * world,
                        [0] * world, halo_ids, colidx_local, edge_id_base, num_edges_total, "dense", stride, rank)
    if world > 1:
        asked_ids, send_counts, recv_counts = asked
        send_index = asked_ids.to(dev) - row_begin
        if send_index.numel() and (int(send_index.min()) < 0 or int(send_index.max()) >= n_loc):
            raise RuntimeError("halo plan: a peer asked for rows this rank does not own")
    else:
        if halo_ids.numel():
            raise ValueError(f"single shard references {halo_ids.numel()} nodes outside [{row_begin}, {row_end})")
        recv_counts, send_counts = [0], [0]
        send_index = torch.zeros(0, dtype=torch.int64, device=dev)
    slot = n_loc + torch.searchsorted(halo_ids, c)
    colidx_local = torch.where(own, c - row_begin, slot).to(torch.int32)
    return HaloPlan(row_begin, row_end, n_loc, int(halo_ids.numel()), bounds, send_index, list(send_counts),
                    list(recv_counts), halo_ids, colidx_local, edge_id_base, num_edges_total, "sparse", n_loc, rank)


class _HaloExchange(torch.autograd.Function):
    @staticmethod
    def forward(ctx, X_loc: torch.Tensor, plan: HaloPlan, group):
        with trace("grl.halo_exchange"):
            return _HaloExchange._forward(ctx, X_loc, plan, group)

    @staticmethod
    def _forward(ctx, X_loc: torch.Tensor, plan: HaloPlan, group):
        F = X_loc.shape[1]
        X_ext = X_loc.new_empty(plan.n_loc + plan.n_halo, F)
        X_ext[: plan.n_loc].copy_(X_loc)
        if plan.mode == "dense":
            X_ext[plan.n_loc: plan.stride].zero_()
            all_gather_into(X_ext[plan.stride:], X_ext[: plan.stride], group)
        elif _world(group) > 1 or plan.n_halo:
            send = X_loc.index_select(0, plan.send_index)
            all_to_all_v(X_ext[plan.n_loc:], send, plan.recv_counts, plan.send_counts, group)
        ctx.plan, ctx.group = plan, group
        return X_ext

    @staticmethod
    def backward(ctx, dX_ext: torch.Tensor):
        plan, group = ctx.plan, ctx.group
        dX_ext = dX_ext.contiguous()
        dX_loc = dX_ext[: plan.n_loc].clone()
        if plan.mode == "dense":
            world, st = len(plan.bounds) - 1, plan.stride
            back = dX_ext.new_empty(world * st, dX_ext.shape[1])
            all_to_all_v(back, dX_ext[st:], [st] * world, [st] * world, group)
            me = plan.rank
            for q in range(world):  # peer order, like the sparse path
                if q != me:
                    dX_loc += back[q * st: q * st + plan.n_loc]
        elif _world(group) > 1 or plan.n_halo:
            back = dX_ext.new_empty(sum(plan.send_counts), dX_ext.shape[1])
            all_to_all_v(back, dX_ext[plan.n_loc:], plan.send_counts, plan.recv_counts, group)
            off = 0
            for cnt in plan.send_counts:  # peer order; indices unique within a peer -> deterministic
                if cnt:
                    dX_loc.index_add_(0, plan.send_index[off:off + cnt], back[off:off + cnt])
                off += cnt
        return dX_loc, None, None


def halo_exchange(X_loc: torch.Tensor, plan: HaloPlan, group=None) -> torch.Tensor:
    """[own rows; halo rows] feature matrix for the local aggregation."""
    if plan.n_halo == 0 and _world(group) == 1:
        return X_loc
    return _HaloExchange.apply(X_loc, plan, group)


def halo_exchange_into(X_loc: torch.Tensor, X_ext: torch.Tensor, send_buf: torch.Tensor, plan: HaloPlan,
                       group=None) -> None:
    """No-autograd, no-allocation form for inference / benchmarking:
    X_ext[:n_loc] must already alias or hold X_loc; fills X_ext[n_loc:]
    (dense plans: the pad rows X_ext[n_loc:stride] travel as they are and are
    never read by the kernel; send_buf is unused and may be empty)."""
    if _world(group) == 1 and plan.n_halo == 0:
        return
    if plan.mode == "dense":
        all_gather_into(X_ext[plan.stride:], X_ext[: plan.stride], group)
        return
    torch.index_select(X_loc, 0, plan.send_index, out=send_buf)
    all_to_all_v(X_ext[plan.n_loc:], send_buf, plan.recv_counts, plan.send_counts, group)


class HaloPipeline:
    """Halo exchange overlapped with the aggregation (forward, no autograd).

    The feature columns are cut into `chunks` slices of F/chunks columns.
    Slice c's halo rows travel (RCCL all-gather or all-to-all-v on a side
    stream, in slice order) while the compute stream aggregates slice c-1
    with grl_typed_spmm_fwd_slice into Z's columns of that slice.  Every Z
    element is the same edges in the same order as the unsliced aggregation,
    so the result is bitwise equal to it (and to the single-GPU run); what
    changes is that after the first slice the exchange runs under the
    gather.  chunks=1 is the serial exchange-then-aggregate step.

    Tables (HBM, per slice c, rows as the plan's X_ext, F/chunks columns):
      dense:  [own rows padded to stride | every rank's rows]
      sparse: [own rows | referenced halo rows in owner order]
    """

    def __init__(self, sg: "ShardedGraph", F: int, chunks: int = 2, device=None, exchange=None):
        """exchange: None = torch.distributed collectives on sg.group.
        Otherwise an object standing in for them (several shards driven from
        one process, e.g. the one-GPU tests of the overlapped branch) with
          .world, .async_op                     (the side-stream branch runs iff async_op)
          .forward(pipe, c, async_op)           fill pipe.tables[c]'s halo rows
          .backward(pipe, c, async_op)          fill pipe.gback[c] from the peers' pipe.gtables[c]
        each returning None (done, in stream order) or, when async_op, a
        handle whose .wait() orders the current stream after the transfer --
        torch.distributed's async work semantics: the transfer starts after
        the work queued on the current stream when it was issued."""
        plan = sg.plan
        if chunks < 1 or F % chunks:
            raise ValueError(f"chunks must divide F={F} (got {chunks}); slices of a multiple of 4 columns take "
                             "the vector path")
        self.sg, self.plan, self.F, self.K, self.Fc = sg, plan, F, chunks, F // chunks
        self.group = sg.group
        self.xchg = exchange
        self.world = exchange.world if exchange is not None else _world(self.group)
        dev = torch.device(device) if device is not None else sg.graph.device
        rows = plan.n_loc + plan.n_halo
        self.tables = torch.empty(chunks, rows, self.Fc, device=dev)
        if plan.mode == "dense":
            self.tables[:, plan.n_loc:plan.stride].zero_()  # shard padding rows: travel, never read
        # a shard exchanges when its group has peers or its plan has halo rows
        # (a one-rank group with a loopback plan: tests/rccl_loopback.py)
        self.moves = self.world > 1 or plan.n_halo > 0
        self.send = None
        if plan.mode == "sparse" and self.moves:
            self.send = torch.empty(chunks, plan.send_index.numel(), self.Fc, device=dev)
        if exchange is not None:
            self.side = torch.cuda.Stream(dev) if dev.type == "cuda" and exchange.async_op else None
        else:
            self.side = torch.cuda.Stream(dev) if dev.type == "cuda" and not _host_staged(self.group) else None

    def _slices(self, X: torch.Tensor) -> torch.Tensor:
        """[rows, F] -> [chunks, rows, Fc] view (no copy)."""
        return X.view(X.shape[0], self.K, self.Fc).permute(1, 0, 2)

    def _pack(self, X_loc: torch.Tensor) -> None:
        p = self.plan
        self.tables[:, :p.n_loc].copy_(self._slices(X_loc))
        if self.send is not None:
            self.send.copy_(self._slices(X_loc.index_select(0, p.send_index)))

    def _exchange(self, c: int):
        """Start slice c's exchange; returns a work handle (or None if done)."""
        if not self.moves:
            return None
        with trace(f"grl.halo_slice{c}"):
            return self._exchange_slice(c)

    def _exchange_slice(self, c: int):
        if self.xchg is not None:
            return self.xchg.forward(self, c, self.side is not None)
        p, t = self.plan, self.tables[c]
        if p.mode == "dense":
            if self.side is None:
                all_gather_into(t[p.stride:], t[:p.stride], self.group)
                return None
            return _c_all_gather_into_tensor(t[p.stride:], t[:p.stride], self.group, async_op=True)
        if self.side is None:
            all_to_all_v(t[p.n_loc:], self.send[c], p.recv_counts, p.send_counts, self.group)
            return None
        return _c_all_to_all_single(t[p.n_loc:], self.send[c], p.recv_counts, p.send_counts, self.group,
                                    async_op=True)

    def run(self, X_loc: torch.Tensor, Z: torch.Tensor, dropedge: Optional[DropEdge] = None,
            aggregate_slice=None) -> torch.Tensor:
        """Z[:, s*F + c*Fc : s*F + (c+1)*Fc] for every slice c (Z contiguous
        [n_loc, segments*F]).  aggregate_slice(table, graph, Z, col0) replaces
        the HIP slice aggregation (CPU tests only)."""
        from .ops import spmm_forward_slice

        agg = aggregate_slice or (lambda table, g, out, col0: spmm_forward_slice(table, g, out, col0))
        graph = self.sg.graph.with_dropedge(dropedge)
        if self.side is None:  # host-staged (gloo) or single rank: in order, no overlap
            self._pack(X_loc)
            for c in range(self.K):
                self._exchange(c)
                agg(self.tables[c], graph, Z, c * self.Fc)
            return Z
        main = torch.cuda.current_stream(X_loc.device)
        self.side.wait_stream(main)  # X_loc is final on the compute stream
        with torch.cuda.stream(self.side):
            self._pack(X_loc)
            works = [self._exchange(c) for c in range(self.K)]
        for c in range(self.K):
            if works[c] is not None:
                works[c].wait()  # the compute stream waits for slice c only
            else:
                main.wait_stream(self.side)
            agg(self.tables[c], graph, Z, c * self.Fc)
        main.wait_stream(self.side)  # buffers are reused by the next call
        return Z

    # ------------------------------------------------------------- backward
    def _grad_buffers(self, device):
        """Slice tables of dX_ext ([chunks, rows, Fc], the forward tables'
        shape) and the receive buffers of the reverse exchange (dense: every
        peer's gradient of my rows, world * stride rows; sparse: the rows I
        sent, sum(send_counts)); allocated on first use, then reused."""
        if getattr(self, "gtables", None) is None:
            p = self.plan
            self.gtables = torch.empty_like(self.tables, device=device)
            back_rows = self.world * p.stride if p.mode == "dense" else sum(p.send_counts)
            self.gback = torch.empty(self.K, back_rows, self.Fc, device=device)
        return self.gtables, self.gback

    def _exchange_back(self, c: int, async_op: bool):
        """Send slice c's halo-row gradients to their owners (the reverse of
        the forward exchange); returns a work handle when async_op."""
        if not self.moves:
            return None
        p, g, back = self.plan, self.gtables[c], self.gback[c]
        with trace(f"grl.halo_back_slice{c}"):
            if self.xchg is not None:
                return self.xchg.backward(self, c, async_op)
            if p.mode == "dense":
                splits = [p.stride] * self.world
                if not async_op:
                    all_to_all_v(back, g[p.stride:], splits, splits, self.group)
                    return None
                return _c_all_to_all_single(back, g[p.stride:], splits, splits, self.group, async_op=True)
            if not async_op:
                all_to_all_v(back, g[p.n_loc:], p.send_counts, p.recv_counts, self.group)
                return None
            return _c_all_to_all_single(back, g[p.n_loc:], p.send_counts, p.recv_counts, self.group,
                                        async_op=True)

    def _combine(self, c: int, dX_loc: torch.Tensor) -> None:
        """dX_loc's columns of slice c = my own rows' gradient + every peer's
        partial for them, in peer order (_HaloExchange.backward's order, so
        the same bits)."""
        p, g, back = self.plan, self.gtables[c], self.gback[c]
        out = dX_loc[:, c * self.Fc:(c + 1) * self.Fc]
        out.copy_(g[:p.n_loc])
        if not self.moves:
            return
        if p.mode == "dense":
            st = p.stride
            for q in range(self.world):
                if q != p.rank:
                    out += back[q * st: q * st + p.n_loc]
            return
        off = 0
        for cnt in p.send_counts:  # indices unique within a peer -> deterministic
            if cnt:
                out.index_add_(0, p.send_index[off:off + cnt], back[off:off + cnt])
            off += cnt

    def backward(self, dZ: torch.Tensor, dropedge: Optional[DropEdge] = None, backward_slice=None) -> torch.Tensor:
        """dX_loc = the shard's share of A_drop^T dZ, with the reverse halo
        exchange overlapped with the gather: slice c's halo-row gradients
        travel home (RCCL all-to-all, async on the collective's own stream)
        while the compute stream gathers slice c+1 with
        grl_typed_spmm_bwd_slice; the owner then adds the peers' partials in
        peer order.  Per element the same operations as the unsliced
        exchange + spmm_backward: bitwise equal to it.
        backward_slice(dZ, graph, col0, out) replaces the HIP slice gather
        (CPU tests only)."""
        from .ops import spmm_backward_slice

        gather = backward_slice or spmm_backward_slice
        graph = self.sg.graph.with_dropedge(dropedge)
        dZ = dZ.contiguous()
        gt, _ = self._grad_buffers(dZ.device)
        dX_loc = torch.empty(self.plan.n_loc, self.F, dtype=dZ.dtype, device=dZ.device)
        if self.side is None:  # host-staged (gloo) or single rank: in order, no overlap
            for c in range(self.K):
                gather(dZ, graph, c * self.Fc, gt[c])
                self._exchange_back(c, async_op=False)
                self._combine(c, dX_loc)
            return dX_loc
        works = []
        for c in range(self.K):
            gather(dZ, graph, c * self.Fc, gt[c])
            works.append(self._exchange_back(c, async_op=True))  # waits for slice c's gather only
        for c in range(self.K):
            if works[c] is not None:
                works[c].wait()  # the compute stream waits for slice c's exchange only
            self._combine(c, dX_loc)
        return dX_loc


class _PipelinedAggregate(torch.autograd.Function):
    """Z = A_drop X_ext of a shard with both halo exchanges pipelined over
    column slices (HaloPipeline.run forward, HaloPipeline.backward)."""

    @staticmethod
    def forward(ctx, X_loc: torch.Tensor, pipe: "HaloPipeline", dropedge):
        with trace("grl.halo_pipeline_fwd"):
            Z = X_loc.new_empty(pipe.plan.n_loc, pipe.sg.graph.segments * pipe.F)
            pipe.run(X_loc.detach().contiguous(), Z, dropedge)
        ctx.pipe, ctx.dropedge = pipe, dropedge
        return Z

    @staticmethod
    def backward(ctx, dZ: torch.Tensor):
        with trace("grl.halo_pipeline_bwd"):
            return ctx.pipe.backward(dZ, ctx.dropedge), None, None


def _p2p_exchange(sends, recvs, group):
    """Post point-to-point transfers: sends [(tensor, dst)], recvs [(tensor,
    src)], peers given as ranks OF `group` (P2POp's group_peer: a subgroup's
    rank q is not global rank q).  RCCL: one batch_isend_irecv, asynchronous
    (the transfer waits for the work queued on the current stream); a send
    to this rank itself pairs with a receive from it (a loopback plan).
    Returns the works and a finish() that copies host-staged receives back
    (gloo moves device tensors through host copies)."""
    if not sends and not recvs:
        return [], lambda: None
    staged = _host_staged(group)
    snd, rcv, back = [], [], []
    for t, dst in sends:
        snd.append((t.cpu() if staged and t.is_cuda else t, dst))
    for t, src in recvs:
        buf = torch.empty(t.shape, dtype=t.dtype) if staged and t.is_cuda else t
        if buf is not t:
            back.append((t, buf))
        rcv.append((buf, src))
    works = _c_p2p(snd, rcv, group)

    def finish():
        for t, buf in back:
            t.copy_(buf)

    return works, finish


def _all_agree(flag: bool, group, device) -> bool:
    """True iff `flag` holds on every rank of `group` (a MIN all-reduce): a
    decision that picks between two different collective sequences must be
    the same on every rank, or the ranks post mismatched collectives and
    hang.  Runs on any communicating group, a one-rank one included."""
    if not _comm_on(group):
        return flag
    t = torch.tensor([1 if flag else 0], dtype=torch.int32,
                     device="cpu" if _host_staged(group) or device is None else device)
    _c_all_reduce(t, dist.ReduceOp.MIN, group)
    return bool(int(t.item()))


def stream_chunks(stride: int, n_loc: int, blocks: int, path_ok):
    """The streamed inference layer's schedule (ShardedGraph._graphconv_streamed):
    [(r0, r1, posts)] -- compute rows [r0, r1) of the shard, then post the
    row blocks `posts` ([a0, a1) of the padded own block; the same blocks,
    in the same order, on every rank: `blocks` equal parts of `stride`).
    A compute chunk is a run of whole blocks that takes the same GEMM path as
    the whole shard (path_ok(rows): ops.x6_rows_ok), so the layer's bits do
    not depend on the blocking; when the whole shard fails path_ok it is one
    chunk (the unstreamed layer), its blocks posted after it."""
    nb = max(1, int(blocks))
    bs = -(-stride // nb)
    parts = [(j * bs, min((j + 1) * bs, stride)) for j in range(nb) if j * bs < stride]
    whole_ok = n_loc > 0 and path_ok(n_loc)
    out, start, held = [], 0, []
    for j, (a0, a1) in enumerate(parts):
        held.append((a0, a1))
        e = min(a1, n_loc)
        if j + 1 < len(parts):
            if not (whole_ok and e > start and path_ok(e - start) and (e == n_loc or path_ok(n_loc - e))):
                continue
        else:
            e = n_loc
        out.append((start, e, held))
        start, held = e, []
    return out


class _Landing:
    """A collective's handle whose wait() also lands the received rows where
    they belong (a stream-ordered copy after the collective)."""

    def __init__(self, work, land, keep):
        self.work, self.land, self.keep = work, land, keep

    def wait(self):
        if self.work is not None:
            self.work.wait()
            self.work = None
            self.land()
            self.keep = None


class _RowPipelinedGraphConv(torch.autograd.Function):
    """One GraphConv layer (robust_gcn.py:45-51) on a node-range shard with
    the one-kernel forms in both directions and the reverse halo exchange
    pipelined over ROW blocks (ShardedGraph.graphconv(pipeline="rows")).

    forward:  the halo exchange (every slot), then the one-kernel training
              forward over [own | halo] rows (grl_graphconv_fwd_train: out,
              and Z for dW) -- out bitwise the one-GPU rows.
    backward: dW, db from Z (partials: allreduce_gradients completes them);
              dX_ext = the one-kernel data gradient over the shard's typed
              transpose computed in row blocks -- peer q's halo rows for
              q = rank+1, rank+2, ... first, each block's partials posted to
              q (RCCL point-to-point, asynchronous) while the next block
              computes, the own rows last -- and the owner adds the peers'
              partials in peer order, as the unpipelined exchange does: dX
              bitwise the unpipelined one-kernel sharded layer's.
    ER shards reference nearly every remote row, so no forward overlap exists
    that keeps out's per-element summation order (a row's sum needs all its
    sources); the column-slice pipeline (chunks=k) overlaps the forward
    exchange but runs the two-kernel layer."""

    @staticmethod
    def forward(ctx, X_loc: torch.Tensor, sg: "ShardedGraph", W: torch.Tensor, b, relu: bool, dropedge,
                fdrop=None, stream: bool = False):
        from .ops import feature_dropout_apply, graph_conv_fwd_train

        with trace("grl.rows_pipeline_fwd"):
            X_ext = sg.exchange_table(X_loc)
            graph = sg.graph.with_dropedge(dropedge)
            Wc, bc = W.contiguous(), b.contiguous() if b is not None else None
            row0 = sg.plan.row_begin
            if stream:  # the output streamed to the peers by row blocks as it is written (training forward)
                out, D, Z = sg._graphconv_train_streamed(X_ext, graph, Wc, bc, relu, fdrop)
            else:
                out, Z = graph_conv_fwd_train(X_ext, graph, Wc, bc, relu)
                D = out if fdrop is None else feature_dropout_apply(out, fdrop, row0)
        ctx.sg, ctx.graph, ctx.relu, ctx.has_b, ctx.F = sg, graph, relu, b is not None, X_loc.shape[1]
        ctx.fdrop, ctx.row0 = fdrop, row0
        ctx.save_for_backward(Z, Wc, out if relu else None)
        return D

    @staticmethod
    def backward(ctx, g: torch.Tensor):
        from .ops import feature_dropout_apply, graph_conv_bwd_data, linear_bwd_weight, relu_grad

        Z, W, out = ctx.saved_tensors
        sg, graph, F = ctx.sg, ctx.graph, ctx.F
        g = g.contiguous().float()
        if ctx.fdrop is not None:  # the fused feature dropout's backward: the same mask on the gradient
            g = feature_dropout_apply(g, ctx.fdrop, ctx.row0)
        # the ReLU handling of ops._GraphConv.backward (same kernels, same bits)
        want_w, want_b = ctx.needs_input_grad[2], ctx.has_b and ctx.needs_input_grad[3]
        g, mask, db_pre = relu_grad(g, out if ctx.relu else None, want_b)
        dW = db = None
        if want_w or (want_b and db_pre is None):
            dW, db = linear_bwd_weight(Z, g, mask, want_b and db_pre is None)
        if db_pre is not None:
            db = db_pre
        dX_loc = None
        if ctx.needs_input_grad[0]:
            g_data = g if mask is None else torch.where(mask > 0, g, torch.zeros((), dtype=g.dtype, device=g.device))
            with trace("grl.rows_pipeline_bwd"):
                dX_loc = sg.rows_backward(g_data, W, F, graph)
            if dX_loc is None:  # a block outside the one-kernel path: whole range, then the exchange
                dX_ext = graph_conv_bwd_data(g_data, graph, W, F)
                if dX_ext is None:
                    from .ops import linear_bwd_data, spmm_backward

                    dX_ext = spmm_backward(linear_bwd_data(g_data, None, W), graph, F)
                dX_loc = _HaloExchange.backward(types_ns(plan=sg.plan, group=sg.group), dX_ext)[0]
        return dX_loc, None, dW if want_w else None, db, None, None, None, None


def types_ns(**kw):
    import types

    return types.SimpleNamespace(**kw)


def broadcast_module(module: torch.nn.Module, src: int = 0, group=None) -> None:
    """Copy `src`'s parameters and buffers to every rank (replica start)."""
    if _world(group) == 1:
        return
    src_in_group = src if _local(group) or group is None else dist.get_group_rank(group, src)
    for t in list(module.parameters()) + list(module.buffers()):
        if _host_staged(group) and t.is_cuda:
            h = t.detach().cpu()
            _c_broadcast(h, src_in_group, group)
            t.data.copy_(h)
        else:
            _c_broadcast(t.data, src_in_group, group)


def allreduce_gradients(params, group=None, bucket_bytes: int = 64 << 20, average: bool = False,
                        check: bool = True) -> None:
    """Sum the .grad of `params` over the ranks of `group` in place.

    With node-range shards every rank's weight gradient of a GraphConv
    (dW = Z_r^T g_r, db = colsum g_r) is a partial sum over its own rows, so
    one all_reduce per step completes it (1.8 MB for gcn1 at
    d=256).  Gradients are packed into flat fp32 buckets of <= bucket_bytes
    (one RCCL call each; all of GraphCNNDropEdge's fit one bucket).
    average=True divides by the world size (data parallelism's mean).
    Without a process group nothing runs; a one-rank group runs the real
    collectives (a sum over one rank: the gradients unchanged).
    check: then surface a persistent kernel's stream-ordered failure of this
    step (grl_check, which waits for the stream) before any optimizer step
    reads the gradients: the sharded training step's sync point."""
    if not _comm_on(group):
        return
    grads = [p.grad for p in params if p.grad is not None]
    bucket: List[torch.Tensor] = []
    size = 0

    def flush():
        nonlocal bucket, size
        if not bucket:
            return
        flat = torch.cat([g.reshape(-1) for g in bucket])
        if average:
            flat.div_(_world(group))
        if _host_staged(group) and flat.is_cuda:
            h = flat.cpu()
            _c_all_reduce(h, dist.ReduceOp.SUM, group)
            flat.copy_(h)
        else:
            _c_all_reduce(flat, dist.ReduceOp.SUM, group)
        off = 0
        for g in bucket:
            g.copy_(flat[off:off + g.numel()].view_as(g))
            off += g.numel()
        bucket, size = [], 0

    for g in grads:
        if bucket and (g.dtype != bucket[0].dtype or g.device != bucket[0].device
                       or size + g.numel() * g.element_size() > bucket_bytes):
            flush()
        bucket.append(g)
        size += g.numel() * g.element_size()
    flush()
    if check and grads and grads[0].is_cuda:
        from .graph import device_check

        device_check(grads[0].device)


def edge_balanced_bounds(deg: torch.Tensor, world: int) -> List[int]:
    """Node-range boundaries [b_0=0, ..., b_P=N] such that rank r's range
    holds ~r/P of the edges (every rank computes the same bounds from the
    same deterministic degree histogram, no communication)."""
    cum = torch.cumsum(deg.to(torch.int64), 0)
    total = int(cum[-1]) if cum.numel() else 0
    targets = torch.tensor([total * r // world for r in range(1, world)], dtype=torch.int64, device=deg.device)
    inner = (torch.searchsorted(cum, targets, right=False) + 1).cpu().tolist()
    n = deg.numel()
    bounds = [0] + [min(n, max(b, 0)) for b in inner] + [n]
    for i in range(1, len(bounds)):  # monotone
        bounds[i] = max(bounds[i], bounds[i - 1])
    return bounds


class ShardedGraph:
    """This rank's node-range shard of a global typed graph, ready to aggregate."""

    def __init__(self, rowptr: torch.Tensor, colidx_global: torch.Tensor, num_types: int, row_begin: int,
                 row_end: int, *, vals: Optional[torch.Tensor] = None, group=None, halo: str = "auto"):
        self._init(rowptr, build_halo_plan(colidx_global, row_begin, row_end, group, mode=halo), num_types, vals,
                   group)

    dropedge: Optional[DropEdge] = None  # the edge_dropout draw this view carries (with_dropedge)

    def _init(self, rowptr, plan: HaloPlan, num_types: int, vals, group):
        self.group, self.plan = group, plan
        p = plan
        self.graph = TypedGraph(rowptr, p.colidx_local, num_types, vals=vals, has_self=True,
                                num_cols=p.n_loc + p.n_halo, edge_id_base=p.edge_id_base,
                                self_id_base=p.num_edges_total + p.row_begin, self_rows=p.n_loc)
        # the GEMM path of every layer is chosen for the whole graph's rows: a shard's rows are bitwise the
        # one-GPU layer's (GrlTypedCsr.path_rows)
        self.graph.path_rows = self.global_rows

    @staticmethod
    def cache_key(graph: TypedGraph, **kw):
        """A BUCKET key for `graph`'s structure (rows, types, edges and
        position-weighted checksums of rowptr, colidx and the bits of vals)
        plus the sharding options: every rank computes the same key from the
        same graph, so a procedure that meets one large graph step after step
        reuses its shard plan instead of rebuilding it (from_graph exchanges
        index lists).  Two graphs can still share a key; a cache hit must be
        confirmed with same_graph (sharded_graph_cached does)."""
        L = graph.num_types
        dev = graph.colidx.device

        def wsum(t: torch.Tensor) -> int:  # sum_i t[i] * (2 i + 1) * golden, wrapped in int64
            t = t.reshape(-1).to(torch.int64)
            w = torch.arange(t.numel(), device=dev, dtype=torch.int64) * 2 + 1
            return int((t * w * 0x9E3779B1).sum())

        vbits = graph.vals.contiguous().view(torch.int32) if graph.vals is not None else None
        chk = (wsum(graph.rowptr), wsum(graph.colidx), wsum(vbits) if vbits is not None else 0)
        return (graph.num_rows, L, int(graph.colidx.numel()), chk, tuple(sorted(kw.items())))

    @staticmethod
    def same_graph(a: TypedGraph, b: TypedGraph) -> bool:
        """Exact equality of two graphs' CSR arrays (the confirmation of a
        cache_key hit: O(E) on the device, about the checksum's cost)."""
        if (a.num_rows, a.num_types, a.colidx.numel()) != (b.num_rows, b.num_types, b.colidx.numel()):
            return False
        if (a.vals is None) != (b.vals is None):
            return False
        return bool(torch.equal(a.rowptr, b.rowptr) and torch.equal(a.colidx, b.colidx)
                    and (a.vals is None or torch.equal(a.vals.contiguous().view(torch.int32),
                                                  b.vals.contiguous().view(torch.int32))))

    @property
    def global_rows(self) -> int:
        """Rows of the whole graph this shard belongs to."""
        return self.plan.bounds[-1] - self.plan.bounds[0]

    @classmethod
    def in_process(cls, graph: TypedGraph, bounds: List[int], halo: str = "auto",
                   group: Optional[LocalGroup] = None) -> List["ShardedGraph"]:
        """All P node-range shards of `graph` in this process: shard r is what
        ShardedGraph.from_graph builds on rank r of a P-rank group with these
        bounds.  For driving several shards from one process: group, a
        LocalGroup of P virtual ranks (shard r communicates as its member r,
        each driven by its own thread), or None (the exchanges then go
        through a HaloPipeline `exchange` object)."""
        if group is not None and group.world != len(bounds) - 1:
            raise ValueError(f"a LocalGroup of {group.world} ranks for {len(bounds) - 1} node ranges")
        L = graph.num_types
        parts = []
        for r in range(len(bounds) - 1):
            e0, e1 = int(graph.rowptr[bounds[r] * L]), int(graph.rowptr[bounds[r + 1] * L])
            parts.append(((graph.rowptr[bounds[r] * L: bounds[r + 1] * L + 1] - e0).contiguous(),
                          graph.colidx[e0:e1], None if graph.vals is None else graph.vals[e0:e1]))
        plans = build_halo_plans_local([c for _, c, _ in parts], bounds, mode=halo)
        out = []
        for (rowptr, _, vals), plan in zip(parts, plans):
            sg = cls.__new__(cls)
            sg._init(rowptr, plan, L, vals, None if group is None else group.member(len(out)))
            sg.graph.split_threshold, sg.graph.split_chunk = graph.split_threshold, graph.split_chunk
            out.append(sg)
        return out

    @classmethod
    def synthetic(cls, num_nodes: int, avg_deg: float, num_types: int = 6, *, kind: str = "er", seed: int = 0,
                  device="cuda", group=None, balance: Optional[str] = None, halo: str = "auto") -> "ShardedGraph":
        """balance "nodes": equal node ranges (ER); "edges": ranges holding
        ~E/P candidate edges each (power-law graphs; default for R-MAT)."""
        world, rank = _world(group), _rank(group)
        balance = balance or ("edges" if kind == "rmat" else "nodes")
        if balance == "edges" and world > 1:
            deg = TypedGraph.synthetic_degrees(num_nodes, avg_deg, num_types, kind=kind, seed=seed, device=device)
            bounds = edge_balanced_bounds(deg, world)
        else:
            per = -(-num_nodes // world)
            bounds = [min(num_nodes, r * per) for r in range(world + 1)]
        rb, re = bounds[rank], bounds[rank + 1]
        g = TypedGraph.synthetic(num_nodes, avg_deg, num_types, kind=kind, seed=seed, row_range=(rb, re),
                                 device=device)
        return cls(g.rowptr, g.colidx, num_types, rb, re, group=group, halo=halo)

    @classmethod
    def from_graph(cls, graph: TypedGraph, *, group=None, balance: str = "edges", halo: str = "auto") -> "ShardedGraph":
        """This rank's node-range shard of a global typed graph every rank
        holds (e.g. a generated graph after grl.graph.degree_order: C5's
        528M-edge CSR is 2.3 GB, small next to its 17 GB of features).
        balance "edges": ranges holding ~E/P edges each; "nodes": equal ranges."""
        if graph.num_cols != graph.num_rows:
            raise ValueError("from_graph needs a square graph (rows and sources are the same nodes)")
        world, rank = _world(group), _rank(group)
        L, n = graph.num_types, graph.num_rows
        if balance == "edges":
            bounds = edge_balanced_bounds((graph.rowptr[L::L] - graph.rowptr[:-1:L]).to(torch.int64), world)
        else:
            per = -(-n // world)
            bounds = [min(n, r * per) for r in range(world + 1)]
        rb, re = bounds[rank], bounds[rank + 1]
        e0, e1 = int(graph.rowptr[rb * L]), int(graph.rowptr[re * L])
        sg = cls((graph.rowptr[rb * L: re * L + 1] - e0).contiguous(), graph.colidx[e0:e1], L, rb, re,
                 vals=None if graph.vals is None else graph.vals[e0:e1], group=group, halo=halo)
        sg.graph.split_threshold, sg.graph.split_chunk = graph.split_threshold, graph.split_chunk
        return sg

    @property
    def halo_rows(self) -> int:
        return self.plan.n_halo

    @property
    def device(self) -> torch.device:
        return self.graph.device

    def with_dropedge(self, de: Optional[DropEdge]) -> "ShardedGraph":
        """Shallow copy carrying a DropEdge draw (shares the plan, the local
        graph and its caches): the sharded counterpart of
        TypedGraph.with_dropedge, i.e. the reference's edge_dropout(A).  The
        draw's edge ids are global, so every rank masks its edges exactly as
        the one-GPU graph would."""
        sg = ShardedGraph.__new__(ShardedGraph)
        sg.__dict__.update(self.__dict__)
        sg.dropedge = de
        return sg

    def gather_rows(self, X_loc: torch.Tensor) -> torch.Tensor:
        """Every rank's rows of a node-range-sharded [n_loc, d] tensor, in
        global node order ([N, d]): one all-gather of shards padded to the
        largest one (no autograd)."""
        p = self.plan
        world = len(p.bounds) - 1
        if not _comm_on(self.group):  # (a one-rank group still runs the collective)
            return X_loc
        stride = max(p.bounds[q + 1] - p.bounds[q] for q in range(world))
        X_loc = X_loc.reshape(-1, X_loc.shape[-1])
        pad = X_loc.new_zeros(stride, X_loc.shape[1])
        pad[: X_loc.shape[0]] = X_loc
        out = X_loc.new_empty(world * stride, X_loc.shape[1])
        all_gather_into(out, pad, self.group)
        return torch.cat([out[q * stride: q * stride + p.bounds[q + 1] - p.bounds[q]] for q in range(world)])

    def reduce_rows(self, P: torch.Tensor) -> torch.Tensor:
        """This rank's rows of the sum over ranks of a per-rank [N, d] partial
        (global node order), added in rank order: every rank sends each peer
        that peer's row block (all-to-all-v) and adds the P blocks it receives
        in rank order -- deterministic, the bits independent of the
        collective's algorithm."""
        p = self.plan
        world = len(p.bounds) - 1
        if not _comm_on(self.group):  # (a one-rank group still runs the collective)
            return P.contiguous()
        sizes = [p.bounds[q + 1] - p.bounds[q] for q in range(world)]
        recv = P.new_empty(world * p.n_loc, P.shape[1])
        all_to_all_v(recv, P.contiguous(), [p.n_loc] * world, sizes, self.group)
        acc = recv[: p.n_loc].clone()
        for q in range(1, world):
            acc += recv[q * p.n_loc: (q + 1) * p.n_loc]
        return acc

    def broadcast_seed(self, seed_t: torch.Tensor) -> torch.Tensor:
        """Rank 0's value of a 1-element device tensor on every rank of the
        shard's group (a device-drawn DropEdge seed: the masks of a sharded
        graph must be the one-GPU graph's on every rank)."""
        if not _comm_on(self.group):
            return seed_t
        if _host_staged(self.group):
            h = seed_t.cpu()
            _c_broadcast(h, 0, self.group)
            seed_t.copy_(h)
        else:
            _c_broadcast(seed_t, 0, self.group)
        return seed_t

    def exchange(self, X_loc: torch.Tensor) -> torch.Tensor:
        return halo_exchange(X_loc, self.plan, self.group)

    # ---- halo tables reused within one forward (GraphCNNDropEdge: gcn3's
    # input is cat[g1, g2] and g1's table was exchanged for gcn2) ----
    halo_memo: Optional[dict] = None

    def with_halo_memo(self) -> "ShardedGraph":
        """Shallow copy (like with_dropedge; its own copies share the memo)
        whose exchanges consult a per-forward memo: remember(X) keeps X's
        table once exchanged, note_concat(X, parts) lets a column concat of
        remembered tensors be assembled from their tables (only the parts
        not yet exchanged travel).  Same rows, same values as exchanging the
        concat itself, so every layer's output keeps its bits."""
        sg = ShardedGraph.__new__(ShardedGraph)
        sg.__dict__.update(self.__dict__)
        sg.halo_memo = {"keep": {}, "tables": {}, "concat": {}, "pending": {}}
        return sg

    @staticmethod
    def _tkey(X: torch.Tensor):
        """Identity of a contiguous tensor's [rows, cols] view (a (B, n, F)
        tensor and its 2-D view are one key); None for other layouts."""
        if not X.is_contiguous() or X.dim() == 0:
            return None
        return (X.data_ptr(), X._version, X.numel() // max(X.shape[-1], 1), X.shape[-1], X.dtype)

    def remember(self, X: torch.Tensor) -> None:
        k = self._tkey(X)
        if self.halo_memo is not None and k is not None:
            self.halo_memo["keep"][k] = X  # the reference keeps X's storage from being reused

    def note_concat(self, X: torch.Tensor, parts) -> None:
        k = self._tkey(X)
        if self.halo_memo is not None and k is not None:
            self.halo_memo["concat"][k] = (X, list(parts))

    def clear_halo_memo(self) -> None:
        if self.halo_memo is not None:
            for _, works, _ in self.halo_memo["pending"].values():  # tables still being filled: finish first
                for w in works:
                    if w is not None:
                        w.wait()
            for d in self.halo_memo.values():
                d.clear()

    # ---- inference: each layer's output streamed to the peers by row blocks ----
    stream_rows = True   # under a memo (the drop-in model's forward): see _graphconv_streamed
    stream_blocks = 2

    def without_streaming(self) -> "ShardedGraph":
        """Shallow copy (the memo shared) whose GraphConv does not stream its
        output: for a layer whose output no later GraphConv reads (the
        model's gcn3), whose rows would travel for nothing."""
        sg = ShardedGraph.__new__(ShardedGraph)
        sg.__dict__.update(self.__dict__)
        sg.stream_rows = False
        return sg

    def _can_stream(self, X_loc: torch.Tensor) -> bool:
        p = self.plan
        # peers, or a one-rank loopback plan whose sources all come through the exchange (tests/rccl_loopback.py)
        return bool(self.stream_rows and self.halo_memo is not None and (len(p.bounds) > 2 or p.n_halo > 0)
                    and _comm_on(self.group) and X_loc.is_cuda)

    def _stream_extent(self) -> int:
        """Rows of the uniform block grid: the largest shard (every rank
        posts the same blocks, so each collective matches)."""
        b = self.plan.bounds
        return max(b[q + 1] - b[q] for q in range(len(b) - 1))

    def _stream_table(self, C: int, like: torch.Tensor) -> torch.Tensor:
        """The next layer's X_ext, to be filled by blocks: the dense layout
        [own | pad | P slots] (pad rows zero) or the sparse [own | halo]."""
        p, world = self.plan, len(self.plan.bounds) - 1
        if p.mode == "dense":
            T = like.new_empty(p.stride * (1 + world), C)
            T[p.n_loc:p.stride].zero_()
        else:
            T = like.new_empty(p.n_loc + p.n_halo, C)
        return T

    def _sparse_block_lists(self, a0: int, a1: int):
        """Sparse halos, block [a0, a1) of every rank's own rows: (rows of my
        block the peers asked for, concatenated per peer; per-peer send
        counts; per-peer receive counts; the X_ext rows the received rows go
        to).  Cached per block; one host read when built."""
        cache = self.__dict__.setdefault("_stream_lists", {})
        if (a0, a1) in cache:
            return cache[(a0, a1)]
        p, world = self.plan, len(self.plan.bounds) - 1
        dev = p.send_index.device
        send_idx, send_counts, recv_counts, dest = [], [], [], []
        off = roff = 0
        for q in range(world):
            seg = p.send_index[off:off + p.send_counts[q]]  # ascending: the peer's halo ids are
            lo, hi = (int(x) for x in torch.searchsorted(seg, torch.tensor([a0, a1], device=dev)).tolist())
            send_idx.append(seg[lo:hi])
            send_counts.append(hi - lo)
            off += p.send_counts[q]
            ids = p.halo_ids[roff:roff + p.recv_counts[q]] - p.bounds[q]  # owner q's rows I read, ascending
            lo, hi = (int(x) for x in torch.searchsorted(ids, torch.tensor([a0, a1], device=ids.device)).tolist())
            dest.append(torch.arange(p.n_loc + roff + lo, p.n_loc + roff + hi, device=dev))
            recv_counts.append(hi - lo)
            roff += p.recv_counts[q]
        cache[(a0, a1)] = out = (torch.cat(send_idx), send_counts, recv_counts, torch.cat(dest))
        return out

    def _post_block(self, T: torch.Tensor, a0: int, a1: int):
        """Rows [a0, a1) of every rank's own block into every peer's table T:
        dense halos, one all-gather of the padded block into the P slots;
        sparse halos, one all-to-all-v of the rows each peer asked for (their
        slots in T written when the handle is waited on).  Asynchronous on
        RCCL (the next blocks compute meanwhile); host-staged and synchronous
        on gloo.  Returns a handle with wait(), or None when done."""
        p, world = self.plan, len(self.plan.bounds) - 1
        if p.mode == "dense":
            a1 = min(a1, p.stride)
            slots = [T[p.stride * (1 + q) + a0: p.stride * (1 + q) + a1] for q in range(world)]
            if _host_staged(self.group):
                h = T[a0:a1].cpu()
                outs = [torch.empty_like(h) for _ in range(world)]
                _c_all_gather(outs, h, self.group)
                for v, o in zip(slots, outs):
                    v.copy_(o)
                return None
            return _c_all_gather(slots, T[a0:a1], self.group, async_op=True)
        send_idx, sc, rc, dest = self._sparse_block_lists(a0, a1)
        send = T.index_select(0, send_idx)
        recv = T.new_empty(sum(rc), T.shape[1])
        if _host_staged(self.group):
            all_to_all_v(recv, send, rc, sc, self.group)
            T.index_copy_(0, dest, recv)
            return None
        work = _c_all_to_all_single(recv, send, rc, sc, self.group, async_op=True)
        return _Landing(work, lambda: T.index_copy_(0, dest, recv), (send, recv))

    def _stream_fill(self, T: torch.Tensor, C: int, K: int, compute) -> list:
        """Fill T's own rows by compute(r0, r1) (writing T[r0:r1]) in the
        stream_chunks schedule, posting each block as soon as its rows are
        written; returns the handles."""
        from .ops import x6_rows_ok

        works = []
        pr = self.global_rows
        for r0, r1, posts in stream_chunks(self._stream_extent(), self.plan.n_loc, int(self.stream_blocks),
                                           lambda m: x6_rows_ok(m, C, K, pr)):
            if r1 > r0:
                compute(r0, r1)
            works += [self._post_block(T, a0, a1) for a0, a1 in posts]
        return works

    def _graphconv_streamed(self, X_loc: torch.Tensor, layer, dropedge, relu: bool) -> torch.Tensor:
        """Inference GraphConv whose output rows go to the peers while the
        rest of the layer computes: the output is written straight into the
        NEXT layer's halo table T (the plan's X_ext layout) in stream_blocks
        row blocks (one-kernel forward over row-range views of the shard
        graph, TypedGraph.rows_view -- every row the whole shard's
        arithmetic), each block sent to the peers as soon as it is written
        (_post_block).  The next layer finds T through the memo
        (exchange_table waits for the blocks' collectives) instead of
        exchanging its input.  The output is T's own rows, bitwise the
        unstreamed layer's: blocks are computed in runs that take the same
        GEMM path as the whole shard (x6_rows_ok), a shard too small for the
        split-bf16 GEMM in one call (its fp32 linear splits K by rows)."""
        from .ops import graph_conv_infer

        p = self.plan
        X_ext = self.exchange_table(X_loc)
        W, b = layer.h_weights, layer.bias
        C = W.shape[1]
        T = self._stream_table(C, X_ext)
        assert T.shape[0] == self.graph.num_cols, "T is the next layer's X_ext"
        g = self.graph.with_dropedge(dropedge)
        works = self._stream_fill(T, C, g.segments * X_ext.shape[1],
                                  lambda r0, r1: graph_conv_infer(X_ext, g.rows_view(r0, r1), W, b, relu,
                                                                  out=T[r0:r1]))
        out = T[:p.n_loc]
        k = self._tkey(out)
        self.halo_memo["pending"][k[:1] + k[2:]] = (T, works, out)
        return out

    def _graphconv_train_streamed(self, X_ext: torch.Tensor, graph: TypedGraph, W: torch.Tensor, b, relu: bool,
                                  fdrop):
        """Training forward of a GraphConv whose output (through the feature
        dropout that follows it in the model, fused: drop_robust_gcn.py:77,
        81) goes to the peers while the rest of the layer computes.  Row
        blocks [r0, r1) of the shard run the one-kernel training forward over
        row-range views (out and Z rows, the whole shard's arithmetic: the
        GEMM path is pinned by path_rows); each block's dropout mask is the
        hash of its global element ids (feature_dropout), so the block is
        final as soon as it is written: D[r0:r1] = dropout(out[r0:r1]) is
        copied into the NEXT layer's halo table T and posted (_post_block),
        exactly as streamed inference does.  Returns (out, D, Z): the ReLU
        output (the backward's mask), the layer's output D (its own storage,
        not a view of T, whose halo rows the collectives write in place: a
        view would tie the autograd output to those writes) and Z."""
        from .ops import feature_dropout_apply, graph_conv_fwd_train

        p = self.plan
        C = W.shape[1]
        K = graph.segments * X_ext.shape[1]
        out = X_ext.new_empty(p.n_loc, C)
        Z = X_ext.new_empty(p.n_loc, K)
        D = X_ext.new_empty(p.n_loc, C) if fdrop is not None else out
        T = self._stream_table(C, X_ext)

        def compute(r0, r1):
            graph_conv_fwd_train(X_ext, graph.rows_view(r0, r1), W, b, relu, out=out[r0:r1], Z=Z[r0:r1])
            if fdrop is not None:
                feature_dropout_apply(out[r0:r1], fdrop, p.row_begin + r0, out=D[r0:r1])
            T[r0:r1].copy_(D[r0:r1])

        works = self._stream_fill(T, C, K, compute)
        k = self._tkey(D)
        self.halo_memo["pending"][k[:1] + k[2:]] = (T, works, D)
        return out, D, Z

    def exchange_table(self, X_loc: torch.Tensor) -> torch.Tensor:
        """X_ext = [own | halo] rows of X_loc without autograd (the layers'
        backward sends the halo gradients home themselves), through the memo
        when one is attached."""
        X_loc = X_loc.detach()
        X_loc = X_loc.reshape(-1, X_loc.shape[-1])
        memo = self.halo_memo
        if memo is None:
            with torch.no_grad():
                return halo_exchange(X_loc.contiguous(), self.plan, self.group)
        k = self._tkey(X_loc)
        if k is None:
            with torch.no_grad():
                return halo_exchange(X_loc.contiguous(), self.plan, self.group)
        hit = memo["tables"].get(k)
        if hit is not None:
            return hit
        pend = memo["pending"].pop(k[:1] + k[2:], None)  # a streamed layer's output (its version may have moved)
        if pend is not None and pend[2].data_ptr() == X_loc.data_ptr():
            T, works, _ = pend
            for w in works:
                if w is not None:
                    w.wait()
            # landing the received rows (T.index_copy_) bumped the version X shares with T: re-key
            k1 = self._tkey(X_loc)
            if k in memo["keep"]:
                memo["keep"][k1] = memo["keep"].pop(k)
                memo["tables"][k1] = T
            return T
        cat = memo["concat"].get(k)
        if cat is not None:
            return torch.cat([self.exchange_table(part.reshape(-1, part.shape[-1])) for part in cat[1]], dim=1)
        with torch.no_grad():
            X_ext = halo_exchange(X_loc.contiguous(), self.plan, self.group)
        if k in memo["keep"]:
            memo["tables"][k] = X_ext
        return X_ext

    def pipeline(self, F: int, chunks: int) -> HaloPipeline:
        """The HaloPipeline of this shard for F-wide features in `chunks`
        column slices (built once, buffers reused by every call)."""
        cache = self.__dict__.setdefault("_pipelines", {})
        key = (F, chunks)
        if key not in cache:
            cache[key] = HaloPipeline(self, F, chunks=chunks, device=self.graph.device)
        return cache[key]

    def aggregate(self, X_loc: torch.Tensor, dropedge: Optional[DropEdge] = None,
                  chunks: Optional[int] = None) -> torch.Tensor:
        """Z rows of this shard: halo exchange + typed SpMM (autograd through
        both).  chunks=k pipelines both exchanges with the gathers over k
        column slices (forward HaloPipeline.run, backward
        HaloPipeline.backward); same bits as chunks=None."""
        if chunks is None:
            return typed_aggregate(self.exchange(X_loc), self.graph.with_dropedge(dropedge))
        return _PipelinedAggregate.apply(X_loc, self.pipeline(X_loc.shape[1], chunks), dropedge)

    def halo_blocks(self):
        """[(peer q, r0, r1)]: the X_ext rows holding peer q's rows, for
        q = rank+1, rank+2, ... (mod P) -- the order rows_backward sends in.
        A loopback plan (a one-rank group whose sources all come through the
        exchange, tests/rccl_loopback.py) has one block, its own rows' copy."""
        p, world = self.plan, len(self.plan.bounds) - 1
        out = []
        for j in range(1, world + 1):
            q = (p.rank + j) % world
            if p.mode == "dense":
                if q == p.rank:
                    continue  # own rows: X_ext[:n_loc], not a gathered slot
                r0 = p.stride * (1 + q)
                out.append((q, r0, r0 + p.bounds[q + 1] - p.bounds[q]))
            else:
                if q == p.rank and p.recv_counts[q] == 0:
                    continue
                r0 = p.n_loc + sum(p.recv_counts[:q])
                out.append((q, r0, r0 + p.recv_counts[q]))
        return out

    def rows_backward(self, g: torch.Tensor, W: torch.Tensor, F: int, graph: TypedGraph):
        """dX_loc of a GraphConv layer on this shard (g: the output gradient
        through the ReLU): the one-kernel data gradient in row blocks, each
        peer's halo block posted to that peer as soon as it is computed, the
        own rows last, then the peers' partials for my rows added in peer
        order.  None -- on EVERY rank -- when a block of some rank is outside
        the one-kernel path: the ranks agree on the choice (one small
        all-reduce) before any point-to-point transfer is posted, since the
        fallback runs the unpipelined exchange, another collective sequence."""
        from .ops import graph_conv_bwd_data_rows, graph_conv_bwd_data_rows_views

        p, world = self.plan, len(self.plan.bounds) - 1
        dev = g.device
        blocks = self.halo_blocks()
        order = [(r0, r1) for _, r0, r1 in blocks] + [(0, p.n_loc)]
        views = graph_conv_bwd_data_rows_views(g, graph, W, F, order)
        # the ranks agree once per layer shape (the choice depends on static shapes and the plan only), not
        # in every backward: the all-reduce's host read would drain the launch queue
        agreed = self.graph._shared.setdefault("rows_backward_agreed", {})
        key = (F, tuple(g.shape), None if W is None else tuple(W.shape))
        if key not in agreed:
            agreed[key] = _all_agree(views is not None, self.group, dev)
        if not agreed[key]:
            return None
        if views is None:
            raise RuntimeError("rows_backward: the ranks agreed on the one-kernel path, but this rank's blocks "
                               "no longer qualify for it")
        dX_ext = torch.empty(graph.num_cols, F, dtype=torch.float32, device=dev)
        # receive buffers: the partials for my rows from the peer whose j-th block they are (src_j = rank - j;
        # dense: all my rows; sparse: the ones that peer referenced)
        srcs = [(p.rank - j) % world for j in range(1, len(blocks) + 1)]
        recv = {q: torch.empty(p.n_loc if p.mode == "dense" else p.send_counts[q], F, dtype=torch.float32,
                               device=dev) for q in srcs}
        pending = []
        step = {"j": 0}

        def post(r0, r1):
            step["j"] += 1
            j = step["j"]
            if j > len(blocks):
                return  # the own rows: nothing to send
            dst, src = blocks[j - 1][0], srcs[j - 1]
            sends = [(dX_ext[r0:r1], dst)] if r1 > r0 else []
            recvs = [(recv[src], src)] if recv[src].shape[0] else []
            pending.append(_p2p_exchange(sends, recvs, self.group))

        graph_conv_bwd_data_rows(g, graph, W, F, order, dX_ext, on_block=post, views=views)
        for works, finish in pending:
            for w in works:
                w.wait()
            finish()
        dX_loc = dX_ext[:p.n_loc].clone()
        off = 0
        for q in range(world):  # peer order: the unpipelined exchange's (_HaloExchange.backward)
            if q in recv:
                if p.mode == "dense":
                    dX_loc += recv[q]
                elif p.send_counts[q]:
                    cnt = p.send_counts[q]
                    dX_loc.index_add_(0, p.send_index[off:off + cnt], recv[q])
            off += p.send_counts[q] if p.mode != "dense" else 0
        return dX_loc

    def graphconv(self, X_loc: torch.Tensor, layer, dropedge: Optional[DropEdge] = None,
                  relu: bool = False, chunks: Optional[int] = None, pipeline: Optional[str] = None,
                  fdrop: Optional[DropEdge] = None) -> torch.Tensor:
        """One GraphConv (gnn.models.GraphConv or anything with h_weights /
        bias) over this shard: halo exchange -> typed SpMM -> MFMA linear
        (+ fused ReLU).  Output rows = this rank's nodes.  After backward,
        call allreduce_gradients(layer.parameters()) to complete dW / db.
        chunks: see aggregate.  Unpipelined (chunks=None), the layer after the
        exchange is grl.ops.graph_conv on [own | halo] rows: on large shards
        its forward is one kernel and its data gradient the one-kernel form
        over the shard's typed transpose, whose halo rows then travel home
        in the exchange's backward.  pipeline="rows": the one-kernel forms in
        both directions with the reverse exchange pipelined over row blocks
        (_RowPipelinedGraphConv); out and dX bitwise the unpipelined layer's.
        fdrop (pipeline="rows"): the feature dropout that follows the layer
        (drop_robust_gcn.py:77,81,86), fused into it; with a halo memo and
        peers the output is then streamed to them by row blocks as it is
        written (_graphconv_train_streamed), bitwise the unstreamed layer."""
        if dropedge is None:
            dropedge = self.dropedge
        if pipeline == "rows":
            return _RowPipelinedGraphConv.apply(X_loc, self, layer.h_weights, layer.bias, relu, dropedge, fdrop,
                                                self._can_stream(X_loc))
        if fdrop is not None:
            raise ValueError("fdrop (a fused feature dropout) needs pipeline='rows'")
        if pipeline is not None:
            raise ValueError(f"pipeline must be None or 'rows', got {pipeline!r}")
        if chunks is None:
            if not (torch.is_grad_enabled() and X_loc.requires_grad):  # no gradient to send home: memo table
                if self._can_stream(X_loc):
                    return self._graphconv_streamed(X_loc, layer, dropedge, relu)
                return graph_conv(self.exchange_table(X_loc), self.graph.with_dropedge(dropedge), layer.h_weights,
                                  layer.bias, relu=relu)
            return graph_conv(self.exchange(X_loc), self.graph.with_dropedge(dropedge), layer.h_weights, layer.bias,
                              relu=relu)
        Z = self.aggregate(X_loc, dropedge, chunks)
        return graph_linear(Z, layer.h_weights, layer.bias, relu=relu, path_rows=self.global_rows)


class _ShardedNodeAttention(torch.autograd.Function):
    """NodeSelfAtten (robust_gcn.py:78-99) over a node-range-sharded graph:
    out_loc = gamma * softmax(Q K^T) H + V for this rank's rows, the softmax
    over EVERY node.  Forward: K and H of every rank are all-gathered (RCCL)
    and the fused kernels run this rank's queries only against every key
    (grl_node_attention_fwd_rows): the O(N^2) work is split P ways.
    Backward (grl_node_attention_bwd_rows): dQ of the own queries is
    complete; dK and dH come out for every key as the own queries'
    contribution, and each key row's owner adds the P partials in rank
    order (an all-to-all of the row blocks, then an ordered sum:
    deterministic, unlike a reduce-scatter's); dgamma from the own rows
    (allreduce_gradients adds the ranks' partials, as for every weight)."""

    @staticmethod
    def forward(ctx, Q, K, H, V, gamma, sg):
        from .ops import node_attention_forward

        p = sg.plan
        dk, dv = Q.shape[-1], H.shape[-1]
        Kg = sg.gather_rows(K.detach().reshape(-1, dk).contiguous())
        Hg = sg.gather_rows(H.detach().reshape(-1, dv).contiguous())
        N = Kg.shape[0]
        r0 = p.row_begin - p.bounds[0] if N != p.n_loc else 0
        r1 = r0 + p.n_loc
        Qf = Q.new_zeros(1, N, dk)
        Qf[0, r0:r1] = Q.detach().reshape(-1, dk)
        Vf = V.new_zeros(1, N, dv)
        Vf[0, r0:r1] = V.detach().reshape(-1, dv)
        out, onorm, rmax, rsum = node_attention_forward(Qf, Kg[None], Hg[None], Vf, gamma, stats=True,
                                                        q_range=(r0, r1))
        ctx.rows, ctx.shapes, ctx.sg = (r0, r1), (Q.shape, K.shape, H.shape), sg
        ctx.save_for_backward(Qf, Kg, Hg, gamma, onorm, rmax, rsum)
        return out[0, r0:r1].reshape(V.shape)

    @staticmethod
    def backward(ctx, dout):
        from .ops import node_attention_backward

        Qf, Kg, Hg, gamma, onorm, rmax, rsum = ctx.saved_tensors
        r0, r1 = ctx.rows
        d_loc = dout.reshape(-1, dout.shape[-1]).contiguous().float()
        dOf = d_loc.new_zeros(1, Qf.shape[1], d_loc.shape[1])
        dOf[0, r0:r1] = d_loc
        dQ, dK, dH = node_attention_backward(Qf, Kg[None], Hg[None], gamma, onorm, rmax, rsum, dOf, q_range=(r0, r1))
        dgamma = (d_loc * onorm[0, r0:r1]).sum(0)
        dKH = ctx.sg.reduce_rows(torch.cat([dK[0], dH[0]], 1))
        dk = dK.shape[-1]
        qs, ks, hs = ctx.shapes
        return (dQ[0, r0:r1].reshape(qs), dKH[:, :dk].reshape(ks), dKH[:, dk:].reshape(hs), dout, dgamma, None)


def sharded_node_attention(Q: torch.Tensor, K: torch.Tensor, H: torch.Tensor, V: torch.Tensor, gamma: torch.Tensor,
                           sg: "ShardedGraph") -> torch.Tensor:
    """gamma * softmax_rows(Q K^T) H + V for this rank's rows of a sharded
    graph, the softmax over all nodes (_ShardedNodeAttention)."""
    return _ShardedNodeAttention.apply(Q, K, H, V, gamma, sg)
