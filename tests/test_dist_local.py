"""CPU: grl.dist.LocalGroup, the in-process stand-in for a P-rank process
group (P virtual ranks as threads of one process).

The sharded model's RCCL-side code -- async handles, slot views, landing
copies, peer-order combines -- runs on the GPU box with P > 1 only through
this group (RCCL refuses two ranks on one device), so its collectives are
pinned here against their torch.distributed definitions: all_gather,
all_gather_into_tensor, all_to_all_single with split sizes, all_reduce
(sum / min / max, added in rank order), broadcast, point-to-point sends
matched per (source, destination), mismatched collectives raising instead
of hanging -- and the module's halo exchange on CPU tensors filling X_ext
exactly as the plan says (the values the gloo tests check)."""
import threading

import pytest
import torch
import torch.distributed as dist

from grl import dist as gdist
from grl.dist import LocalGroup, build_halo_plans_local


def _run(world, fn, timeout=60):
    grp = LocalGroup(world, timeout=timeout)
    out, errs = [None] * world, [None] * world

    def body(r):
        try:
            out[r] = fn(grp.member(r))
        except BaseException as e:  # reported below; a failed rank must not hang the others
            errs[r] = e
            grp.abort()

    ts = [threading.Thread(target=body, args=(r,)) for r in range(world)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout + 10)
        assert not t.is_alive(), "virtual rank hung"
    for e in errs:
        if e is not None and not isinstance(e, threading.BrokenBarrierError):
            raise e
    for e in errs:
        if e is not None:
            raise e
    return out


@pytest.mark.parametrize("world", [1, 2, 3])
def test_collectives_match_their_definitions(world):
    def fn(m):
        r = m.rank
        x = torch.arange(4, dtype=torch.float32) + 10 * r
        outs = [torch.empty(4) for _ in range(world)]
        gdist._c_all_gather(outs, x, m)
        big = torch.empty(4 * world)
        gdist._c_all_gather_into_tensor(big, x, m)
        # rank r sends q + 1 rows to peer q (row values identify the sender and the row)
        in_splits = [q + 1 for q in range(world)]
        inp = torch.cat([torch.full((q + 1, 2), 100.0 * r + q) for q in range(world)])
        out_splits = [r + 1] * world
        recv = torch.empty(sum(out_splits), 2)
        gdist._c_all_to_all_single(recv, inp, out_splits, in_splits, m)
        s = torch.tensor([float(r + 1), 0.5 * r])
        gdist._c_all_reduce(s, dist.ReduceOp.SUM, m)
        mn = torch.tensor([r + 3], dtype=torch.int32)
        gdist._c_all_reduce(mn, dist.ReduceOp.MIN, m)
        b = torch.full((3,), float(r))
        gdist._c_broadcast(b, 0, m)
        return outs, big, recv, s, mn, b

    res = _run(world, fn)
    for r, (outs, big, recv, s, mn, b) in enumerate(res):
        for q in range(world):
            assert torch.equal(outs[q], torch.arange(4, dtype=torch.float32) + 10 * q)
        assert torch.equal(big, torch.cat([torch.arange(4, dtype=torch.float32) + 10 * q for q in range(world)]))
        assert torch.equal(recv, torch.cat([torch.full((r + 1, 2), 100.0 * q + r) for q in range(world)]))
        assert torch.equal(s, torch.tensor([sum(q + 1.0 for q in range(world)), sum(0.5 * q for q in range(world))]))
        assert int(mn) == 3 and torch.equal(b, torch.zeros(3))


def test_all_reduce_adds_in_rank_order():
    vals = [1e8, 1.0, -1e8]  # (1e8 + 1) - 1e8 = 0 in fp32; 1e8 + (1 - 1e8) = 0 too, but 1 + (-1e8 + 1e8) would be 1

    def fn(m):
        t = torch.tensor([vals[m.rank]], dtype=torch.float32)
        gdist._c_all_reduce(t, dist.ReduceOp.SUM, m)
        return t

    want = (torch.tensor(vals[0]) + torch.tensor(vals[1])) + torch.tensor(vals[2])
    assert all(torch.equal(t, want.reshape(1)) for t in _run(3, fn))


def test_point_to_point_pairs_sends_and_receives():
    def fn(m):
        r, W = m.rank, m.world
        dst, src = (r + 1) % W, (r - 1) % W
        works, finish = gdist._p2p_exchange([(torch.full((2,), float(r)), dst)], [(torch.empty(2), src)], m)
        recv = None
        for w in works:
            w.wait()
        finish()
        # a second round to the other side, posted before the first is waited on elsewhere
        a = torch.full((3,), 10.0 + r)
        b = torch.empty(3)
        w2, _ = gdist._p2p_exchange([(a, src)], [(b, dst)], m)
        for w in w2:
            w.wait()
        return b

    for r, b in enumerate(_run(3, fn)):
        assert torch.equal(b, torch.full((3,), 10.0 + (r + 1) % 3))


def test_mismatched_collectives_raise():
    def fn(m):
        t = torch.zeros(2)
        if m.rank == 0:
            gdist._c_all_reduce(t, dist.ReduceOp.SUM, m)
        else:
            gdist._c_broadcast(t, 0, m)

    with pytest.raises((RuntimeError, threading.BrokenBarrierError)):
        _run(2, fn, timeout=10)


@pytest.mark.parametrize("mode", ["dense", "sparse"])
def test_halo_exchange_over_local_ranks(mode):
    """The module's exchange (autograd _HaloExchange, forward and backward)
    over a LocalGroup: X_ext = [own | halo] in the plan's layout, and dX the
    owner's row plus every peer's partial in peer order."""
    gen = torch.Generator().manual_seed(3)
    N, world, F = 30, 3, 5
    bounds = [0, 9, 21, 30]
    cols = [torch.randint(0, N, (4 * (bounds[r + 1] - bounds[r]),), generator=gen) for r in range(world)]
    plans = build_halo_plans_local(cols, bounds, mode=mode)
    X = torch.randn(N, F, generator=gen)
    G = [torch.randn(plans[r].n_loc + plans[r].n_halo, F, generator=gen) for r in range(world)]

    def fn(m):
        p = plans[m.rank]
        x = X[bounds[m.rank]:bounds[m.rank + 1]].clone().requires_grad_(True)
        X_ext = gdist.halo_exchange(x, p, m)
        X_ext.backward(G[m.rank])
        return X_ext.detach(), x.grad

    res = _run(world, fn)
    for r, (X_ext, dx) in enumerate(res):
        p = plans[r]
        c = cols[r]
        # every edge's source row is where the plan's local column points
        assert torch.equal(X_ext[p.colidx_local.long()], X[c])
        want = G[r][:p.n_loc].clone()
        for q in range(world):  # peer q's partials for my rows, in peer order
            if q == r:
                continue
            pq = plans[q]
            if mode == "dense":
                want += G[q][pq.stride * (1 + r): pq.stride * (1 + r) + p.n_loc]
            else:
                ids = pq.halo_ids
                off = pq.n_loc + sum(pq.recv_counts[:r])
                mine = ids[sum(pq.recv_counts[:r]): sum(pq.recv_counts[:r + 1])] - bounds[r]
                want.index_add_(0, mine, G[q][off: off + pq.recv_counts[r]])
        torch.testing.assert_close(dx, want, rtol=0, atol=1e-6)
