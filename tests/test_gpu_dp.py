"""GPU: data parallelism across documents (the reference's
declared DP at cl_warper.py:73-75 / base_dataloader.py:91-106) against a
single process.  Two gloo ranks share the box's GPU; each runs the product's
training step (KVProcedure._run_train_step, kv_procedure.py:143-164 in the
reference: forward, loss, backward, then the procedure's averaged bucketed
gradient all-reduce, clip, Adam) on its half of the batch.  A single-process
procedure runs the same steps on the union batch.  With equal-size graphs
the union mean loss is the mean of the two halves' losses, so:
  * the averaged gradients equal the union batch's gradients (1e-4),
  * the loss curve over three Adam steps matches (1e-4).
Feature dropout and DropEdge are off (p = 0) so both runs draw nothing.

With randomness on (test_dp_dropedge_matches_oracle_with_per_rank_masks):
DropEdge p = 0.3 with a fixed dropedge_seed; the procedure gives rank r the
DropEdge stream r (call c -> c + r * 2^32), so the ranks' masks are
independent although every rank is seeded alike.  Each step is checked
against the oracle (oracle/dense_torch.py, float64, dense A_pre) on the
UNION batch with every document's mask regenerated from its rank's
(seed, call, edge id): the mean loss and the averaged, clipped gradients
(1e-4).  A device-drawn seed (dropedge_seed=None) and feature dropout differ
across ranks too."""
import os
import socket

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

B, N, L, F_IN, C_OUT, NET = 4, 24, 6, 64, 15, 32
STEPS = 3


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _batches():
    """Three union batches of B equal-size graphs (every node labelled)."""
    rng = np.random.default_rng(42)
    out = []
    for _ in range(STEPS):
        V = (rng.random((B, N, F_IN)) < 0.1).astype(np.float32)
        A = (rng.random((B, N, L, N)) < 3.0 / (L * N)).astype(np.float32)
        y = rng.integers(0, C_OUT, (B, N)).astype(np.int64)
        out.append({"textline_encoding": torch.from_numpy(V), "adjacency_matrix": torch.from_numpy(A),
                    "node_label": torch.from_numpy(y)})
    return out


def _half(batch, rank, world):
    per = B // world
    return {k: v[rank * per:(rank + 1) * per] for k, v in batch.items()}


def _procedure(cfg, distributed):
    from gnn.models import GraphCNNDropEdge
    from gnn.trainer.training_procedures import KVProcedure

    torch.manual_seed(0)
    model = GraphCNNDropEdge(F_IN, C_OUT, L, net_size=NET)
    model.dropout.p = 0.0
    model.edge_dropout.p = 0.0
    c = type(cfg)(dict(cfg))
    c.distributed = distributed
    return KVProcedure(model, c)


def _worker(rank, world, port, cfg):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        cfg.num_gpus, cfg.local_rank = world, rank
        dp = _procedure(cfg, True)
        single = _procedure(cfg, False)
        assert dp.distributed and not single.distributed
        for step, batch in enumerate(_batches()):
            s_dp, _ = dp._run_train_step(_half(batch, rank, world))
            s_one, _ = single._run_train_step(batch)
            losses = [None] * world
            dist.all_gather_object(losses, s_dp["loss"])
            assert abs(np.mean(losses) - s_one["loss"]) <= 1e-4 * max(1.0, abs(s_one["loss"])), (step, losses, s_one)
            if step == 0:  # the (clipped) gradients each optimizer stepped with
                for (name, p_dp), (_, p_one) in zip(dp.model.named_parameters(), single.model.named_parameters()):
                    if p_one.grad is None:
                        assert p_dp.grad is None, name
                        continue
                    torch.testing.assert_close(p_dp.grad, p_one.grad, rtol=1e-4, atol=1e-6, msg=name)
        # the replicas stayed identical to each other
        flat = torch.cat([p.detach().reshape(-1).cpu() for p in dp.model.parameters()])
        gathered = [torch.empty_like(flat) for _ in range(world)]
        dist.all_gather(gathered, flat)
        assert torch.equal(gathered[0], gathered[1])
    finally:
        dist.destroy_process_group()


def test_dp_step_equals_single_process_on_union_batch(tmp_path):
    import torch.multiprocessing as mp

    from test_data_pipeline import make_config

    cfg = make_config(str(tmp_path), epochs=1)
    cfg.capture_train_step = False  # the eager step: the oracle regenerates its (seed, call) masks
    cfg.dist_backend = "gloo"
    mp.spawn(_worker, args=(2, _free_port(), cfg), nprocs=2, join=True)


SEED = 11
P_EDGE = 0.3


def _oracle_step(P64, batch, rank_halves, step, max_norm):
    """Union-batch loss and clipped gradients of the dense float64 oracle with
    each document's three DropEdge masks regenerated from its rank's stream."""
    import torch.nn.functional as F

    from oracle import dense_ref, dense_torch

    world = len(rank_halves)
    mults = []
    for i in range(3):
        per_rank = []
        for q, half in enumerate(rank_halves):
            call = 3 * step + i + (q << 32)
            per_rank.append(dense_ref.dropedge_weights_pre(half["adjacency_matrix"].numpy(), P_EDGE, SEED, call, True))
        mults.append(torch.from_numpy(np.concatenate(per_rank, 0)).double())
    P = {k: v.clone().requires_grad_(k != "w_rand.projection.weight") for k, v in P64.items()}
    logits = dense_torch.forward(P, batch["textline_encoding"].double(), batch["adjacency_matrix"].double(),
                                 train=False, edge_mults=mults)
    loss = F.cross_entropy(logits.transpose(1, 2), batch["node_label"])
    loss.backward()
    params = [v for k, v in P.items() if v.requires_grad]
    torch.nn.utils.clip_grad_norm_(params, max_norm)
    assert world == 2
    return float(loss.detach()), {k: v.grad for k, v in P.items() if v.requires_grad}


def _worker_random(rank, world, port, cfg):
    import torch.distributed as dist

    from gnn.models import GraphCNNDropEdge
    from gnn.trainer.training_procedures import KVProcedure
    from oracle import hash as ohash

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        cfg.num_gpus, cfg.local_rank = world, rank
        c = type(cfg)(dict(cfg))
        c.distributed = True
        torch.manual_seed(0)
        model = GraphCNNDropEdge(F_IN, C_OUT, L, net_size=NET, dropedge_seed=SEED)
        model.dropout.p = 0.0  # feature dropout cannot be regenerated by the oracle; DropEdge can
        assert model.edge_dropout.p == P_EDGE
        dp = KVProcedure(model, c)
        assert dp.distributed and dp.model.edge_dropout.stream == rank
        # the two ranks' DropEdge masks differ (same seed, call numbers in disjoint streams)
        keep = torch.from_numpy(ohash.dropedge_keep(P_EDGE, SEED, 0 + (rank << 32), np.arange(4096, dtype=np.uint64)))
        both = [torch.empty_like(keep) for _ in range(world)]
        dist.all_gather(both, keep)
        assert not torch.equal(both[0], both[1])
        for step, batch in enumerate(_batches()):
            P64 = {k: v.detach().double().cpu() for k, v in dp.model.state_dict().items()}
            s_dp, _ = dp._run_train_step(_half(batch, rank, world))
            losses = [None] * world
            dist.all_gather_object(losses, s_dp["loss"])
            ref_loss, ref_grads = _oracle_step(P64, batch, [_half(batch, q, world) for q in range(world)], step,
                                               c.max_grad_norm)
            assert abs(np.mean(losses) - ref_loss) <= 1e-4 * max(1.0, abs(ref_loss)), (step, losses, ref_loss)
            for name, p in dp.model.named_parameters():
                if name in ref_grads:
                    torch.testing.assert_close(p.grad.double().cpu(), ref_grads[name], rtol=1e-4, atol=1e-6,
                                               msg=f"step {step} {name}")
        # the replicas stayed identical to each other
        flat = torch.cat([p.detach().reshape(-1).cpu() for p in dp.model.parameters()])
        gathered = [torch.empty_like(flat) for _ in range(world)]
        dist.all_gather(gathered, flat)
        assert torch.equal(gathered[0], gathered[1])
        # device-drawn DropEdge seeds and feature dropout: independent per rank too
        torch.manual_seed(0)
        model2 = GraphCNNDropEdge(F_IN, C_OUT, L, net_size=NET)
        dp2 = KVProcedure(model2, c)
        g = dp2.model.to_graph(_batches()[0]["adjacency_matrix"][:1].to(dp2.device))
        dp2.model.train()
        de = dp2.model.edge_dropout(g).dropedge
        assert de.call == rank and de.seed_tensor is not None
        fmask = dp2.model.dropout(torch.ones(4, 256, device=dp2.device)).cpu()  # the model's hash-keyed dropout
        draws = [(de.seed_tensor.cpu(), fmask) for _ in range(world)]
        dist.all_gather_object(draws, (de.seed_tensor.cpu(), fmask))
        assert int(draws[0][0]) != int(draws[1][0])  # DropEdge seeds drawn on the device
        assert not torch.equal(draws[0][1], draws[1][1])  # feature-dropout masks
    finally:
        dist.destroy_process_group()


def test_dp_dropedge_matches_oracle_with_per_rank_masks(tmp_path):
    import torch.multiprocessing as mp

    from test_data_pipeline import make_config

    cfg = make_config(str(tmp_path), epochs=1)
    cfg.capture_train_step = False  # the eager step: the oracle regenerates its (seed, call) masks
    cfg.dist_backend = "gloo"
    mp.spawn(_worker_random, args=(2, _free_port(), cfg), nprocs=2, join=True)
