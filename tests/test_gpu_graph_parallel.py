"""GPU: the warper-level entry to node-range graph parallelism
(`graph_parallel: node_range`, gnn.utils.config.node_range_parallel; the
reference's multi-GPU entry is data parallelism over documents,
cl_warper.py:73-75).  Two gloo ranks share the box's GPU; each runs the
product's training step (KVProcedure._run_train_step: forward, loss,
backward, the procedure's gradient all-reduce, clip, Adam) on its node range
of the WHOLE batch's graph (grl.dist.ShardedGraph).  A single-process
procedure runs the same steps on the same batch.  DropEdge p = 0.3 with a
fixed seed is on (its masks are keyed on global edge ids, so both runs drop
the same edges); feature dropout is off (the one-process model runs graphs
this small on torch's dropout).  Checked per step: the loss (1e-4), the
first step's gradients (1e-4 of each gradient's scale, as the sharded-model
tests), the validation loss (1e-4); after the steps the two ranks' weights
are bitwise equal and within 1e-4 of the one-process weights."""
import os
import socket

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

B, N, L, F_IN, C_OUT, NET = 1, 160, 6, 64, 15, 32  # one graph per step (batch_size 1)
STEPS = 3
SEED = 11


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _batches():
    rng = np.random.default_rng(7)
    out = []
    for _ in range(STEPS):
        V = (rng.random((B, N, F_IN)) < 0.1).astype(np.float32)
        A = (rng.random((B, N, L, N)) < 3.0 / (L * N)).astype(np.float32)
        y = rng.integers(0, C_OUT, (B, N)).astype(np.int64)
        y[:, -30:] = -100  # unlabelled nodes: ignored by the loss, so the ranks' shares are unequal
        out.append({"textline_encoding": torch.from_numpy(V), "adjacency_matrix": torch.from_numpy(A),
                    "node_label": torch.from_numpy(y)})
    return out


def _procedure(cfg, distributed):
    from gnn.models import GraphCNNDropEdge
    from gnn.trainer.training_procedures import KVProcedure

    torch.manual_seed(0)
    model = GraphCNNDropEdge(F_IN, C_OUT, L, net_size=NET, dropedge_seed=SEED)
    model.dropout.p = 0.0
    assert model.edge_dropout.p == 0.3
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
        gp = _procedure(cfg, True)
        single = _procedure(cfg, False)
        assert gp.graph_parallel and not single.graph_parallel and gp.step_graph is None
        for step, batch in enumerate(_batches()):
            s_gp, _ = gp._run_train_step(batch)
            s_one, _ = single._run_train_step(batch)
            assert abs(s_gp["loss"] - s_one["loss"]) <= 1e-4 * max(1.0, abs(s_one["loss"])), (step, s_gp, s_one)
            if step == 0:  # the (clipped, summed) gradients the optimizer stepped with
                for (name, p_gp), (_, p_one) in zip(gp.model.named_parameters(), single.model.named_parameters()):
                    if p_one.grad is None:
                        assert p_gp.grad is None, name
                        continue
                    scale = float(p_one.grad.abs().max())
                    err = float((p_gp.grad - p_one.grad).abs().max())
                    assert err <= 1e-4 * max(scale, 1e-6), (name, err, scale)  # of the gradient's scale
            if step + 1 < STEPS:
                gp.model.zero_grad()
                single.model.zero_grad()
            v_gp, _ = gp._run_val_step(batch)
            v_one, _ = single._run_val_step(batch)
            assert abs(v_gp["loss"] - v_one["loss"]) <= 1e-4 * max(1.0, abs(v_one["loss"])), (step, v_gp, v_one)
        assert len(gp._shard_cache) == STEPS  # each step's validation reused its training step's shard plan
        flat = torch.cat([p.detach().reshape(-1).cpu() for p in gp.model.parameters()])
        gathered = [torch.empty_like(flat) for _ in range(world)]
        dist.all_gather(gathered, flat)
        assert torch.equal(gathered[0], gathered[1])
        for (name, p_gp), (_, p_one) in zip(gp.model.named_parameters(), single.model.named_parameters()):
            err = float((p_gp - p_one).abs().max())
            assert err <= 1e-4 * max(1.0, float(p_one.abs().max())), (name, err)
    finally:
        dist.destroy_process_group()


def test_graph_parallel_step_equals_single_process(tmp_path):
    import torch.multiprocessing as mp

    from test_data_pipeline import make_config

    cfg = make_config(str(tmp_path), epochs=1)
    cfg.capture_train_step = False
    cfg.dist_backend = "gloo"
    cfg.graph_parallel = "node_range"
    mp.spawn(_worker, args=(2, _free_port(), cfg), nprocs=2, join=True)


def _predict_worker(rank, world, port, cfg_dir):
    import json

    import torch.distributed as dist

    from gnn.cl_warper import GNNLearningWarper
    from gnn.models import GraphCNNDropEdge
    from test_data_pipeline import ASSETS, make_config

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    classes = os.path.join(cfg_dir, "classes26.json")
    out = {}
    for mode in ("single", "node_range"):
        cfg = make_config(os.path.join(cfg_dir, f"{mode}{rank}"), is_train=False)
        cfg.inference_settings.datasets.args.class_path = classes
        if mode == "node_range":
            cfg.distributed, cfg.num_gpus, cfg.local_rank, cfg.dist_backend = True, world, rank, "gloo"
            cfg.graph_parallel = "node_range"
            cfg.graph_parallel_args = {"balance": "nodes", "halo": "dense"}
        torch.manual_seed(0)
        warper = GNNLearningWarper(GraphCNNDropEdge(4369, 53, 6, 256), config=cfg)
        assert warper.inferencer.graph_parallel == (mode == "node_range")
        with open(os.path.join(ASSETS, "debug.json"), encoding="utf-8-sig") as f:
            out[mode] = warper.predict([json.load(f)])[0]
    try:
        assert len(out["single"]) == len(out["node_range"]) == 74
        conf = np.array([[b["confidence"] for b in out[m]] for m in ("single", "node_range")])
        np.testing.assert_allclose(conf[1], conf[0], rtol=0, atol=1e-5)
        same = sum((a["formal_key"], a["key_type"]) == (b["formal_key"], b["key_type"])
                   for a, b in zip(out["single"], out["node_range"]))
        assert same >= 73, same  # a near-tie may flip one argmax
        got = [None] * world
        dist.all_gather_object(got, conf[1].tolist())
        assert got[0] == got[1]  # every rank returns the whole document's boxes
    finally:
        dist.destroy_process_group()


def test_graph_parallel_predict_equals_single_process(tmp_path):
    """warper.predict() with graph_parallel: node_range on two gloo ranks:
    each rank predicts its node range of debug.json's graph (74 nodes, the
    config-1 model) and all-gathers the logits; every rank returns the
    single-process boxes (confidences within 1e-5)."""
    import json

    import torch.multiprocessing as mp

    with open(os.path.join(str(tmp_path), "classes26.json"), "w") as f:
        json.dump({"classes": [f"c{i}" for i in range(26)]}, f)
    mp.spawn(_predict_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)


def test_shard_cache_confirms_a_key_hit(monkeypatch):
    """A cache_key collision (forced here: every graph gets one key) must not
    hand a graph another graph's shard plan: the hit is confirmed by exact
    equality of the CSR arrays (ShardedGraph.same_graph), so a different
    graph gets its own plan and the same graph met again reuses its plan."""
    from grl import TypedGraph
    from grl.dist import ShardedGraph
    from gnn.trainer.training_procedures.kv_procedure import sharded_graph_cached

    dev = torch.device("cuda")
    rng = np.random.default_rng(3)

    def graph():
        A = (rng.random((1, 40, L, 40)) < 0.05).astype(np.float32)
        return TypedGraph.from_dense(torch.from_numpy(A).to(dev), layout="bnln")

    g1, g2 = graph(), graph()
    assert not ShardedGraph.same_graph(g1, g2)
    monkeypatch.setattr(ShardedGraph, "cache_key", staticmethod(lambda g, **kw: ("collide",)))

    class Owner:
        pass

    o = Owner()
    s1 = sharded_graph_cached(o, g1, {})
    s2 = sharded_graph_cached(o, g2, {})
    assert s2 is not s1
    assert torch.equal(s2.graph.colidx, ShardedGraph.from_graph(g2).graph.colidx)
    g2_again = TypedGraph(g2.rowptr.clone(), g2.colidx.clone(), L, has_self=True, num_cols=g2.num_cols)
    assert sharded_graph_cached(o, g2_again, {}) is s2
    # vals compared by their bits: the same structure with other weights is another graph
    g3 = TypedGraph(g2.rowptr.clone(), g2.colidx.clone(), L, has_self=True, num_cols=g2.num_cols,
                    vals=torch.rand(g2.colidx.numel(), device=dev))
    assert not ShardedGraph.same_graph(g2, g3)
    assert sharded_graph_cached(o, g3, {}) is not s2
