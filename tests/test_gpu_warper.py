"""GPU: the reference's public API end to end on the engine --
GNNLearningWarper(model, config).train() / .predict() (gnn/cl_warper.py)."""
import json
import os

import numpy as np
import pytest
import torch

from gnn.cl_warper import GNNLearningWarper
from gnn.models import GraphCNNDropEdge
from test_data_pipeline import ASSETS, make_config

pytestmark = pytest.mark.gpu


def test_train_two_epochs_and_checkpoint(tmp_path):
    cfg = make_config(str(tmp_path), epochs=2)
    torch.manual_seed(0)
    model = GraphCNNDropEdge(4369, 15, 6, net_size=64)
    warper = GNNLearningWarper(model, config=cfg)
    f1 = warper.train()
    assert isinstance(f1, float) and 0.0 <= f1 <= 1.0
    # the warper moves output_dir to <output_dir>/<experiment_name> (cl_warper.py:43, 81-86)
    assert warper.config.output_dir == os.path.join(cfg.output_dir, cfg.experiment_name)
    ckpt_path = os.path.join(warper.config.output_dir, "models", "model_latest.pt")
    ckpt = torch.load(ckpt_path, weights_only=True)  # plain-dict config: safe loader works
    assert set(ckpt) == {"epoch", "config", "meta_data", "state_dict"}
    assert set(ckpt["state_dict"]) == set(model.state_dict())
    assert warper.trainer.global_step == 2 * 3  # 5 docs, batch 2, drop_last False
    assert hasattr(warper.trainer.model, "lambda_value")


def test_edge_batches_equal_dense_batches(tmp_path):
    """HeuristicGraphBuilder(emit="edges") + TypedEdgePadding gives the same
    training step as the reference's dense adjacency + NumpyPadding."""
    losses, grads = {}, {}
    for emit in ("dense", "edges"):
        cfg = make_config(str(tmp_path / emit), emit=emit, epochs=1)
        torch.manual_seed(0)
        model = GraphCNNDropEdge(4369, 15, 6, net_size=32)
        warper = GNNLearningWarper(model, config=cfg)
        proc = warper.trainer
        batch = next(iter(proc.train_loader))
        torch.manual_seed(7)
        scores, _ = proc._run_train_step(batch)
        losses[emit] = scores["loss"]
        grads[emit] = model.gcn1.h_weights.detach().clone()
    assert losses["dense"] == losses["edges"]
    assert torch.equal(grads["dense"], grads["edges"])


def test_predict_matches_reference_logits(golden, tmp_path):
    """predict() on debug.json (cassia format) with the config-1 model under
    torch.manual_seed(0): per-box class and confidence from the reference's
    logits (model_debug.npz) through softmax."""
    g = golden("model_debug.npz")
    classes = os.path.join(str(tmp_path), "classes26.json")
    with open(classes, "w") as f:
        json.dump({"classes": [f"c{i}" for i in range(26)]}, f)  # 26 x {key,value} + other = 53 outputs
    cfg = make_config(str(tmp_path), is_train=False)
    cfg.inference_settings.datasets.args.class_path = classes
    torch.manual_seed(0)
    model = GraphCNNDropEdge(4369, 53, 6, 256)
    warper = GNNLearningWarper(model, config=cfg)
    with open(os.path.join(ASSETS, "debug.json"), encoding="utf-8-sig") as f:
        doc = json.load(f)
    out = warper.predict([doc])
    assert len(out) == 1 and len(out[0]) == 74
    logits = g["logits"].astype(np.float64)
    p = np.exp(logits - logits.max(-1, keepdims=True))
    p /= p.sum(-1, keepdims=True)
    conf = np.array([b["confidence"] for b in out[0]])
    np.testing.assert_allclose(conf, p.max(-1), rtol=0, atol=1e-4)
    cls = p.argmax(-1)
    id_to_class = dict(warper.inferencer.id_to_class)
    for box, k in zip(out[0], cls):
        if abs(np.sort(p[list(out[0]).index(box)])[-1] - np.sort(p[list(out[0]).index(box)])[-2]) > 1e-4:
            assert (box["formal_key"], box["key_type"]) == tuple(id_to_class[int(k)])
    # a single document (not wrapped in a list) is accepted like the reference's
    # handle_single_input when given as a JSON path
    one = warper.predict(os.path.join(ASSETS, "debug.json"))
    assert len(one) == 74


def _dp_worker(rank, world, port, cfg):
    """One rank of data-parallel warper training (distributed: true): two gloo
    ranks sharing the box's GPU; replicas must end bitwise identical."""
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    cfg.distributed, cfg.num_gpus, cfg.local_rank, cfg.dist_backend = True, world, rank, "gloo"
    torch.manual_seed(100 + rank)  # different inits: the procedure must broadcast rank 0's
    model = GraphCNNDropEdge(4369, 15, 6, net_size=32)
    warper = GNNLearningWarper(model, config=cfg)
    assert dist.is_initialized() and warper.trainer.distributed
    f1 = warper.train()
    assert 0.0 <= f1 <= 1.0
    assert warper.trainer.global_step == 3  # 5 docs / 2 ranks -> 3 per rank, per-rank batch 2 // 2 = 1
    flat = torch.cat([p.detach().reshape(-1).cpu() for p in model.parameters()])
    gathered = [torch.empty_like(flat) for _ in range(world)]
    dist.all_gather(gathered, flat)
    assert torch.equal(gathered[0], gathered[1])
    dist.destroy_process_group()


def test_data_parallel_training_keeps_replicas_identical(tmp_path):
    import socket

    import torch.multiprocessing as mp

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cfg = make_config(str(tmp_path), epochs=1)  # writes the dataset once, before the ranks start
    mp.spawn(_dp_worker, args=(2, port, cfg), nprocs=2, join=True)


def _fixed_size_datapile(root, n_docs, n_regions, seed=3):
    """Datapile pages of one size (so every batch of 2 has the same shape and
    the captured training step replays)."""
    import inputs as gi
    from test_data_pipeline import _via

    rng = np.random.default_rng(seed)
    with open(os.path.join(ASSETS, "sumi_classes.json"), encoding="utf-8-sig") as f:
        classes = json.load(f)["classes"]
    os.makedirs(root, exist_ok=True)
    for d in range(n_docs):
        regs = gi.synthetic_document(200 + d, n_regions)
        labels = [(classes[int(rng.integers(len(classes)))], ["key", "value"][int(rng.integers(2))])
                  if rng.random() < 0.5 else (None, None) for _ in regs]
        with open(os.path.join(root, f"doc{d}.json"), "w", encoding="utf-8") as f:
            json.dump(_via(regs, labels), f)
    return root


def test_captured_train_step_equals_eager(tmp_path, monkeypatch):
    """capture_train_step: warper.train() replays each batch shape's whole
    training step (forward, CE, backward, clip, Adam) as one HIP graph
    (gnn/trainer/training_procedures/step_graph.py).  Against the same static
    pipeline run eagerly ("static": same static graphs, same per-step DropEdge
    seeds from a fixed dropedge_seed): the same per-step losses and the same
    trained weights, bit for bit, with most steps replayed."""
    from gnn.trainer.training_procedures import base_procedure

    losses = {}
    recorded = []
    monkeypatch.setattr(base_procedure.NullWriter, "add_scalar",
                        lambda self, tag, value, step=None: recorded.append(float(value)))
    models = {}
    for mode in ("static", True):
        recorded.clear()
        cfg = make_config(str(tmp_path / str(mode)), epochs=3)
        root = _fixed_size_datapile(str(tmp_path / str(mode) / "fixed"), n_docs=6, n_regions=40)
        cfg.data_config.training.data_path = [root]
        cfg.data_config.validation.data_path = [root]
        cfg.capture_train_step = mode
        torch.manual_seed(0)
        model = GraphCNNDropEdge(4369, 15, 6, net_size=64, dropedge_seed=5)
        model.dropout.p = 0.0  # feature dropout's CUDA RNG is not part of the comparison
        warper = GNNLearningWarper(model, config=cfg)
        warper.train()
        sg = warper.trainer.step_graph
        assert sg is not None and sg.step == 9, sg.stats()
        if mode is True:
            assert sg.captures >= 1 and sg.replays >= 6, sg.stats()
        else:
            assert sg.replays == 0
        losses[mode] = list(recorded)
        models[mode] = {k: v.detach().clone() for k, v in model.state_dict().items()}
    assert len(losses["static"]) == 9 and losses["static"] == losses[True], losses
    for k in models["static"]:
        assert torch.equal(models["static"][k], models[True][k]), k


def test_dense_bucket_builds_the_graph_of_from_dense():
    """A dense batch's captured step builds its typed CSR and CSC inside the
    replay (step_graph._Bucket.build_graph: no host sync on nnz): rowptr and
    the first nnz entries of colidx / vals / colptr / zrow / eid / cvals are
    TypedGraph.from_dense's bit for bit, the padding entries carry the
    sentinel column B*N that the CSC puts last; eager and from a HIP graph
    replayed on new data in the same static buffers."""
    from gnn.trainer.training_procedures.step_graph import _Bucket
    from grl import TypedGraph

    dev = torch.device("cuda:0")
    gen = torch.Generator().manual_seed(3)

    def batch(B, N, p, vals):
        A = (torch.rand(B, N, 6, N, generator=gen) < p).float()
        if vals:
            A = A * (0.5 + torch.rand(B, N, 6, N, generator=gen))
        A[0, 0, 0, :] = 0  # an empty row segment
        return A

    def check(b, A, vals):
        B, N = A.shape[0], A.shape[1]
        ref = TypedGraph.from_dense(A.to(dev), layout="bnln", keep_values=vals)
        n = ref.nnz  # 0 too: a page without edges
        assert torch.equal(b.rowptr, ref.rowptr)
        assert torch.equal(b.colidx[:n], ref.colidx) and bool((b.colidx[n:] == B * N).all())
        c, rc = b.csc, ref.csc()
        assert torch.equal(c["colptr"][:B * N + 1], rc["colptr"]) and int(c["colptr"][B * N + 1]) == b.cap
        for k in ("zrow", "eid"):
            assert torch.equal(c[k][:n], rc[k][:n]), k
        if vals:
            assert torch.equal(b.vals[:n], ref.vals) and torch.equal(c["cvals"][:n], rc["cvals"][:n])

    for B, N, vals in ((4, 74, False), (2, 33, True), (1, 5, False)):
        b = _Bucket(B, N, 8, 6, B * N * 6 * N, vals, dev, dense=True)
        V, y = torch.zeros(B, N, 8), torch.zeros(B, N, dtype=torch.int64)
        A = batch(B, N, 0.03, vals)
        b.load_dense(V, A, y)
        b.build_graph()
        check(b, A, vals)
        torch.cuda.synchronize()
        hg = torch.cuda.CUDAGraph()
        with torch.cuda.graph(hg):
            b.build_graph()
        for p in (0.08, 0.01):  # new batches into the same static buffers, replayed
            A = batch(B, N, p, vals)
            b.load_dense(V, A, y)
            hg.replay()
            check(b, A, vals)
