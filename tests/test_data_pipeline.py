"""CPU-only: the document pipeline feeding the hot path, against the
reference's own outputs (tests/golden/: normalize_text.json, layout_graphs.npz,
model_debug.npz -- all produced by make_golden.py from the reference)."""
import json
import os

import numpy as np
import pytest
import torch

import inputs as gi
from gnn.data_generator.base_dataloader import BaseDataLoader
from gnn.data_generator.data_collate import NumpyPadding, TypedEdgePadding
from gnn.data_generator.data_process import HeuristicGraphBuilder, NodeLabeling, TextlineEncoding
from gnn.data_generator.data_process.normalize_text import normalize_text
from gnn.utils.config import AttrDict

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
ASSETS = os.path.join(GOLDEN, "assets")


def charset():
    with open(os.path.join(ASSETS, "master_charset.json"), encoding="utf-8-sig") as f:
        cs = json.load(f)["charset"]
    return {c: i for i, c in enumerate(cs)}


def test_normalize_text_matches_reference():
    with open(os.path.join(GOLDEN, "normalize_text.json"), encoding="utf-8") as f:
        d = json.load(f)
    for src, ref in zip(d["inputs"], d["outputs"]):
        assert normalize_text(src) == ref, src


@pytest.mark.parametrize("name", ["debug", "float80", "plain30"])
def test_textline_encoding_matches_reference(golden, name):
    fx = golden("layout_graphs.npz")
    regs = json.loads(str(fx[f"{name}::regions"]))
    label = {i: {"polygon": r["location"], "text": r["text"], "label": r.get("label", "other")}
             for i, r in enumerate(regs)}
    out = TextlineEncoding(is_normalized_text=True)({"label": label, "char_to_id": charset()})
    V = out["textline_encoding"]
    assert V.dtype == np.float32 and V.shape == (len(regs), 4365 + 4)
    r, c = np.nonzero(V[:, :-4])
    np.testing.assert_array_equal(r, fx[f"{name}::bow_rows"])
    np.testing.assert_array_equal(c, fx[f"{name}::bow_cols"])
    np.testing.assert_array_equal(V[:, -4:], fx[f"{name}::spatial"])


def test_debug_features_match_model_fixture(golden):
    """V and A of debug.json through TextlineEncoding + HeuristicGraphBuilder
    equal the inputs the reference fed its model (model_debug.npz)."""
    g = golden("model_debug.npz")
    with open(os.path.join(ASSETS, "debug.json"), encoding="utf-8-sig") as f:
        regions = json.load(f)
    label = {i: dict(r, polygon=r["location"]) for i, r in enumerate(regions)}
    s = {"label": label, "char_to_id": charset()}
    s = TextlineEncoding(True)(s)
    s = HeuristicGraphBuilder(6, "normal_binary")(s)
    Vref = np.zeros(tuple(g["V_shape"]), dtype=np.float32)
    Vref[g["V_rows"], g["V_cols"]] = g["V_vals"]
    np.testing.assert_array_equal(s["textline_encoding"], Vref)
    Aref = np.unpackbits(g["A_bits"])[: int(np.prod(g["A_shape"]))].reshape(tuple(g["A_shape"]))
    assert s["adjacency_matrix"].dtype == np.float16
    np.testing.assert_array_equal(s["adjacency_matrix"] != 0, Aref.astype(bool))


def test_node_labeling():
    class_to_id = {"a": {"key": 1, "value": 2}, "b": {"key": 3, "value": 4}}
    label = {2: {"label": "b", "key_type": "value"}, 0: {"label": "a", "key_type": "key"},
             5: {"label": None, "key_type": None}}
    out = NodeLabeling()({"label": label, "class_to_id": class_to_id})
    np.testing.assert_array_equal(out["node_label"], [1, 4, 0])


def test_numpy_padding_is_symmetric():
    pad = NumpyPadding({"x": 0.0, "node_label": -100}, only_selected_items=True)
    items = [{"x": np.ones((3, 2), np.float32), "node_label": np.array([1, 2, 3]), "drop": 1},
             {"x": np.ones((6, 2), np.float32), "node_label": np.arange(6)}]
    out = pad(items)
    assert set(out[0]) == {"x", "node_label"}
    np.testing.assert_array_equal(out[0]["node_label"], [-100, 1, 2, 3, -100, -100])  # (3//2, 3 - 3//2)
    assert out[0]["x"].shape == (6, 2) and out[0]["x"][0].sum() == 0 and out[0]["x"][1].sum() == 2


def test_typed_edge_padding_equals_dense_padding(golden):
    """The edge-list batch is exactly the dense NumpyPadding batch's graph."""
    fx = golden("layout_graphs.npz")
    docs = []
    for name in ("plain30", "tiny2", "cells60"):
        regs = json.loads(str(fx[f"{name}::regions"]))
        label = {i: {"polygon": r["location"], "text": r["text"], "label": r["label"]} for i, r in enumerate(regs)}
        s = HeuristicGraphBuilder(6, "normal_binary", emit="both")({"label": label})
        s["node_label"] = np.arange(s["adjacency_matrix"].shape[0])
        docs.append(s)
    dense = NumpyPadding({"adjacency_matrix": 0.0, "node_label": -100}, True)([dict(d) for d in docs])
    A = np.stack([d["adjacency_matrix"] for d in dense])  # (B, N, 6, N)
    batch = TypedEdgePadding({"node_label": -100}, True)([dict(d) for d in docs])
    B, N = batch["graph_shape"]
    e = batch["typed_edges"]
    rebuilt = np.zeros((B * N, 6, B * N), dtype=bool)
    rebuilt[e[:, 0], e[:, 1], e[:, 2]] = True
    for b in range(B):
        blk = rebuilt[b * N:(b + 1) * N, :, b * N:(b + 1) * N]
        np.testing.assert_array_equal(blk, A[b] != 0)
    np.testing.assert_array_equal(batch["node_label"], np.stack([d["node_label"] for d in dense]))


def _via(regions, labels):
    """VIA-format document from cassia-style regions + (formal_key, key_type) labels."""
    regs = []
    for r, (fk, kt) in zip(regions, labels):
        xs = [p[0] for p in r["location"]]
        ys = [p[1] for p in r["location"]]
        regs.append({"shape_attributes": {"name": "polygon", "all_points_x": xs, "all_points_y": ys},
                     "region_attributes": {"label": r["text"], "formal_key": fk, "key_type": kt}})
    return {"attributes": {"_via_img_metadata": {"regions": regs}}}


def write_datapile(root, n_docs=5, seed=0):
    """A tiny on-disk datapile dataset from debug.json-like synthetic pages
    with random sumi labels; returns the folder."""
    rng = np.random.default_rng(seed)
    with open(os.path.join(ASSETS, "sumi_classes.json"), encoding="utf-8-sig") as f:
        classes = json.load(f)["classes"]
    os.makedirs(root, exist_ok=True)
    for d in range(n_docs):
        regs = gi.synthetic_document(100 + d, int(rng.integers(20, 60)))
        labels = [(classes[int(rng.integers(len(classes)))], ["key", "value"][int(rng.integers(2))])
                  if rng.random() < 0.5 else (None, None) for _ in regs]
        with open(os.path.join(root, f"doc{d}.json"), "w", encoding="utf-8") as f:
            json.dump(_via(regs, labels), f)
    return root


def make_config(tmp, emit="dense", epochs=2, is_train=True):
    data_root = write_datapile(os.path.join(tmp, "data"))
    collate = ({"NumpyPadding": {"name_value_pairs": {"textline_encoding": 0.0, "adjacency_matrix": 0.0,
                                                       "node_label": -100.0}, "only_selected_items": True}}
               if emit == "dense" else
               {"TypedEdgePadding": {"name_value_pairs": {"textline_encoding": 0.0, "node_label": -100.0},
                                     "only_selected_items": True}})
    split = {"data_path": [data_root], "class_path": os.path.join(ASSETS, "sumi_classes.json"),
             "charset_path": os.path.join(ASSETS, "master_charset.json"), "key_types": ["key", "value"],
             "batch_size": 2, "num_workers": 0, "shuffle": True, "drop_last": False, "pin_memory": False,
             "augmentations": [], "data_collate": collate,
             "data_process": {"TextlineEncoding": {"is_normalized_text": True},
                              "HeuristicGraphBuilder": {"num_edges": 6, "edge_type": "normal_binary", "emit": emit},
                              "NodeLabeling": {}}}
    return AttrDict({
        "experiment_name": "t", "seed": 1111, "is_train": is_train, "output_dir": os.path.join(tmp, "out"),
        "checkpoint_path": None, "num_gpus": 1, "distributed": False, "local_rank": 0, "num_epochs": epochs,
        "max_grad_norm": 5.0, "model_dir_name": "models", "benchmark": False, "deterministic": True,
        "data_config": {"dataset": {"type": "DatapileDataset",
                                    "args": {"node_label_padding_value": -100, "other_class_index": None}},
                        "training": split, "validation": dict(split, batch_size=1)},
        "procedure": {"type": "KVProcedure" if is_train else "KVInference", "args": {}},
        "loss": {"type": "CrossEntropyLoss", "args": {}},
        "lr_scheduler": {"type": "DecayLearningRate", "args": {"lr": 0.001, "factor": 0.9, "num_epochs": 100}},
        "optimizer": {"type": "BuitlinOptimizer", "args": {"type_optimizer": "Adam", "lr": 0.001}},
        "inference_settings": {"num_gpus": 1, "output_dir_name": "infer",
                               "activation": {"type": "Softmax", "args": {"dim": -1}},
                               "datasets": {"type": "CassiaDataset",
                                            "args": dict(split, data_path=None)},
                               "post_processing": {}},
    })


def test_datapile_loader_batches(tmp_path):
    cfg = make_config(str(tmp_path))
    loader = BaseDataLoader(cfg)
    ds = loader._load_dataset("DatapileDataset", cfg.data_config.training, data_type="training")
    assert len(ds) == 5 and ds.class_to_id["surgery_name"]["value"] == 14
    dl = loader._get_dataloader(ds, ds.data_config)
    batch = next(iter(dl))
    V, A, y = batch["textline_encoding"], batch["adjacency_matrix"], batch["node_label"]
    assert V.shape[0] == 2 and V.shape[2] == 4369 and A.shape[1:] == (V.shape[1], 6, V.shape[1])
    assert A.dtype == torch.float16 and y.dtype == torch.int64 and (y == -100).any() == (V.shape[1] > 0)


def test_warper_refuses_cpu(tmp_path):
    """Without a GPU the engine fails loudly instead of computing on the host."""
    from gnn.cl_warper import GNNLearningWarper
    from gnn.models import GraphCNNDropEdge
    from grl import GrlError

    if torch.cuda.is_available():
        pytest.skip("checks the no-GPU behaviour")
    cfg = make_config(str(tmp_path), epochs=1)
    warper = GNNLearningWarper(GraphCNNDropEdge(4369, 15, 6, net_size=16), config=cfg)
    with pytest.raises(GrlError, match="ROCm device"):
        warper.train()


def test_macro_report_equals_sklearn():
    """The procedure's per-step metric (kv_procedure.macro_report, class ids +
    bincounts) gives exactly sklearn's classification_report macro avg on the
    class names, including absent classes, zero divisions and repeated names."""
    from sklearn.metrics import classification_report

    from gnn.trainer.training_procedures.kv_procedure import macro_report

    rng = np.random.default_rng(0)
    names = tuple(["other"] + [f"k{i}_{t}" for i in range(12) for t in ("key", "value")])
    for trial in range(60):
        n = int(rng.integers(0, 300))
        k = int(rng.integers(1, len(names)))
        yt = rng.integers(0, k, n)
        yp = np.where(rng.random(n) < 0.6, yt, rng.integers(0, len(names), n))
        nm = names if trial % 3 else tuple(names[:5]) + tuple(names[1:])  # repeated names
        got = macro_report(yt, yp, nm)
        tn, pn = [nm[i] for i in yt.tolist()], [nm[i] for i in yp.tolist()]
        if n == 0:
            assert got == {"precision": 0.0, "recall": 0.0, "f1-score": 0.0, "support": 0.0}
            continue
        ref = classification_report(tn, pn, output_dict=True, zero_division=0)["macro avg"]
        assert got == {k2: ref[k2] for k2 in ("precision", "recall", "f1-score", "support")}, (trial, got, ref)


def test_graph_parallel_config_switch():
    """graph_parallel: node_range needs distributed; anything else is refused
    (gnn.utils.config.node_range_parallel)."""
    from gnn.utils.config import node_range_parallel

    assert not node_range_parallel({})
    assert not node_range_parallel({"graph_parallel": "documents", "distributed": True})
    assert not node_range_parallel({"graph_parallel": "node_range"})
    assert node_range_parallel({"graph_parallel": "node_range", "distributed": True})
    with pytest.raises(ValueError):
        node_range_parallel({"graph_parallel": "edges", "distributed": True})


@pytest.mark.parametrize("weight", [None, [0.5 + 0.1 * i for i in range(5)]])
def test_shard_loss_shares_add_up_to_the_batch_mean(weight):
    """graph_parallel: node_range -- each rank's loss is its rows' criterion
    times their share of the batch's (class-weighted) valid targets, so the
    shares over any node-range split add up to the one-process mean
    (KVProcedure._shard_loss; ignore_index -100 rows carry no weight), and a
    rank with no labelled row contributes an exact zero."""
    from gnn.trainer.losses import CrossEntropyLoss
    from gnn.trainer.training_procedures.kv_procedure import KVProcedure

    torch.manual_seed(0)
    proc = KVProcedure.__new__(KVProcedure)
    proc.criterion = CrossEntropyLoss(weight=weight)
    N, C = 37, 5
    logits = torch.randn(1, N, C, dtype=torch.float64)
    t = torch.randint(0, C, (1, N))
    t[0, 10:20] = -100
    full = proc.criterion(logits.float(), t).double()
    for bounds in ([0, 18, 37], [0, 5, 12, 30, 37], [0, 10, 20, 37]):
        parts = [proc._shard_loss(logits[:, a:b].float(), t[:, a:b], t) for a, b in zip(bounds[:-1], bounds[1:])]
        assert abs(float(sum(p.double() for p in parts)) - float(full)) <= 1e-6 * max(1.0, abs(float(full)))
    empty = proc._shard_loss(logits[:, 10:20].float().requires_grad_(), t[:, 10:20], t)
    assert float(empty) == 0.0 and empty.requires_grad


def test_node_range_honours_shuffle_with_one_order_for_every_rank(tmp_path):
    """graph_parallel: node_range with shuffle: true -- every rank must train
    on the same batch each step, so the loader shuffles through a fixed-seed
    one-replica sampler (the same order wherever it is built, a new order per
    epoch through set_epoch) instead of ignoring shuffle."""
    from torch.utils.data import DistributedSampler

    cfg = make_config(str(tmp_path))
    cfg.distributed = True
    cfg.graph_parallel = "node_range"
    orders = []
    for _ in range(2):  # two "ranks": two independently built loaders
        loader = BaseDataLoader(cfg)
        ds = loader._load_dataset("DatapileDataset", cfg.data_config.training, data_type="training")
        dl = loader._get_dataloader(ds, ds.data_config)
        assert isinstance(dl.sampler, DistributedSampler) and dl.sampler.num_replicas == 1
        per_epoch = []
        for ep in range(3):
            dl.sampler.set_epoch(ep)
            per_epoch.append(list(iter(dl.sampler)))
        orders.append(per_epoch)
    assert orders[0] == orders[1]
    assert sorted(orders[0][0]) == list(range(5))
    assert len({tuple(o) for o in orders[0]}) > 1  # reshuffled across epochs
    cfg.data_config.training.shuffle = False
    loader = BaseDataLoader(cfg)
    ds = loader._load_dataset("DatapileDataset", cfg.data_config.training, data_type="training")
    assert not isinstance(loader._get_dataloader(ds, ds.data_config).sampler, DistributedSampler)
