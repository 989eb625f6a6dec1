"""Where the drop-in training step's time goes on the reference's workload
(B=4 batches of debug.json pages, KVProcedure with capture_train_step):
per-phase host wall times, averaged over steps after warm-up."""
import os
import sys
import tempfile
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "graph-representation-learning_amd"))
sys.path.insert(0, os.path.join(HERE, ".."))
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    from gnn.trainer.training_procedures.kv_procedure import batch_graph

    dev = torch.device("cuda:0")
    res = {}
    orig = bench.c1_procedure_steps
    # build the procedure the bench builds, then time the phases of its step
    import types

    holder = {}

    def grab(proc):
        holder["proc"] = proc

    with tempfile.TemporaryDirectory() as tmp:
        from gnn.models import GraphCNNDropEdge
        from gnn.trainer.training_procedures import KVProcedure
        from gnn.utils.config import AttrDict

        root = bench._debug_datapile(os.path.join(tmp, "pages"))
        assets = os.path.join(bench.HERE, "tests", "golden", "assets")
        split = {"data_path": [root], "class_path": os.path.join(tmp, "classes26.json"),
                 "charset_path": os.path.join(assets, "master_charset.json"), "key_types": ["key", "value"],
                 "batch_size": 4, "num_workers": 0, "shuffle": False, "drop_last": True, "pin_memory": False,
                 "augmentations": [],
                 "data_collate": {"NumpyPadding": {"name_value_pairs": {"textline_encoding": 0.0,
                                                                        "adjacency_matrix": 0.0, "node_label": -100.0},
                                                   "only_selected_items": True}},
                 "data_process": {"TextlineEncoding": {"is_normalized_text": True},
                                  "HeuristicGraphBuilder": {"num_edges": 6, "edge_type": "normal_binary"},
                                  "NodeLabeling": {}}}
        cfg = AttrDict({
            "experiment_name": "probe", "seed": 1111, "is_train": True, "output_dir": os.path.join(tmp, "out"),
            "checkpoint_path": None, "num_gpus": 1, "distributed": False, "local_rank": 0, "num_epochs": 1,
            "max_grad_norm": 5.0, "model_dir_name": "models", "capture_train_step": True,
            "data_config": {"dataset": {"type": "DatapileDataset",
                                        "args": {"node_label_padding_value": -100, "other_class_index": None}},
                            "training": split, "validation": dict(split, batch_size=1)},
            "loss": {"type": "CrossEntropyLoss", "args": {}},
            "lr_scheduler": {"type": "DecayLearningRate", "args": {"lr": 0.001, "factor": 0.9, "num_epochs": 100}},
            "optimizer": {"type": "BuitlinOptimizer", "args": {"type_optimizer": "Adam", "lr": 0.001}}})
        torch.manual_seed(0)
        proc = KVProcedure(GraphCNNDropEdge(4369, 53, 6, 256), cfg)
        batches = list(proc.train_loader)
        for i in range(6):
            proc._run_train_step(batches[i % len(batches)])
        torch.cuda.synchronize()
        n = 30
        t = {"total": 0.0, "graph": 0.0, "load": 0.0, "replay_to_loss": 0.0, "metrics": 0.0}
        sg = proc.step_graph
        for i in range(n):
            b = batches[i % len(batches)]
            t0 = time.perf_counter()
            proc._run_train_step(b)
            t["total"] += time.perf_counter() - t0
        key, bk = next(reversed(sg.buckets.items()))  # every batch here has one shape: one bucket
        for i in range(n):
            b = batches[i % len(batches)]
            t0 = time.perf_counter()
            V = b["textline_encoding"].float().to(dev)
            y = b["node_label"].to(dev)
            if bk.A is None:  # the graph is built on the host path, then copied in
                A = batch_graph(b, dev)
                g = proc.model.to_graph(A)
                g.csc()
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            if bk.A is None:
                bk.load(V, g, y)
            else:  # dense: the graph is built inside the replay from the static A
                bk.load_dense(V, b["adjacency_matrix"], y)
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            bk.hip_graph.replay()
            loss = bk.out[0].item()
            t3 = time.perf_counter()
            pred = proc.activator(bk.out[1]).argmax(dim=-1)
            proc._get_metric_scores(pred, bk.y, item_name="Node classification")
            t4 = time.perf_counter()
            t["graph"] += t1 - t0
            t["load"] += t2 - t1
            t["replay_to_loss"] += t3 - t2
            t["metrics"] += t4 - t3
        t["bucket"] = str(key)
        print({k: (round(v / n * 1e3, 3) if isinstance(v, float) else v) for k, v in t.items()}, sg.stats(), flush=True)


if __name__ == "__main__":
    main()
