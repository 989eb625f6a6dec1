"""Key-value prediction (the reference's KVInference,
gnn/inferencer/inference_procedures/kv_inference.py:13-118): one document at
a time, softmax (inference_settings.activation), argmax class and score per
text line, returned as the input boxes annotated with formal_key, key_type
and confidence.  With `graph_parallel: node_range` every rank predicts its
node range of the document's graph (grl.dist.ShardedGraph) and the logits
are all-gathered, so every rank returns the whole document's boxes."""
from __future__ import annotations

from typing import Any, Dict, List

import torch
import torch.nn as nn

from gnn.data_generator.base_dataloader import BaseDataLoader
from gnn.inferencer.inference_procedures.base_procedure import BaseProcedure
from gnn.utils.input_wrapper import cast_label_to_list, handle_single_input
from grl import TypedGraph
from grl.graph import device_check
from grl.layout import edges_to_typed_csr


class KVInference(BaseProcedure):
    def __init__(self, model: nn.Module, config: Dict[str, Any], **kwargs):
        super().__init__(model, config, **kwargs)
        settings = config.inference_settings
        act = settings.get("activation") or {"type": "Softmax", "args": {"dim": -1}}
        self.activator = getattr(torch.nn, act["type"])(**(act.get("args") or {}))
        self.dataloader = BaseDataLoader(config)
        self.dataset = self.dataloader._load_dataset(settings.datasets.type, settings.datasets.args,
                                                     data_type="inference")
        self.id_to_class = dict(self.dataset.id_to_class)
        self.id_to_class[0] = ("other", "other")

    def _graph(self, sample: Dict[str, Any]):
        if "adjacency_matrix" in sample:
            return torch.tensor(sample["adjacency_matrix"], dtype=torch.float, device=self.device).unsqueeze(0)
        n = int(sample["num_nodes"])
        rowptr, colidx = edges_to_typed_csr(sample["typed_edges"], n)
        return TypedGraph.from_csr_host(rowptr, colidx, 6, self.device, num_cols=n, batch_shape=(1, n))

    def _sharded_logits(self, V: torch.Tensor, g) -> torch.Tensor:
        """The model's logits (1, N, C) from this rank's node range of the
        document's graph, all-gathered (graph_parallel: node_range)."""
        from gnn.trainer.training_procedures.kv_procedure import sharded_graph_cached

        if not isinstance(g, TypedGraph):
            g = TypedGraph.from_dense(g, layout="bnln")
        sg = sharded_graph_cached(self, g, self.config.get("graph_parallel_args") or {})
        rb, re = sg.plan.row_begin, sg.plan.row_end
        rows = self.model([V.reshape(-1, V.shape[-1])[rb:re], sg])
        return sg.gather_rows(rows.reshape(re - rb, -1)).unsqueeze(0)

    def step_process(self, sample: Dict[str, Any]) -> List[Dict[str, Any]]:
        raw = sample["label"]
        V = torch.tensor(sample["textline_encoding"], dtype=torch.float, device=self.device).unsqueeze(0)
        g = self._graph(sample)
        logits = self.activator(self._sharded_logits(V, g) if self.graph_parallel else self.model([V, g]))
        scores, classes = logits.max(dim=-1)
        classes = classes.reshape(-1).cpu().tolist()
        scores = scores.reshape(-1).cpu().tolist()
        device_check(self.device)  # synced already: surface a kernel's stream-ordered failure
        if not (len(raw) == len(classes) == len(scores)):
            raise ValueError(f"{len(raw)} boxes but {len(classes)} predictions")
        out = []
        for i, (cls_idx, score) in enumerate(zip(classes, scores)):
            box = raw[i]
            box["formal_key"], box["key_type"] = self.id_to_class[cls_idx]
            box["confidence"] = score
            out.append(box)
        for post in self.post_processors:
            out = post(out)
        return out

    @handle_single_input(cast_label_to_list)
    def __call__(self, samples: List[Any]) -> List[List[Dict[str, Any]]]:
        self.model.eval()
        self.dataset.list_samples = self.dataset._load_samples(samples)
        with torch.no_grad():
            return [self.step_process(self.dataset[i]) for i in range(len(self.dataset))]
