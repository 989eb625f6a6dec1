"""Key-value node classification training loop (the reference's KVProcedure,
gnn/trainer/training_procedures/kv_procedure.py:19-377).

Per batch: V, A to the device, model.forward([V, A]) (the GraphCNNDropEdge
hot path on libgrl), CE loss, backward, clip_grad_norm_, optimizer step;
macro P/R/F1 over non-padding, non-"other" nodes; validation each epoch;
checkpoint on best validation loss.  Additive: a batch produced by
TypedEdgePadding carries "typed_edges" instead of a dense adjacency and is
turned into a TypedGraph directly (O(E) host->device instead of O(N^2)).
Additive: with `graph_parallel: node_range` and `distributed: true` each
rank trains and validates on a node range of every batch's graph
(_step_process_shard; base_procedure.py's docstring), for graphs too large
for one GPU; the reference's multi-GPU mode (data parallelism over
documents) stays the default.
"""
from __future__ import annotations

import functools
import math
from collections import defaultdict
from typing import Any, Dict, List, Tuple

import numpy as np
import torch
import torch.nn as nn

from gnn.data_generator.base_dataloader import BaseDataLoader
from gnn.trainer.training_procedures.base_procedure import BaseProcedure
from gnn.utils.config import to_plain
from gnn.utils.metric_tracker import Dictlist
from grl import TypedGraph
from grl.graph import device_check
from grl.layout import edges_to_typed_csr


def batch_graph(batch: Dict[str, Any], device: torch.device, num_types: int = 6):
    """The batch's adjacency for model.forward: dense (B, N, L, N) float, or
    a block-diagonal TypedGraph built from "typed_edges"."""
    if "typed_edges" in batch:
        B, N = (int(x) for x in batch["graph_shape"])
        rowptr, colidx = edges_to_typed_csr(np.asarray(batch["typed_edges"]), B * N, num_types)
        return TypedGraph.from_csr_host(rowptr, colidx, num_types, device, num_cols=B * N, batch_shape=(B, N))
    return batch["adjacency_matrix"].float().to(device)


def sharded_graph_cached(owner, graph: TypedGraph, args: Dict[str, Any]):
    """This rank's node-range shard of `graph` (graph_parallel: node_range),
    from a small per-owner cache bucketed on the graph's structure
    (ShardedGraph.cache_key) and confirmed by exact equality of the CSR
    arrays (ShardedGraph.same_graph): a graph met again reuses its shard
    plan; a different graph whose key collides gets its own plan.  Every
    rank holds the same graph, so every rank takes the same branch."""
    from collections import OrderedDict

    from grl.dist import ShardedGraph

    kw = {"balance": args.get("balance", "edges"), "halo": args.get("halo", "auto")}
    cache = owner.__dict__.setdefault("_shard_cache", OrderedDict())
    key = ShardedGraph.cache_key(graph, **kw)
    hit = cache.get(key)
    if hit is not None and ShardedGraph.same_graph(hit[1], graph):
        sg = hit[0]
    else:
        sg = ShardedGraph.from_graph(graph, **kw)
        cache[key] = (sg, graph)
        while len(cache) > 4:
            cache.popitem(last=False)
    cache.move_to_end(key)
    return sg


@functools.lru_cache(maxsize=16)
def _label_map(names: Tuple[str, ...]):
    """class id -> label index in sorted-name order (sklearn works on the names: equal names are one
    label), and the label count; built once per class list, not on every step."""
    uniq = sorted(set(names))
    pos = {nm: j for j, nm in enumerate(uniq)}
    idmap = np.array([pos[nm] for nm in names], dtype=np.int64)
    idmap.setflags(write=False)
    return idmap, len(uniq)


def macro_report(y_true: np.ndarray, y_pred: np.ndarray, names) -> Dict[str, Any]:
    """sklearn's classification_report(true_names, pred_names, output_dict=True,
    zero_division=0)["macro avg"] (the reference's per-step metric,
    kv_procedure.py:83-96) from class ids with bincounts: the labels are the
    names present in either list, in sorted-name order; per label precision
    tp / predicted, recall tp / true, F1 2 tp / (true + predicted), 0 on a
    zero denominator; the macro value is numpy's mean over the labels in that
    order -- the same operations as sklearn 1.7's, so the same floats
    (tests/test_data_pipeline.py checks it against sklearn), at ~1/100 of
    its host time (it ran on every training step)."""
    if y_true.size == 0 and y_pred.size == 0:
        return {"precision": 0.0, "recall": 0.0, "f1-score": 0.0, "support": 0.0}
    idmap, U = _label_map(tuple(names))
    yt, yp = idmap[y_true], idmap[y_pred]
    true_sum = np.bincount(yt, minlength=U)
    pred_sum = np.bincount(yp, minlength=U)
    tp_sum = np.bincount(yt[yt == yp], minlength=U)
    present = (true_sum + pred_sum) > 0  # labels in either list, sorted by name
    t, pr, tp = true_sum[present], pred_sum[present], tp_sum[present]

    def div(num, den):
        den = den.astype(np.float64)
        mask = den == 0
        den[mask] = 1
        out = num.astype(np.float64) / den
        out[mask] = 0.0
        return out

    precision = div(tp, pr)
    recall = div(tp, t)
    f1 = div(2.0 * tp.astype(np.float64), 1.0 * t.astype(np.float64) + pr.astype(np.float64))
    return {"precision": float(np.average(precision)), "recall": float(np.average(recall)),
            "f1-score": float(np.average(f1)), "support": float(t.sum())}


class KVProcedure(BaseProcedure):
    def __init__(self, model: nn.Module, config: Dict[str, Any], ems_exp: Any = None, **kwargs):
        super().__init__(model, config, ems_exp, **kwargs)
        self.global_step = 0
        self.activator = torch.nn.Softmax(dim=2)
        self.train_loader, self.val_loader, self.class_names = self._init_dataloaders()
        # additive config key capture_train_step: "capture" (the default on a ROCm
        # device when the key is absent) replays each batch shape's training step as one HIP graph
        # from its second occurrence on (step_graph.py; ineligible batches run
        # eagerly); false opts out (the reference's eager step); "static" runs the
        # same static-buffer step eagerly (the replays' parity reference)
        from gnn.trainer.training_procedures.step_graph import StepGraph, as_mode

        mode = as_mode(config.get("capture_train_step", "capture" if self.device.type == "cuda" else None))
        if self.graph_parallel:  # the sharded step exchanges halos through collectives: eager
            mode = None
        self.step_graph = StepGraph(self, mode) if mode else None

    def _init_dataloaders(self):
        loader = BaseDataLoader(self.config)
        dcfg = self.config.data_config
        train_ds = loader._load_dataset(dcfg.dataset.type, dcfg.training, data_type="training")
        val_ds = loader._load_dataset(dcfg.dataset.type, dcfg.validation, data_type="validation")
        names = ["other"] + ["_".join(v) for _, v in sorted(train_ds.id_to_class.items())]
        return (loader._get_dataloader(train_ds, train_ds.data_config),
                loader._get_dataloader(val_ds, val_ds.data_config), tuple(names))

    def _get_metric_scores(self, preds: torch.Tensor, gts: torch.Tensor,
                           item_name: str = "item") -> Tuple[Dict[str, Any], Dict[str, Any]]:
        both = torch.stack([preds.reshape(-1), gts.reshape(-1).to(preds.dtype)]).cpu().numpy()  # one device sync
        y_pred, y_true = both[0], both[1]
        args = self.config.data_config.dataset.get("args") or {}
        ignore = [args.get("node_label_padding_value", -100), args.get("other_class_index")]
        keep = np.isin(y_true, [v for v in ignore if v is not None], invert=True)
        yp, yt = y_pred[keep], y_true[keep]
        pred_names = [self.class_names[i] for i in yp.tolist()]
        true_names = [self.class_names[i] for i in yt.tolist()]
        scores = macro_report(yt, yp, self.class_names)
        return ({f"{item_name}_{k}": v for k, v in scores.items()}, {"pred": pred_names, "lbl": true_names})

    def _step_process(self, batch: Dict[str, Any], **kwargs):
        if self.graph_parallel:
            return self._step_process_shard(batch)
        V = batch["textline_encoding"].float().to(self.device)
        A = batch_graph(batch, self.device)
        targets = batch["node_label"].to(self.device)
        logits = self.model.forward([V, A])
        loss = self.criterion(logits, targets)
        predicts = self.activator(logits).argmax(dim=-1)
        scores, items = self._get_metric_scores(predicts, targets, item_name="Node classification")
        scores["loss"] = loss.item()
        if not torch.is_grad_enabled():
            # validation: the step already synced, surface a kernel's stream-ordered failure here (a
            # training step checks once, after backward: _run_train_step)
            device_check(self.device)
        return loss, scores, items

    def _step_process_shard(self, batch: Dict[str, Any]):
        """_step_process on this rank's node range of the batch's graph
        (graph_parallel: node_range; batch_size 1: the model's attention is a
        softmax over one graph); rank r runs the model on rows [b_r, b_{r+1})
        (GraphCNNDropEdge.forward([V_rows, ShardedGraph]): halo exchanges
        inside, softmax of the attention over every node).  The returned loss
        is this rank's share -- the criterion on its rows, weighted by its
        rows' share of the batch's weighted targets -- so the ranks' losses
        (and, summed, their gradients) are the one-process step's.  Metrics
        and the reported loss are those of the whole batch on every rank."""
        from grl.dist import all_reduce_sum

        V = batch["textline_encoding"].float().to(self.device)
        A = batch_graph(batch, self.device)
        if not isinstance(A, TypedGraph):  # the collate's dense (B, N, L, N) batch
            A = TypedGraph.from_dense(A, layout="bnln")
        targets = batch["node_label"].to(self.device)
        B, N = targets.shape[0], targets.shape[1]
        if B != 1:  # NodeSelfAtten's softmax runs per page; a shard's runs over its whole graph
            raise ValueError(f"graph_parallel: node_range trains one graph per step (batch_size: 1), got {B}")
        sg = sharded_graph_cached(self, A, self.config.get("graph_parallel_args") or {})
        rb, re = sg.plan.row_begin, sg.plan.row_end
        logits = self.model.forward([V.reshape(B * N, -1)[rb:re], sg]).reshape(1, re - rb, -1)
        t_rows = targets.reshape(1, -1)[:, rb:re]
        loss = self._shard_loss(logits, t_rows, targets)
        logits_all = sg.gather_rows(logits.detach().reshape(re - rb, -1)).reshape(B, N, -1)
        predicts = self.activator(logits_all).argmax(dim=-1)
        scores, items = self._get_metric_scores(predicts, targets, item_name="Node classification")
        scores["loss"] = float(all_reduce_sum(loss.detach().clone().reshape(1)).item())
        if not torch.is_grad_enabled():  # as _step_process: training steps check after backward
            device_check(self.device)
        return loss, scores, items

    def _shard_loss(self, logits: torch.Tensor, t_rows: torch.Tensor, targets: torch.Tensor) -> torch.Tensor:
        """This rank's share of a mean-reduced criterion: its rows' loss times
        their share of the batch's target weight (valid targets, or their
        class weights), so the shares add up to the whole batch's mean."""
        inner = getattr(self.criterion, "criterion", self.criterion)
        if getattr(inner, "reduction", "mean") != "mean":
            return self.criterion(logits, t_rows)
        ignore = getattr(inner, "ignore_index", None)
        weight = getattr(inner, "weight", None)

        def mass(t: torch.Tensor) -> torch.Tensor:
            valid = t != ignore if ignore is not None else torch.ones_like(t, dtype=torch.bool)
            if weight is None:
                return valid.sum().to(torch.float32)
            w = weight.to(t.device)[t.clamp(min=0)]
            return torch.where(valid, w, torch.zeros((), device=t.device)).sum()

        m_loc, m_all = mass(t_rows), mass(targets)
        if float(m_loc) == 0.0:  # no labelled row here: a zero share that still reaches every parameter's graph
            return logits.sum() * 0.0
        return self.criterion(logits, t_rows) * (m_loc / m_all)

    def _run_train_step(self, batch: Dict[str, Any], **kwargs):
        if self.step_graph is not None:
            out = self.step_graph.run(batch)
            if out is not None:  # forward .. optimizer step done (replayed or static); metrics outside the graph
                loss, logits, targets = out
                predicts = self.activator(logits).argmax(dim=-1)
                scores, items = self._get_metric_scores(predicts, targets, item_name="Node classification")
                scores["loss"] = loss.item()
                # a captured step replays forward .. optimizer step as one graph: its stream-ordered
                # failure report is read only here, AFTER the update (a poisoned step's weights are
                # NaN by then; the error still stops training)
                device_check(self.device)
                return scores, items
        self.model.train()
        self.optimizer.zero_grad()
        with torch.set_grad_enabled(True):
            loss, scores, items = self._step_process(batch, **kwargs)
            loss.backward()
            self._sync_gradients()
            device_check(self.device)  # a poisoned (NaN) backward must not reach the weights
            nn.utils.clip_grad_norm_(self.model.parameters(), self.config.max_grad_norm)
            self.optimizer.step()
        return scores, items

    def _run_val_step(self, batch: Dict[str, Any], **kwargs):
        self.model.eval()
        with torch.set_grad_enabled(False):
            _, scores, items = self._step_process(batch, **kwargs)
        return scores, items

    def cosine_schedule_lambda(self, step: int, epoch: int, total_steps: int, base_value: float, max_value: float,
                               warmup_steps: int = 0) -> float:
        """Linear warm-up then cosine annealing (kv_procedure.py:264-292); the
        value is stored on model.lambda_value each step like the reference."""
        step = max(0, min(step, total_steps))
        warmup_steps = min(warmup_steps, total_steps)
        if step < warmup_steps:
            return base_value + (max_value - base_value) * (step / warmup_steps)
        progress = float(step - warmup_steps) / float(max(1, total_steps - warmup_steps))
        return base_value + 0.5 * (max_value - base_value) * (1 + math.cos(math.pi * progress))

    def _optimize_per_epoch(self, epoch: int) -> Dict[str, Any]:
        from sklearn.metrics import classification_report

        train = Dictlist()
        sampler = getattr(self.train_loader, "sampler", None)
        if hasattr(sampler, "set_epoch"):  # DistributedSampler: a new shuffle every epoch, same on every rank
            sampler.set_epoch(epoch)
        for batch in self.train_loader:
            scores, _ = self._run_train_step(batch)
            train._update(scores)
            self.tb_writer.add_scalar("Train_step_loss", scores["loss"], self.global_step)
            if self.step_graph is None:  # a captured step's .grad buffers belong to its graph
                self.model.zero_grad()
            self.global_step += 1
            n = len(self.train_loader)
            self.model.lambda_value = self.cosine_schedule_lambda(self.global_step, epoch, self.config.num_epochs * n,
                                                                  base_value=1e-4, max_value=1.0, warmup_steps=5 * n)
        self.logger.info(f"Training epoch: {epoch} step: {self.global_step} metrics: {train._result() if train else {}}")
        val = Dictlist()
        items: Dict[str, List[str]] = defaultdict(list)
        for batch in self.val_loader:
            scores, vitems = self._run_val_step(batch)
            val._update(scores)
            for k, v in vitems.items():
                items[k].extend(v)
        val_metrics = val._result() if val else {"loss": float("inf")}
        report = classification_report(items["lbl"], items["pred"], output_dict=True, zero_division=0) \
            if items["lbl"] else {"macro avg": {"precision": 0.0, "recall": 0.0, "f1-score": 0.0, "support": 0}}
        macro = dict(report["macro avg"])
        macro["loss"] = val_metrics["loss"]
        self.logger.info(f"Validation metrics: {val_metrics}")
        return macro

    def __call__(self) -> float:
        best = float("inf")
        self.model.zero_grad()
        metrics: Dict[str, Any] = {"f1-score": 0.0}
        for epoch in range(self.config.num_epochs):
            metrics = self._optimize_per_epoch(epoch)
            if self.lr_scheduler is not None:
                self._update_learning_rate(epoch, self.global_step)
            if metrics["loss"] < best:
                best = metrics["loss"]
                if self.rank == 0:
                    self.checkpointer.save_checkpoint(
                        {"epoch": epoch, "config": to_plain(self.config), "meta_data": to_plain(metrics),
                         "state_dict": self.model.state_dict()}, self.model_dir)
        device_check(self.device)  # the last step's backward
        self.tb_writer.close()
        return metrics["f1-score"]
