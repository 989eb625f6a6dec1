"""Shared training setup (the reference's trainer BaseProcedure,
gnn/trainer/training_procedures/base_procedure.py:14-197): output dir,
device choice from num_gpus, checkpoint restore (strict=False), and the
criterion / optimizer / LR schedule resolved by name from config.

Data parallel over documents (`distributed: true`, the reference's
declared-but-broken DDP, base_procedure.py:79-93 / cl_warper.py:73-75):
each rank trains on its DistributedSampler shard; parameters and buffers
are broadcast from rank 0 once, and after every backward the gradients are
averaged over the ranks with one bucketed all-reduce (RCCL), so the
replicas stay identical.  Only rank 0 writes checkpoints.  Every rank is
seeded alike (cl_warper.py:36-40), so after the broadcast each rank's CUDA
generator is re-seeded with seed + rank and its EdgeDropout modules get
stream = rank: ranks draw independent feature-dropout and DropEdge masks
instead of the same ones on different documents.

Node-range graph parallelism (additive `graph_parallel: node_range` with
`distributed: true`; gnn.utils.config.node_range_parallel): every rank loads
the same batches, takes a node range of each batch's graph
(grl.dist.ShardedGraph) and runs the model on its rows; the loss is weighted
so the ranks' losses add up to the one-process loss, and the gradients are
SUMMED over ranks -- the one-process step's.  The ranks then draw the
one-process masks (no per-rank dropout streams: the sharded model's masks
are keyed on global rows / edges and rank 0's seeds)."""
from __future__ import annotations

import logging
import os
from typing import Any, Dict, List, Tuple

import torch
import torch.nn as nn

from gnn.trainer import losses, lr_schedulers, optimizers
from gnn.utils.checkpoint_handler import CheckpointHandler
from gnn.utils.config import node_range_parallel


class NullWriter:
    """Stands in for tensorboardX.SummaryWriter (logging is out of scope)."""

    def add_scalar(self, *args, **kwargs):
        pass

    def add_histogram(self, *args, **kwargs):
        pass

    def close(self):
        pass


class BaseProcedure:
    def __init__(self, model: nn.Module, config: Dict[str, Any], ems_exp: Any = None, **kwargs):
        self.logger = logging.getLogger(type(self).__module__)
        self.config = config
        self.ems_exp = ems_exp
        self.model_dir = self._make_output_dir()
        self.checkpointer = CheckpointHandler()
        self.distributed = bool(config.get("distributed")) and torch.distributed.is_available() \
            and torch.distributed.is_initialized()
        self.rank = torch.distributed.get_rank() if self.distributed else 0
        self.graph_parallel = self.distributed and node_range_parallel(config)
        self.device, self.device_ids = self._prepare_device(config.get("num_gpus", 1))
        self.model = self._load_prev_checkpoint(model).to(self.device)
        if self.distributed:
            from grl.dist import broadcast_module

            broadcast_module(self.model, src=0)
            if not self.graph_parallel:
                self._independent_dropout_streams()
        self.criterion = self._init_criterion()
        self.optimizer = self._init_optimizer()
        self.lr_scheduler = self._init_lr_scheduler()
        self.tb_writer = NullWriter()

    @classmethod
    def _from_config(cls, model: nn.Module, config: Dict[str, Any], ems_exp: Any = None, **kwargs) -> "BaseProcedure":
        return cls(model, config, ems_exp, **kwargs)

    def _prepare_device(self, n_gpu_use: int) -> Tuple[torch.device, List[int]]:
        n_gpu = torch.cuda.device_count()
        if n_gpu_use > 0 and n_gpu == 0:
            self.logger.warning("There's no GPU available on this machine; the MI355X engine will refuse CPU tensors.")
            n_gpu_use = 0
        n_gpu_use = min(n_gpu_use, n_gpu)
        if self.distributed and n_gpu > 0:
            return torch.device("cuda", torch.cuda.current_device()), [torch.cuda.current_device()]
        return torch.device("cuda:0" if n_gpu_use > 0 else "cpu"), list(range(n_gpu_use))

    def _independent_dropout_streams(self) -> None:
        from gnn.models.networks.drop_robust_gcn import EdgeDropout, FeatureDropout

        for m in self.model.modules():
            if isinstance(m, (EdgeDropout, FeatureDropout)):
                m.stream = self.rank
        if self.device.type == "cuda":
            torch.cuda.manual_seed(torch.initial_seed() + self.rank)

    def _sync_gradients(self) -> None:
        """DDP's gradient averaging, as one bucketed all-reduce per step; with
        node-range shards the sum (each rank's gradient is its rows' part)."""
        if self.distributed:
            from grl.dist import allreduce_gradients

            # check=False: the step may be a captured HIP graph (no host wait inside); the procedure checks
            # after the step instead
            allreduce_gradients(self.model.parameters(), average=not self.graph_parallel, check=False)

    @staticmethod
    def _resolve(module, section: Dict[str, Any], what: str):
        if not section or not section.get("type"):
            return None
        cls = getattr(module, section["type"], None)
        if cls is None:
            raise ValueError(f"Cannot find {what} {section['type']}")
        return cls._from_config(section.get("args") or {})

    def _init_criterion(self):
        return self._resolve(losses, self.config.get("loss"), "loss")

    def _init_lr_scheduler(self):
        return self._resolve(lr_schedulers, self.config.get("lr_scheduler"), "lr_scheduler")

    def _init_optimizer(self):
        opt = self._resolve(optimizers, self.config.get("optimizer"), "optimizer")
        return opt.get_optimizer(self.model.parameters()) if opt is not None else None

    def _make_output_dir(self) -> str:
        out = os.path.join(self.config.output_dir, self.config.get("model_dir_name", "models"))
        os.makedirs(out, exist_ok=True)
        return out

    def _load_prev_checkpoint(self, model: nn.Module) -> nn.Module:
        path = self.config.get("checkpoint_path")
        if path:
            ckpt = self.checkpointer.restore_checkpoint(path)
            if ckpt.get("state_dict") and ckpt.get("config"):
                model.load_state_dict(ckpt["state_dict"], strict=False)
                self.logger.info("Loading pretrained model success!")
        return model

    def _update_learning_rate(self, epoch: int, step: int) -> float:
        lr = self.lr_scheduler._step_lr(epoch, step)
        for group in self.optimizer.param_groups:
            if isinstance(group["lr"], torch.Tensor):  # a captured step reads it from device memory
                group["lr"].fill_(float(lr))
            else:
                group["lr"] = lr
        return lr

    def __call__(self):
        raise NotImplementedError
