"""Shared inference setup (the reference's inference BaseProcedure,
gnn/inferencer/inference_procedures/base_procedure.py:13-144): output dir,
device from inference_settings.num_gpus, checkpoint restore, post-processors.
Additive: `graph_parallel: node_range` with `distributed: true` predicts
each document's graph as node-range shards, one per rank (KVInference), on
the rank's own device."""
from __future__ import annotations

import logging
import os
from typing import Any, Dict, List, Tuple

import torch
import torch.nn as nn

from gnn.inferencer import post_processing
from gnn.utils.checkpoint_handler import CheckpointHandler
from gnn.utils.config import node_range_parallel


class BaseProcedure:
    def __init__(self, model: nn.Module, config: Dict[str, Any], **kwargs):
        self.logger = logging.getLogger(type(self).__module__)
        self.config = config
        self.checkpointer = CheckpointHandler()
        self.graph_parallel = node_range_parallel(config) and torch.distributed.is_available() \
            and torch.distributed.is_initialized()
        settings = config.inference_settings
        self.inference_dir = os.path.join(config.output_dir, settings.get("output_dir_name", "inference"))
        os.makedirs(self.inference_dir, exist_ok=True)
        self.device, self.device_ids = self._prepare_device(settings.get("num_gpus", 1))
        self.model = self._load_prev_checkpoint(model).to(self.device)
        self.post_processors = [getattr(post_processing, name)._from_config(args)
                                for name, args in (settings.get("post_processing") or {}).items()]

    @classmethod
    def _from_config(cls, model: nn.Module, config: Dict[str, Any], **kwargs) -> "BaseProcedure":
        return cls(model, config, **kwargs)

    def _prepare_device(self, n_gpu_use: int) -> Tuple[torch.device, List[int]]:
        n_gpu = torch.cuda.device_count()
        n_gpu_use = min(n_gpu_use, n_gpu)
        if self.graph_parallel and n_gpu_use > 0:  # one rank per GPU: the device the warper set for this rank
            return torch.device("cuda", torch.cuda.current_device()), [torch.cuda.current_device()]
        return torch.device("cuda:0" if n_gpu_use > 0 else "cpu"), list(range(n_gpu_use))

    def _load_prev_checkpoint(self, model: nn.Module) -> nn.Module:
        path = self.config.get("checkpoint_path")
        if path:
            ckpt = self.checkpointer.restore_checkpoint(path)
            if ckpt.get("state_dict") and ckpt.get("config"):
                model.load_state_dict(ckpt["state_dict"], strict=False)
        return model

    def __call__(self, samples):
        raise NotImplementedError
