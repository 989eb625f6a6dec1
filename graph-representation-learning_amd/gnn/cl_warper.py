"""GNNLearningWarper: the reference's public train/predict API
(gnn/cl_warper.py:19-115) over the MI355X engine.

    warper = GNNLearningWarper(model, config_path="configs/x.yaml")   # or config=AttrDict/dict
    warper.train()              # -> final validation macro F1 (KVProcedure.__call__)
    warper.predict(samples)     # -> annotated boxes (KVInference.__call__)

Config keys, seeding, output-dir layout and the procedure registry follow
the reference.  Differences: YAML is read with yaml.safe_load into an
attribute dict (anyconfig/munch are not installed); there is no Neptune run
and no tensorboard writer (logging is out of scope); with distributed: true
the process group uses backend "nccl" (RCCL on ROCm) exactly as the
reference requests it (cl_warper.py:73-75).
"""
from __future__ import annotations

import logging
import os
import random
from typing import Any, Dict, List, Optional

import numpy as np
import torch
import torch.nn as nn

from gnn.inferencer import inference_procedures
from gnn.trainer import training_procedures
from gnn.utils.checkpoint_handler import CheckpointHandler
from gnn.utils.config import AttrDict, load_config


class GNNLearningWarper:
    def __init__(self, model: nn.Module, config_path: Optional[str] = None, config: Optional[Dict] = None):
        if not (config_path or config is not None):
            raise AssertionError("GNNLearningWarper needs config_path or config")
        self.model = model
        self.device = torch.device("cuda" if torch.cuda.is_available() else "cpu")
        self.config = self._from_config(config_path) if config_path else self._prepare(AttrDict(config))
        random.seed(self.config.seed)
        np.random.seed(self.config.seed)
        torch.manual_seed(self.config.seed)
        if torch.cuda.is_available():
            torch.cuda.manual_seed_all(self.config.seed)
        self.config.output_dir = self._make_output_dir()
        os.environ["OUTPUT_DIR"] = self.config.output_dir
        self.logger = logging.getLogger(__name__)
        self.checkpointer = CheckpointHandler()
        ptype = self.config.procedure.type
        pargs = self.config.procedure.get("args") or {}
        if self.config.is_train:
            self.trainer = getattr(training_procedures, ptype)._from_config(self.model, self.config, ems_exp=None,
                                                                           **pargs)
        else:
            self.inferencer = getattr(inference_procedures, ptype)._from_config(self.model, self.config, **pargs)

    @staticmethod
    def _prepare(cfg: AttrDict) -> AttrDict:
        if cfg.get("distributed"):
            # cl_warper.py:73-75.  local_rank maps onto the visible devices (several
            # ranks may share one GPU in tests); the group is created unless the
            # caller already did; `dist_backend` (additive, default "nccl" = RCCL).
            n = torch.cuda.device_count()
            if n:
                torch.cuda.set_device(int(cfg.local_rank) % n)
            if not torch.distributed.is_initialized():
                torch.distributed.init_process_group(backend=cfg.get("dist_backend", "nccl"), init_method="env://")
        torch.backends.cudnn.benchmark = bool(cfg.get("benchmark", False))
        torch.backends.cudnn.deterministic = bool(cfg.get("deterministic", False))
        return cfg

    @staticmethod
    def _from_config(config_path: str) -> AttrDict:
        return GNNLearningWarper._prepare(load_config(config_path))

    def _make_output_dir(self) -> str:
        out = os.path.join(self.config.output_dir, self.config.experiment_name)
        os.makedirs(out, exist_ok=True)
        return out

    def train(self) -> Any:
        return self.trainer()

    def predict(self, samples: List[Any]) -> List[Any]:
        return self.inferencer(samples)
