"""Optimizer registry (config optimizer.type).  BuitlinOptimizer (sic, the
reference's class name: gnn/trainer/optimizers/builtin_optimizer.py:9-26)
instantiates torch.optim.<type_optimizer>(params, **kwargs); like the
reference it does not forward `lr` (the epoch LR schedule sets it)."""
from typing import Any, Dict

import torch


class BaseOptimizer:
    @classmethod
    def _from_config(cls, config: Dict[str, Any]) -> "BaseOptimizer":
        return cls(**(config or {}))


class BuitlinOptimizer(BaseOptimizer):
    def __init__(self, type_optimizer: str, lr: float, **kwargs):
        self.learning_rate = lr
        self.type_optimizer = type_optimizer
        self.optimizer_args = kwargs

    def get_optimizer(self, parameters) -> torch.optim.Optimizer:
        return getattr(torch.optim, self.type_optimizer)(parameters, **self.optimizer_args)
