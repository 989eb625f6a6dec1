"""Optimizer registry (config optimizer.type).  BuitlinOptimizer (sic, the
reference's class name: gnn/trainer/optimizers/builtin_optimizer.py:9-26)
instantiates torch.optim.<type_optimizer>(params, **kwargs); like the
reference it does not forward `lr` (the epoch LR schedule sets it).  Adam /
AdamW over device parameters run torch's fused implementation (the same
update rule) unless the config names fused / foreach itself."""
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
        kwargs = dict(self.optimizer_args)
        params = list(parameters)
        if (self.type_optimizer in ("Adam", "AdamW") and "fused" not in kwargs and "foreach" not in kwargs and params
                and all(p.is_cuda and p.dtype.is_floating_point for p in params)):
            # the same update rule as one kernel over every parameter, instead of torch's per-tensor launches
            # (19 parameters: 0.05 vs 0.34 ms a step on the device, tools/probe_adam_capturable.py)
            kwargs["fused"] = True
        return getattr(torch.optim, self.type_optimizer)(params, **kwargs)
