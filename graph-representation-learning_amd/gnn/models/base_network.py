"""BaseNetwork with the reference's config-driven constructor.

Mirrors gnn/models/base_network.py:9-56 of the reference: the same
`_from_config({"type", "args"})` lookup, the same KeyError / TypeError
messages for a missing class or bad kwargs, and the same trainable-parameter
count string.  Logging goes to the stdlib logger (the reference's
colorlog/file handlers are I/O, outside this engine's scope).
"""
from __future__ import annotations

import logging
from typing import Any, Dict

import torch.nn as nn


class BaseNetwork(nn.Module):
    def __init__(self):
        super().__init__()
        self.logger = logging.getLogger(type(self).__module__)

    @classmethod
    def _from_config(cls, config: Dict[str, Any]) -> "BaseNetwork":
        from gnn import models

        name = config["type"]
        model_class = getattr(models, name, None)
        if model_class is None:
            raise KeyError(f"Cannot find {name} class. "
                           f"Make sure to import this class in {models.__name__}.__init__.py.")
        if cls is BaseNetwork:
            return model_class._from_config(config)
        kwargs = config.get("args", {}) or {}
        try:
            model = model_class(**kwargs)
        except TypeError as err:
            raise TypeError(f"{err}. Check `args` fields defined in config with the actual keyword args "
                            f"required in {model_class.__name__} `__init__` method.")
        model.logger.info(f"Num parameters of {model.__class__.__name__}: {model._count_parameters()}")
        return model

    def _count_parameters(self) -> str:
        return f"{sum(p.numel() for p in self.parameters() if p.requires_grad):,}"

    def forward(self, *args, **kwargs):
        raise NotImplementedError
