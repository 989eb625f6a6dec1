"""Loss registry (config loss.type).  CrossEntropyLoss matches the
reference's wrapper (gnn/trainer/losses/cross_entropy_loss.py:9-35): logits
(B, N, C) are transposed to (B, C, N) for torch's criterion, optional class
weights, ignore_index -100 (torch's default) for padded nodes."""
from typing import Any, Dict, List

import numpy as np
import torch


class BaseLoss(torch.nn.Module):
    @classmethod
    def _from_config(cls, config: Dict[str, Any]) -> "BaseLoss":
        return cls(**(config or {}))


class CrossEntropyLoss(BaseLoss):
    def __init__(self, weight: List[float] = None):
        super().__init__()
        w = torch.from_numpy(np.array(weight, dtype=np.float32)) if weight is not None else None
        self.criterion = torch.nn.CrossEntropyLoss(w)

    def forward(self, pred: torch.Tensor, target: torch.Tensor, **kwargs) -> torch.Tensor:
        if self.criterion.weight is not None and self.criterion.weight.device != pred.device:
            self.criterion = self.criterion.to(pred.device)
        return self.criterion(pred.transpose(1, 2), target)
