"""Loss registry (config loss.type).  CrossEntropyLoss matches the
reference's wrapper (gnn/trainer/losses/cross_entropy_loss.py:9-35): the
mean cross entropy of logits (B, N, C) against (B, N) labels (the reference
transposes to (B, C, N); here the rows are flattened: the same terms and
mean), optional class weights, ignore_index -100 (torch's default) for
padded nodes."""
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
        # the reference's criterion(pred.transpose(1, 2), target) over (B, C, N) -- the same mean over the
        # same (weighted, non-ignored) nodes, computed on the (B*N, C) rows: torch's last-dim log-softmax
        # instead of its strided "spatial" kernel (27 us forward + 27 us backward per C1 step)
        return self.criterion(pred.reshape(-1, pred.shape[-1]), target.reshape(-1))
