"""Epoch-level LR schedules (config lr_scheduler.type), as in the reference's
gnn/trainer/lr_schedulers/*: `_step_lr(epoch, step)` returns the new LR."""
from bisect import bisect_right
from typing import Any, Dict, List

import numpy as np


class BaseLearningRate:
    @classmethod
    def _from_config(cls, config: Dict[str, Any]) -> "BaseLearningRate":
        return cls(**(config or {}))

    def _step_lr(self, epoch: int, step: int = None) -> float:
        raise NotImplementedError


class DecayLearningRate(BaseLearningRate):
    """lr0 * (1 - epoch / (num_epochs + 1)) ** factor (decay_lr.py:6-25)."""

    def __init__(self, lr: float = 0.002, factor: float = 0.9, num_epochs: int = 100):
        self.lr = self.initial_lr = lr
        self.factor = factor
        self.epochs = num_epochs

    def _step_lr(self, epoch: int, step: int = None) -> float:
        self.lr = self.initial_lr * np.power(1.0 - epoch / float(self.epochs + 1), self.factor)
        return self.lr


class MultiStepLearningRate(BaseLearningRate):
    def __init__(self, lr: float = 0.001, gamma: float = 0.1, milestones: List[int] = ()):
        self.lr = self.initial_lr = lr
        self.gamma = gamma
        self.milestones = list(milestones)

    def _step_lr(self, epoch: int, step: int = None) -> float:
        self.lr = self.initial_lr * self.gamma ** bisect_right(self.milestones, epoch)
        return self.lr


class WarmupLearningRate(BaseLearningRate):
    def __init__(self, lr: float = 0.001, warmup_lr: float = 1e-5, steps: int = 4000):
        self.lr = self.initial_lr = lr
        self.steps = steps
        self.warmup_learning_rate = warmup_lr

    def _step_lr(self, epoch: int, step: int = None) -> float:
        self.lr = self.warmup_learning_rate if (epoch == 0 and step < self.steps) else self.initial_lr
        return self.lr
