"""Checkpoint save/restore (the reference's CheckpointHandler,
gnn/utils/checkpoint_handler.py:9-60): `<dir>/model_latest.pt` holding
{"epoch", "config", "meta_data", "state_dict"}.  Configs are stored as plain
dicts so checkpoints load with torch.load(weights_only=True)."""
import logging
import os
from typing import Any, Dict

import torch


class CheckpointHandler:
    def __init__(self):
        self.device = torch.device("cuda" if torch.cuda.is_available() else "cpu")
        self.logger = logging.getLogger(__name__)

    @staticmethod
    def make_checkpoint_name(name: str, epoch: int = None, step: int = None) -> str:
        if epoch is None or step is None:
            return f"{name}_latest.pt"
        return f"{name}_epoch_{epoch}_minibatch_{step}.pt"

    def save_checkpoint(self, checkpoint: Dict[str, Any], output_path: str, epoch: int = None,
                        step: int = None) -> str:
        os.makedirs(output_path, exist_ok=True)
        path = os.path.join(output_path, self.make_checkpoint_name("model", epoch, step))
        torch.save(checkpoint, path)
        self.logger.info("Saving checkpoint success!")
        return path

    def restore_checkpoint(self, checkpoint_path: str) -> Dict[str, Any]:
        ckpt = torch.load(checkpoint_path, map_location=self.device, weights_only=True)
        self.logger.info("Loading checkpoint success!")
        return ckpt
