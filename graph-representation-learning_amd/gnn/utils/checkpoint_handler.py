"""Checkpoint save/restore (the reference's CheckpointHandler,
gnn/utils/checkpoint_handler.py:9-60): `<dir>/model_latest.pt` holding
{"epoch", "config", "meta_data", "state_dict"}.  Configs are stored as plain
dicts so checkpoints load with torch.load(weights_only=True).

Checkpoints written by the reference load too, still weights-only: its
KVProcedure saves `dict(munch_config)` (kv_procedure.py:364-368, config from
munch.munchify at cl_warper.py:72), so nested config values are pickled as
`munch.Munch`, and its metrics come from sklearn as numpy float64 scalars.
Those globals -- munch.Munch rebuilt as an OrderedDict, and numpy's scalar /
dtype reconstructors -- are allow-listed for the load; nothing else is.
"""
import logging
import os
from collections import OrderedDict
from typing import Any, Dict

import numpy as np
import torch


def _reference_globals():
    """(object, pickled name) pairs a reference checkpoint may reference."""
    # munch.Munch (a dict subclass pickled as NEWOBJ + SETITEMS + BUILD(items)) is
    # rebuilt as an OrderedDict: the weights-only unpickler fills only exact
    # dict / OrderedDict instances, and an OrderedDict's BUILD puts the items
    # in its __dict__ as well, so attribute access (cfg.model.type) keeps working.
    out = [(OrderedDict, "munch.Munch"), (OrderedDict, "munch.DefaultMunch"), (OrderedDict, "munch.AutoMunch")]
    try:
        from numpy._core.multiarray import scalar
    except ImportError:  # numpy < 2
        from numpy.core.multiarray import scalar
    out += [(scalar, "numpy.core.multiarray.scalar"), (scalar, "numpy._core.multiarray.scalar"),
            (np.dtype, "numpy.dtype")]
    for name in ("Float64DType", "Float32DType", "Int64DType", "Int32DType", "BoolDType"):
        cls = getattr(getattr(np, "dtypes", None), name, None)
        if cls is not None:
            out.append((cls, f"numpy.dtypes.{name}"))
    return out


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
        with torch.serialization.safe_globals(_reference_globals()):
            ckpt = torch.load(checkpoint_path, map_location=self.device, weights_only=True)
        self.logger.info("Loading checkpoint success!")
        return ckpt
