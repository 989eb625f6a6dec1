"""CheckpointHandler.restore_checkpoint loads checkpoints written the way the
reference writes them (kv_procedure.py:364-368): "config" is dict(munch
config), so nested values are pickled as munch.Munch, and "meta_data" holds
sklearn's numpy float64 scores -- with torch.load(weights_only=True) and an
allow-list, never a full unpickler."""
import pickle
import sys
import types

import numpy as np
import pytest
import torch

from gnn.utils.checkpoint_handler import CheckpointHandler


def _fake_munch_module():
    """A module named `munch` whose Munch pickles like munch 2.x's: a dict
    subclass with __getstate__/__setstate__ over its items."""
    mod = types.ModuleType("munch")

    class Munch(dict):
        def __getattr__(self, k):
            return self[k]

        def __getstate__(self):
            return {k: v for k, v in self.items()}

        def __setstate__(self, state):
            self.clear()
            self.update(state)

    Munch.__module__ = "munch"
    Munch.__qualname__ = "Munch"
    mod.Munch = Munch
    return mod


@pytest.fixture
def reference_style_checkpoint(tmp_path):
    had = sys.modules.get("munch")
    mod = _fake_munch_module()
    sys.modules["munch"] = mod
    try:
        cfg = mod.Munch(experiment_name="kv", num_epochs=2,
                        model=mod.Munch(type="GraphCNNDropEdge", args=mod.Munch(input_dim=8, net_size=4)),
                        optimizer=mod.Munch(type="Adam", args=mod.Munch(lr=1e-3)))
        sd = {"gcn1.h_weights": torch.randn(28, 4), "gcn1.bias": torch.zeros(4)}
        ckpt = {"epoch": 3, "config": dict(cfg), "meta_data": {"f1-score": np.float64(0.75), "loss": 0.5},
                "state_dict": sd}
        path = tmp_path / "model_latest.pt"
        torch.save(ckpt, path)
    finally:
        if had is None:
            del sys.modules["munch"]
        else:
            sys.modules["munch"] = had
    return path, sd


def test_restores_reference_checkpoint_weights_only(reference_style_checkpoint):
    path, sd = reference_style_checkpoint
    assert "munch" not in sys.modules or not hasattr(sys.modules["munch"], "__fake__")
    with pytest.raises(pickle.UnpicklingError):  # the plain weights-only load refuses it
        torch.load(path, weights_only=True)
    ck = CheckpointHandler().restore_checkpoint(str(path))
    assert ck["epoch"] == 3
    assert ck["config"]["model"]["args"]["net_size"] == 4 and ck["config"]["model"].type == "GraphCNNDropEdge"
    assert ck["config"]["optimizer"]["args"]["lr"] == 1e-3
    assert float(ck["meta_data"]["f1-score"]) == 0.75
    for k, v in sd.items():
        assert torch.equal(ck["state_dict"][k].cpu(), v)


def test_other_globals_stay_refused(tmp_path):
    """The allow-list is narrow: an arbitrary class in a checkpoint is still
    refused."""
    path = tmp_path / "evil.pt"
    torch.save({"x": types.SimpleNamespace(a=1)}, path)
    with pytest.raises(pickle.UnpicklingError):
        CheckpointHandler().restore_checkpoint(str(path))
