"""CPU-only: the drop-in keeps the reference's Python surface -- registry,
constructor signature, module tree, state_dict keys/shapes and init RNG
(gnn/models/base_network.py:15-47, drop_robust_gcn.py:32-59,
robust_gcn.py:15-30)."""
import hashlib

import numpy as np
import pytest
import torch

import gnn.models as models
from gnn.models import BaseNetwork, GraphCNNDropEdge, GraphConv
from grl import GrlError, TypedGraph


def test_registry_from_config():
    m = BaseNetwork._from_config({"type": "GraphCNNDropEdge",
                                  "args": {"input_dim": 40, "output_dim": 5, "num_edges": 6, "net_size": 16}})
    assert isinstance(m, GraphCNNDropEdge)
    assert isinstance(models.GraphCNNDropEdge, type)
    with pytest.raises(KeyError, match="Cannot find NoSuchNet"):
        BaseNetwork._from_config({"type": "NoSuchNet", "args": {}})
    with pytest.raises(TypeError, match="Check `args` fields"):
        BaseNetwork._from_config({"type": "GraphCNNDropEdge", "args": {"bogus": 1}})


def test_state_dict_and_init_rng_match_reference(golden):
    g = golden("model_debug.npz")
    torch.manual_seed(0)
    model = GraphCNNDropEdge(4369, 53, 6, 256)
    sd = model.state_dict()
    assert list(sd.keys()) == [str(k) for k in g["sd_keys"]]
    for (k, v), ref_sha in zip(sd.items(), g["sd_sha256"]):
        assert hashlib.sha256(v.contiguous().numpy().tobytes()).hexdigest() == str(ref_sha), k
    # trainable count as the reference logs it
    assert model._count_parameters() == "3,108,821"
    assert sum(p.numel() for p in model.parameters()) == 3_272_661


def test_small_model_init_matches_reference(golden):
    g = golden("model_small_train.npz")
    torch.manual_seed(1)
    model = GraphCNNDropEdge(64, 7, 6, net_size=32)
    for k, v in model.state_dict().items():
        np.testing.assert_array_equal(v.numpy(), g[f"init::{k}"], err_msg=k)


def test_graphconv_surface():
    torch.manual_seed(0)
    gc = GraphConv(16, 8, 6)
    assert repr(gc) == "GraphConv(in_dim=16, out_dim=8, num_edges=6, bias=True)"
    assert gc.h_weights.shape == (16 * 7, 8) and gc.bias.shape == (8,)
    assert (gc.L, gc.F, gc.C) == (6, 16, 8)
    nb = GraphConv(16, 8, 6, with_bias=False)  # the reference crashes here (robust_gcn.py:30); we do not
    assert nb.bias is None


def test_no_cpu_path():
    """The engine refuses CPU tensors instead of silently computing on the host."""
    gc = GraphConv(4, 4, 2)
    with pytest.raises(GrlError, match="ROCm device"):
        gc(torch.zeros(1, 3, 4), torch.zeros(1, 3, 3, 2))
    with pytest.raises(GrlError, match="ROCm device"):
        TypedGraph.from_dense(torch.zeros(1, 3, 2, 3))
