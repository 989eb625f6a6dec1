"""CPU-only: the native layout-graph builder (libgrl grl_layout_graph_*)
against the reference's own HeuristicGraphBuilder output
(tests/golden/layout_graphs.npz, make_golden.py): bitwise on the fp16
adjacency for all three edge types, incl. debug.json and pages with
"cell"/"table" items, empty texts and fractional coordinates."""
import json

import numpy as np
import pytest

import inputs as gi
from grl.layout import edges_to_typed_csr, layout_adjacency, layout_edges, layout_size

PAGES = ["debug"] + list(gi.LAYOUT_CASES)


@pytest.fixture(scope="module")
def fixtures(golden):
    return golden("layout_graphs.npz")


def _regions(fx, name):
    regs = json.loads(str(fx[f"{name}::regions"]))
    return [{"polygon": r["location"], "text": r["text"], "label": r.get("label", "other")} for r in regs]


@pytest.mark.parametrize("name", PAGES)
def test_normal_binary_matches_reference(fixtures, name):
    regs = _regions(fixtures, name)
    ref = fixtures[f"{name}::normal_binary"]
    adj = layout_adjacency(regs, "normal_binary")
    assert adj.dtype == np.float16 and adj.shape == ref.shape
    np.testing.assert_array_equal(adj != 0, ref)
    assert set(np.unique(adj)) <= {np.float16(0), np.float16(1)}


@pytest.mark.parametrize("name", ["plain30", "cells60", "tiny2", "tables40"])
@pytest.mark.parametrize("et", ["fc_similarity", "fc_binary"])
def test_fully_connected_matches_reference(fixtures, name, et):
    regs = _regions(fixtures, name)
    ref = fixtures[f"{name}::{et}"]
    adj = layout_adjacency(regs, et)
    if et == "fc_similarity":
        np.testing.assert_array_equal(adj.view(np.uint16), ref)  # bitwise fp16
    else:
        np.testing.assert_array_equal(adj != 0, ref)


@pytest.mark.parametrize("name", PAGES)
def test_edge_list_is_the_dense_graph(fixtures, name):
    regs = _regions(fixtures, name)
    edges, n = layout_edges(regs)
    ref = fixtures[f"{name}::normal_binary"]
    assert n == ref.shape[0] == layout_size(regs)
    s, t, d = np.nonzero(ref)
    np.testing.assert_array_equal(edges, np.stack([s, t, d], 1).astype(np.int32))
    rowptr, colidx = edges_to_typed_csr(edges, n)
    assert rowptr[-1] == len(edges)
    for k in range(0, len(edges), max(1, len(edges) // 17)):
        si, ti, di = edges[k]
        seg = si * 6 + ti
        assert di in colidx[rowptr[seg]:rowptr[seg + 1]]


def test_debug_json_edge_counts(fixtures):
    edges, n = layout_edges(_regions(fixtures, "debug"))
    assert n == 74 and len(edges) == 216
    assert np.bincount(edges[:, 1], minlength=6).tolist() == [43, 43, 65, 65, 0, 0]


def test_empty_and_bad_input():
    assert layout_adjacency([], "normal_binary").shape == (0, 6, 0)
    from grl import GrlError

    with pytest.raises(GrlError, match="Invalid edge type"):
        layout_adjacency([], "bogus")
