#!/usr/bin/env python
"""Generate the golden parity fixtures from the REFERENCE implementation.

Run in the build container only (it needs /root/reference):
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

It imports the reference's own GraphConv / GraphCNNDropEdge and data
processors (gnn/models/networks/robust_gcn.py, drop_robust_gcn.py,
gnn/data_generator/data_process/*.py) with test-only shims for logging/IO
packages that are not installed here (colorlog, decouple) -- the shims carry
no arithmetic.  Outputs are small .npz files next to this script; no
reference source is copied.  The fixtures are the parity pin for the oracle
(oracle/) and, through it, for the HIP engine.
"""
from __future__ import annotations

import hashlib
import json
import logging
import os
import sys
import types

sys.dont_write_bytecode = True  # never write __pycache__ into /root/reference
os.environ.setdefault("OUTPUT_DIR", "/tmp/grl_golden_logs")

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.abspath(os.path.join(HERE, "..", ".."))
REF = os.environ.get("GRL_REFERENCE", "/root/reference")
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import inputs as gi  # noqa: E402
from oracle import dense_ref  # noqa: E402


def _install_shims():
    """Logging-only stand-ins for third-party packages absent here."""
    if "colorlog" not in sys.modules:
        try:
            import colorlog  # noqa: F401
        except ImportError:
            m = types.ModuleType("colorlog")
            m.basicConfig = lambda **kw: logging.basicConfig(**{k: v for k, v in kw.items() if k != "format"})
            sys.modules["colorlog"] = m
    if "decouple" not in sys.modules:
        try:
            import decouple  # noqa: F401
        except ImportError:
            m = types.ModuleType("decouple")
            m.config = lambda key, default=None, cast=None: os.environ.get(key, default)
            sys.modules["decouple"] = m
    if not hasattr(np, "float"):
        np.float = float  # textline_encoding.py:71 uses the alias removed in numpy >= 1.24


def _import_reference():
    _install_shims()
    os.makedirs(os.environ["OUTPUT_DIR"], exist_ok=True)
    sys.path.insert(0, REF)
    from gnn.models.networks.drop_robust_gcn import GraphCNNDropEdge
    from gnn.models.networks.robust_gcn import GraphConv
    from gnn.data_generator.data_process.heuristic_graph_builder import HeuristicGraphBuilder
    from gnn.data_generator.data_process.textline_encoding import TextlineEncoding
    return GraphConv, GraphCNNDropEdge, HeuristicGraphBuilder, TextlineEncoding


def _t(x):
    return torch.from_numpy(np.ascontiguousarray(x))


def ref_graphconv_case(GraphConv, A_bnln, V, W, b, dout, mult_pre=None):
    """Run the reference GraphConv forward + backward on given inputs."""
    B, N, L, _ = A_bnln.shape
    F = V.shape[-1]
    C = W.shape[1]
    torch.manual_seed(0)
    gcn = GraphConv(F, C, L)
    with torch.no_grad():
        gcn.h_weights.copy_(_t(W))
        gcn.bias.copy_(_t(b))
    Vt = _t(V).requires_grad_(True)
    A_bnnl = _t(A_bnln).permute(0, 1, 3, 2)  # what GraphConv.forward receives (drop_robust_gcn.py:63)
    if mult_pre is None:
        out = gcn(Vt, A_bnnl, True)
    else:
        A_pre = gcn.preprocess_adj(A_bnnl)
        # nn.Dropout arithmetic: input.mul(mask).mul_(scale) -- mult carries mask*scale
        keep = _t((mult_pre != 0).astype(np.float32))
        scale = float(mult_pre.max()) if (mult_pre != 0).any() else 1.0
        A_drop = A_pre.mul(keep).mul_(scale)
        out = gcn(Vt, A_drop, False)
    out.backward(_t(dout))
    return (out.detach().numpy(), Vt.grad.numpy(), gcn.h_weights.grad.numpy(), gcn.bias.grad.numpy())


def make_graphconv_fixtures(GraphConv):
    for name, (seed, B, N, L, F, C, fv, epn) in gi.GRAPHCONV_CASES.items():
        A = gi.random_adj_bnln(seed, B, N, L, epn, float_vals=fv)
        V = gi.features(seed + 1, B, N, F)
        W, b = gi.graphconv_params(seed + 2, F, C, L)
        dout = gi.features(seed + 3, B, N, C)
        de = gi.DROPEDGE
        mult = dense_ref.dropedge_weights_pre(A, de["p"], de["seed"], de["call"], drop_self=True)
        res = {}
        for tag, m in (("eval", None), ("drop", mult)):
            out, dV, dW, db = ref_graphconv_case(GraphConv, A, V, W, b, dout, m)
            res[f"{tag}_out"] = out
            res[f"{tag}_dV"] = dV
            res[f"{tag}_db"] = db
            if dW.size <= 1 << 16:
                res[f"{tag}_dW"] = dW
            pr = gi.probes(seed + 4, dW.shape[1])
            res[f"{tag}_dW_probe"] = dW @ pr  # (K, 4): projections of the full dW
        small = A.size <= 1 << 16
        np.savez_compressed(
            os.path.join(HERE, f"graphconv_{name}.npz"),
            meta=np.array([seed, B, N, L, F, C, int(fv)], dtype=np.int64),
            **({"A": A, "V": V, "W": W, "b": b, "dout": dout} if small else {}),
            **res)
        print(f"graphconv_{name}: out {res['eval_out'].shape} |out| {np.abs(res['eval_out']).max():.3g}")


def debug_graph(HeuristicGraphBuilder, TextlineEncoding):
    """V (N, 4369) and A (N, 6, N) of assets/samples/debug.json through the
    reference's own data processors (cassia layout, as CassiaDataset feeds
    them: gnn/data_generator/datasets/cassia_dataset.py:199-244)."""
    with open(os.path.join(REF, "assets/samples/debug.json"), encoding="utf-8-sig") as f:
        regions = json.load(f)
    with open(os.path.join(REF, "assets/meta_data/master_charset.json"), encoding="utf-8-sig") as f:
        charset = json.load(f)["charset"]
    char_to_id = {c: i for i, c in enumerate(charset)}
    label = {}
    for i, reg in enumerate(regions):
        reg = dict(reg)
        reg["polygon"] = reg["location"]
        label[i] = reg
    sample = {"label": label, "char_to_id": char_to_id}
    sample = TextlineEncoding(is_normalized_text=True)(sample)
    sample = HeuristicGraphBuilder(num_edges=6, edge_type="normal_binary")(sample)
    V = sample["textline_encoding"].astype(np.float32)
    A = sample["adjacency_matrix"]
    return V, A


def make_model_fixtures(GraphCNNDropEdge, HeuristicGraphBuilder, TextlineEncoding):
    V, A16 = debug_graph(HeuristicGraphBuilder, TextlineEncoding)
    N = V.shape[0]
    A = A16.astype(np.float32)
    print(f"debug.json: N={N} V{V.shape} nnz(V)={int((V != 0).sum())} E={int((A != 0).sum())} "
          f"per type {[(int((A[:, t] != 0).sum())) for t in range(A.shape[1])]}")
    # --- full model, config 1: GraphCNNDropEdge(4369, 53, 6, 256), eval ---
    torch.manual_seed(0)
    model = GraphCNNDropEdge(4369, 53, 6, 256)
    model.eval()
    sd = model.state_dict()
    sha = {k: hashlib.sha256(v.detach().contiguous().numpy().tobytes()).hexdigest() for k, v in sd.items()}
    with torch.no_grad():
        logits = model([_t(V)[None], _t(A)[None]]).numpy()[0]
    nzr, nzc = np.nonzero(V)
    np.savez_compressed(
        os.path.join(HERE, "model_debug.npz"),
        V_shape=np.array(V.shape), V_rows=nzr.astype(np.int32), V_cols=nzc.astype(np.int32),
        V_vals=V[nzr, nzc], A_bits=np.packbits(A != 0), A_shape=np.array(A.shape),
        logits=logits, sd_keys=np.array(list(sha.keys())), sd_sha256=np.array(list(sha.values())),
        sd_sum=np.array([float(v.double().sum()) for v in sd.values()]))
    print(f"model_debug: logits {logits.shape} max|.| {np.abs(logits).max():.4g}")

    # --- reduced model, train mode with injected DropEdge masks -------------
    B, Nr, L, Fin, C, out_dim = 2, 10, 6, 64, 32, 7
    Ar = gi.random_adj_bnln(31, B, Nr, L, 3.0)
    Vr = gi.features(32, B, Nr, Fin)
    labels = gi.rng(33).integers(0, out_dim, size=(B, Nr))
    labels[1, -2:] = -100  # padded nodes (NumpyPadding label -100, configs/sumi_node_classification.yaml)
    torch.manual_seed(1)
    small = GraphCNNDropEdge(Fin, out_dim, L, net_size=C)
    init_sd = {k: v.detach().clone().numpy() for k, v in small.state_dict().items()}
    small.train()
    small.dropout.p = 0.0  # feature dropout off: parity only for the edge masks
    de = gi.DROPEDGE
    mults = [dense_ref.dropedge_weights_pre(Ar, de["p"], de["seed"], c, drop_self=True) for c in range(3)]

    class InjectedEdgeDropout(torch.nn.Module):
        def __init__(self, ms):
            super().__init__()
            self.ms = ms
            self.i = 0

        def forward(self, a):
            m = self.ms[self.i]
            self.i += 1
            keep = _t((m != 0).astype(np.float32))
            scale = float(m.max()) if (m != 0).any() else 1.0
            return a.mul(keep).mul_(scale)

    small.edge_dropout = InjectedEdgeDropout(mults)
    logits_r = small([_t(Vr), _t(Ar)])
    loss = torch.nn.functional.cross_entropy(logits_r.transpose(1, 2), torch.from_numpy(labels), ignore_index=-100)
    loss.backward()
    grads = {f"grad::{k}": p.grad.numpy() for k, p in small.named_parameters() if p.grad is not None}
    np.savez_compressed(
        os.path.join(HERE, "model_small_train.npz"),
        A=Ar, V=Vr, labels=labels, logits=logits_r.detach().numpy(), loss=np.array(loss.item()),
        **{f"init::{k}": v for k, v in init_sd.items()}, **grads)
    print(f"model_small_train: loss {loss.item():.6f}")


def make_layout_fixtures(HeuristicGraphBuilder, TextlineEncoding):
    """Reference HeuristicGraphBuilder (graph_utils.py Graph) adjacency for
    seeded synthetic pages and for assets/samples/debug.json, all three
    edge types; plus TextlineEncoding features of the same pages."""
    with open(os.path.join(REF, "assets/samples/debug.json"), encoding="utf-8-sig") as f:
        debug = json.load(f)
    with open(os.path.join(REF, "assets/meta_data/master_charset.json"), encoding="utf-8-sig") as f:
        charset = json.load(f)["charset"]
    char_to_id = {c: i for i, c in enumerate(charset)}
    pages = {"debug": [dict(r, label=r.get("label", "other")) for r in debug]}
    for name, (seed, n, cells, tables, fc, empty) in gi.LAYOUT_CASES.items():
        pages[name] = gi.synthetic_document(seed, n, cells, tables, fc, empty)
    out = {}
    for name, regions in pages.items():
        label = {}
        for i, reg in enumerate(regions):
            label[i] = {"polygon": reg["location"], "text": reg["text"], "label": reg["label"]}
        for et in ("normal_binary", "fc_similarity", "fc_binary"):
            if et != "normal_binary" and name not in ("plain30", "cells60", "tiny2", "tables40"):
                continue
            sample = HeuristicGraphBuilder(num_edges=6, edge_type=et)({"label": dict(label)})
            adj = sample["adjacency_matrix"]
            out[f"{name}::{et}"] = adj.view(np.uint16) if et == "fc_similarity" else (adj != 0)
        if name in ("debug", "float80", "plain30"):
            enc = TextlineEncoding(is_normalized_text=True)({"label": dict(label), "char_to_id": char_to_id})
            V = enc["textline_encoding"]
            r_, c_ = np.nonzero(V[:, :-4])
            out[f"{name}::bow_rows"] = r_.astype(np.int32)
            out[f"{name}::bow_cols"] = c_.astype(np.int32)
            out[f"{name}::spatial"] = V[:, -4:]
        out[f"{name}::regions"] = np.array(json.dumps(regions, ensure_ascii=False))
    np.savez_compressed(os.path.join(HERE, "layout_graphs.npz"), **out)
    print("layout_graphs:", {k: v.shape for k, v in out.items() if k.endswith("normal_binary")})


NORMALIZE_CASES = [
    "ABC def", "１２３４５６７８９０", "It's; a_test", "tab\there\nnew\rline", "dash—en–minus−hyphen‐",
    "ideo\u3000space\u00a0nbsp\u2028ls", "dots。．・‥…", "「括弧」（全角）［角］【隅】《二重》", "«guillemets» ‹single›",
    "“quotes” ‘single’ „low“", "半角ｶﾀｶﾅ and ﾊﾝｶｸ", "Ⅻ ① ㈱ ㎏ ﬁ", "MiXeD 12:30 p.m. ¥1,000-", "",
]


def make_text_fixtures():
    from gnn.data_generator.data_process.utils.normalize_text import normalize_text

    out = [normalize_text(t) for t in NORMALIZE_CASES]
    with open(os.path.join(HERE, "normalize_text.json"), "w", encoding="utf-8") as f:
        json.dump({"inputs": NORMALIZE_CASES, "outputs": out}, f, ensure_ascii=False, indent=1)
    print("normalize_text:", len(out), "cases")


def make_model_variant_fixtures(GraphCNNDropEdge):
    """model_variants.npz: the reduced model on a padded B=2 batch with a
    float fc_similarity-style adjacency (eval, with and without attention),
    and a train step with efficient_mode=False, whose edge dropout hits the
    raw A (drop_robust_gcn.py:67-72, robust_gcn.py:42-43: the identity is
    added afterwards and never dropped) with injected masks."""
    B, N, L, Fin, C, out_dim = 2, 9, 6, 40, 32, 5
    r = gi.rng(61)
    A = (r.random((B, N, L, N)) < 0.25) * r.uniform(0.05, 1.0, (B, N, L, N))
    A = A.astype(np.float16).astype(np.float32)  # the builders emit fp16 (graph_utils.py:794-806)
    A[1, -3:] = 0.0
    A[1, :, :, -3:] = 0.0  # three padded nodes in the second graph (NumpyPadding)
    V = gi.features(62, B, N, Fin)
    V[1, -3:] = 0.0
    out = {"A": A, "V": V}
    for tag, att in (("att", True), ("noatt", False)):
        torch.manual_seed(5)
        m = GraphCNNDropEdge(Fin, out_dim, L, net_size=C, use_attention=att)
        m.eval()
        with torch.no_grad():
            out[f"{tag}::logits"] = m([_t(V), _t(A)]).numpy()
        out.update({f"{tag}::init::{k}": v.detach().numpy() for k, v in m.state_dict().items()})

    # efficient_mode=False, train mode, feature dropout off, masks on raw A
    Ab = gi.random_adj_bnln(63, B, N, L, 3.0)
    labels = gi.rng(64).integers(0, out_dim, size=(B, N))
    de = gi.DROPEDGE
    raw = []
    for c in range(3):
        mp = dense_ref.dropedge_weights_pre(Ab, de["p"], de["seed"], c, drop_self=False)  # (B,(L+1)N,N)
        mp = mp.reshape(B, N, L + 1, N)[:, :, 1:, :]      # typed blocks, [b, n, t, m]
        raw.append(np.ascontiguousarray(mp.transpose(0, 1, 3, 2)))  # raw A layout after permute: [b, n, m, t]

    class InjectedRawEdgeDropout(torch.nn.Module):
        def __init__(self, ms):
            super().__init__()
            self.ms = ms
            self.i = 0

        def forward(self, a):
            m = self.ms[self.i]
            self.i += 1
            keep = _t((m != 0).astype(np.float32))
            scale = float(m.max()) if (m != 0).any() else 1.0
            return a.mul(keep).mul_(scale)

    torch.manual_seed(6)
    m = GraphCNNDropEdge(Fin, out_dim, L, net_size=C)
    out.update({f"effF::init::{k}": v.detach().clone().numpy() for k, v in m.state_dict().items()})
    m.train()
    m.dropout.p = 0.0
    m.edge_dropout = InjectedRawEdgeDropout(raw)
    logits = m([_t(V), _t(Ab)], efficient_mode=False)
    loss = torch.nn.functional.cross_entropy(logits.transpose(1, 2), torch.from_numpy(labels))
    loss.backward()
    out.update({"effF::A": Ab, "effF::labels": labels, "effF::logits": logits.detach().numpy(),
                "effF::loss": np.array(loss.item())})
    out.update({f"effF::grad::{k}": p.grad.numpy() for k, p in m.named_parameters() if p.grad is not None})
    np.savez_compressed(os.path.join(HERE, "model_variants.npz"), **out)
    print(f"model_variants: att {np.abs(out['att::logits']).max():.4g} noatt {np.abs(out['noatt::logits']).max():.4g}"
          f" effF loss {loss.item():.6f}")


def main(parts=("text", "graphconv", "model", "layout", "variants")):
    GraphConv, GraphCNNDropEdge, HGB, TLE = _import_reference()
    if "text" in parts:
        make_text_fixtures()
    if "graphconv" in parts:
        make_graphconv_fixtures(GraphConv)
    if "model" in parts:
        make_model_fixtures(GraphCNNDropEdge, HGB, TLE)
    if "layout" in parts:
        make_layout_fixtures(HGB, TLE)
    if "variants" in parts:
        make_model_variant_fixtures(GraphCNNDropEdge)


if __name__ == "__main__":
    main(tuple(sys.argv[1:]) or ("text", "graphconv", "model", "layout", "variants"))
