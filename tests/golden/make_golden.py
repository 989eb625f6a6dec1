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


def _procedure_shims():
    """Logging-only stand-ins the reference's training procedure imports
    (gnn/trainer/training_procedures/base_procedure.py:4-7,
    kv_procedure.py:6): neptune (never the real one: gnn/utils/constant.py
    opens a remote run at import) and tensorboardX."""
    if "neptune" not in sys.modules:
        nep = types.ModuleType("neptune")
        nep.new = types.ModuleType("neptune.new")
        nep.init_run = nep.new.init_run = lambda *a, **k: None
        sys.modules["neptune"], sys.modules["neptune.new"] = nep, nep.new
    def _mod(name, **attrs):
        if name not in sys.modules:
            try:
                __import__(name)
                return
            except ImportError:
                m = types.ModuleType(name)
                m.__dict__.update(attrs)
                sys.modules[name] = m

    # config / IO helpers of gnn/data_generator/base_dataloader.py:3-5 (no arithmetic)
    import yaml

    _mod("anyconfig", load=lambda path, **k: yaml.safe_load(open(path)))
    _mod("munch", munchify=lambda d: d, Munch=dict)

    class _Compose:
        def __init__(self, ts):
            self.ts = ts

        def __call__(self, x):
            for t in self.ts:
                x = t(x)
            return x

    _mod("torchvision")
    if not hasattr(sys.modules["torchvision"], "transforms"):
        tv = types.ModuleType("torchvision.transforms")
        tv.Compose = _Compose
        sys.modules["torchvision"].transforms = tv
        sys.modules["torchvision.transforms"] = tv
    _mod("cv2")
    if "tensorboardX" not in sys.modules:
        tb = types.ModuleType("tensorboardX")

        class SummaryWriter:  # no-op
            def __init__(self, *a, **k):
                pass

            def __getattr__(self, name):
                return lambda *a, **k: None

        tb.SummaryWriter = SummaryWriter
        sys.modules["tensorboardX"] = tb


# the procedure fixture: 3 batches of B = 2 pages of N = 40 text lines, a
# reduced GraphCNNDropEdge(4369, 15, 6, net_size=32) -- feature dropout off,
# DropEdge p = 0.3 with the engine's hash masks injected -- and the reference's
# own KVProcedure._run_train_step (kv_procedure.py:143-164: forward, its
# CrossEntropyLoss wrapper (ignore_index -100), backward, clip_grad_norm_(5.0),
# Adam built by its BuitlinOptimizer)
PROC_SEED, PROC_DROPEDGE_SEED, PROC_B, PROC_N, PROC_STEPS = 21, 5, 2, 40, 3


def _step_seed(base: int, step: int) -> int:
    """The per-step DropEdge seed of a captured training step with a fixed
    dropedge_seed (gnn/trainer/training_procedures/step_graph.py
    StepGraph._step_seed), restated."""
    M = (1 << 64) - 1
    x = (base * 0x9E3779B97F4A7C15 + step) & M
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & M
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & M
    return (x ^ (x >> 31)) & ((1 << 62) - 1)


def make_procedure_fixtures(GraphCNNDropEdge, HeuristicGraphBuilder, TextlineEncoding):
    _procedure_shims()
    from gnn.trainer import losses, optimizers
    from gnn.trainer.training_procedures.kv_procedure import KVProcedure

    with open(os.path.join(REF, "assets/meta_data/master_charset.json"), encoding="utf-8-sig") as f:
        charset = json.load(f)["charset"]
    char_to_id = {c: i for i, c in enumerate(charset)}
    r = gi.rng(PROC_SEED)
    batches = []
    for s in range(PROC_STEPS):
        Vs, As = [], []
        for d in range(PROC_B):
            regions = gi.synthetic_document(300 + 10 * s + d, PROC_N)
            label = {i: {"polygon": reg["location"], "text": reg["text"], "label": "other"}
                     for i, reg in enumerate(regions)}
            enc = TextlineEncoding(is_normalized_text=True)({"label": dict(label), "char_to_id": char_to_id})
            adj = HeuristicGraphBuilder(num_edges=6, edge_type="normal_binary")({"label": dict(label)})
            Vs.append(enc["textline_encoding"].astype(np.float32))
            As.append(adj["adjacency_matrix"])
        y = r.integers(0, 15, size=(PROC_B, PROC_N))
        y[r.random((PROC_B, PROC_N)) < 0.1] = -100  # padded / unlabelled nodes (NumpyPadding's -100)
        batches.append((np.stack(Vs), np.stack(As), y))
    out = {}
    for s, (V, A, y) in enumerate(batches):
        nzr = np.nonzero(V)
        out[f"batch{s}::V_idx"] = np.stack(nzr).astype(np.int32)
        out[f"batch{s}::V_vals"] = V[nzr]
        out[f"batch{s}::A_bits"] = np.packbits(A != 0)
        out[f"batch{s}::labels"] = y
    out["V_shape"] = np.array(batches[0][0].shape)
    out["A_shape"] = np.array(batches[0][1].shape)
    touched = np.unique(np.concatenate([np.nonzero(V.reshape(-1, V.shape[-1]).any(0))[0] for V, _, _ in batches]))
    out["emb1_touched_cols"] = touched.astype(np.int32)
    de = gi.DROPEDGE
    for mode in ("eager", "captured"):
        torch.manual_seed(PROC_SEED)
        model = GraphCNNDropEdge(4369, 15, 6, net_size=32)
        if mode == "eager":
            out.update({f"init::{k}": v.detach().clone().numpy() for k, v in model.state_dict().items()
                        if k != "emb1.0.weight"})
            out["init::emb1.0.weight::touched"] = model.emb1[0].weight.detach()[:, touched].clone().numpy()
            out["init_sha256"] = np.array([hashlib.sha256(v.detach().contiguous().numpy().tobytes()).hexdigest()
                                           for v in model.state_dict().values()])
        model.dropout.p = 0.0
        masks = []
        for s, (V, A, y) in enumerate(batches):
            A32 = A.astype(np.float32)
            if mode == "eager":  # the model's EdgeDropout(seed): calls 0, 1, 2, 3, ... across steps
                masks += [dense_ref.dropedge_weights_pre(A32, de["p"], PROC_DROPEDGE_SEED, 3 * s + c) for c in range(3)]
            else:  # StepGraph: a per-step seed, calls 0, 1, 2; static graphs number self loops from 2^31
                masks += [dense_ref.dropedge_weights_pre(A32, de["p"], _step_seed(PROC_DROPEDGE_SEED, s), c,
                                                         self_base=1 << 31) for c in range(3)]

        class InjectedEdgeDropout(torch.nn.Module):
            def __init__(self, ms):
                super().__init__()
                self.ms, self.i = ms, 0

            def forward(self, a):
                m = self.ms[self.i]
                self.i += 1
                keep = _t((m != 0).astype(np.float32))
                scale = float(m.max()) if (m != 0).any() else 1.0
                return a.mul(keep).mul_(scale)

        model.edge_dropout = InjectedEdgeDropout(masks)
        proc = object.__new__(KVProcedure)  # the reference's step methods on a minimal procedure state
        proc.model, proc.device = model, torch.device("cpu")
        proc.criterion = getattr(losses, "CrossEntropyLoss")._from_config({})
        proc.optimizer = getattr(optimizers, "BuitlinOptimizer")._from_config(
            {"type_optimizer": "Adam", "lr": 0.001}).get_optimizer(model.parameters())
        proc.activator = torch.nn.Softmax(dim=2)
        proc.class_names = tuple(["other"] + [f"c{i}" for i in range(14)])
        proc.config = types.SimpleNamespace(max_grad_norm=5.0, data_config=types.SimpleNamespace(
            dataset=types.SimpleNamespace(args=types.SimpleNamespace(node_label_padding_value=-100,
                                                                     other_class_index=None))))
        losses_ = []
        for V, A, y in batches:
            batch = {"textline_encoding": _t(V), "adjacency_matrix": _t(A), "node_label": torch.from_numpy(y)}
            scores, _ = KVProcedure._run_train_step(proc, batch)
            losses_.append(scores["loss"])
        out[f"{mode}::losses"] = np.array(losses_)
        sd = model.state_dict()
        out.update({f"{mode}::final::{k}": v.detach().clone().numpy() for k, v in sd.items()
                    if k != "emb1.0.weight"})
        out[f"{mode}::final::emb1.0.weight::touched"] = sd["emb1.0.weight"][:, touched].clone().numpy()
        print(f"procedure {mode}: losses {losses_}")
    np.savez_compressed(os.path.join(HERE, "procedure_train.npz"), **out)


def main(parts=("text", "graphconv", "model", "layout", "variants", "procedure")):
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
    if "procedure" in parts:
        make_procedure_fixtures(GraphCNNDropEdge, HGB, TLE)


if __name__ == "__main__":
    main(tuple(sys.argv[1:]) or ("text", "graphconv", "model", "layout", "variants", "procedure"))
