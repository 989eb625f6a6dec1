"""GPU: fused NodeSelfAtten (grl_node_attention_fwd/_bwd) against a float64
torch restatement of robust_gcn.py:90-96 (out = gamma * softmax(f g^T) h + V),
forward and every gradient, over ragged shapes, padded dims, large score
magnitudes and N far beyond what a dense N x N softmax would allow."""
import numpy as np
import pytest
import torch

import grl
from grl import _lib
from grl.ops import node_attention_forward, node_self_attention

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _inputs(B, N, dk, dv, seed, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    Q = (torch.relu(torch.randn(B, N, dk, generator=g)) * scale).to(DEV)  # f, g are Linear+ReLU outputs
    K = (torch.relu(torch.randn(B, N, dk, generator=g)) * scale).to(DEV)
    H = torch.relu(torch.randn(B, N, dv, generator=g)).to(DEV)
    V = torch.randn(B, N, dv, generator=g).to(DEV)
    gamma = torch.randn(dv, generator=g).to(DEV)
    return Q, K, H, V, gamma


def _ref(Q, K, H, V, gamma):
    s = torch.softmax(torch.matmul(Q, K.transpose(1, 2)), -1)
    return gamma * torch.matmul(s, H) + V


SHAPES = [(1, 74, 16, 128), (4, 74, 16, 128), (2, 33, 4, 32), (1, 1, 2, 16), (3, 130, 16, 128), (2, 300, 32, 256),
          (2, 64, 5, 40), (1, 500, 16, 100), (2, 9, 0, 4),  # dk = 0: net_size 8 (4 // 8), uniform attention
          (1, 2048, 16, 128), (2, 1000, 5, 100), (1, 777, 32, 128),  # small-N key / query splits (S = 8, 3, 3)
          (64, 1024, 16, 128), (4, 1100, 16, 128),  # >= 4096 rows: LDS-DMA planes, unsplit / split (S = 4)
          (2, 200, 64, 512), (1, 150, 40, 300), (2, 96, 33, 64), (1, 300, 20, 640)]  # net_size 1024 (dk 64,
          # dv 512) and other widths beyond one call: fp32 kernels with 64-wide Q/K, dv in column blocks


MODES = ["x6", "x6-no-workspace", "f32"]


def _set_mode(mode, monkeypatch, grl_option):
    """x6: split-bf16 kernels with the once-per-call operand planes (default);
    x6-no-workspace: the same kernels splitting every block themselves;
    f32: the fp32-MFMA kernels (attn_x6 = 0)."""
    import grl.ops

    grl_option("attn_x6", int("0" if mode == "f32" else "1"))
    if mode == "x6-no-workspace":
        monkeypatch.setattr(grl.ops, "_attn_workspace", lambda *a, **k: (None, 0))


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("B,N,dk,dv", SHAPES)
def test_forward_matches_fp64(B, N, dk, dv, mode, monkeypatch, grl_option):
    _set_mode(mode, monkeypatch, grl_option)
    Q, K, H, V, gamma = _inputs(B, N, dk, dv, seed=N + dk)
    out = node_attention_forward(Q, K, H, V, gamma)
    ref = _ref(*(t.double() for t in (Q, K, H, V, gamma)))
    torch.testing.assert_close(out.double(), ref, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("B,N,dk,dv", SHAPES)
def test_backward_matches_fp64(B, N, dk, dv, mode, monkeypatch, grl_option):
    _set_mode(mode, monkeypatch, grl_option)
    Q, K, H, V, gamma = _inputs(B, N, dk, dv, seed=7 * N + dv)
    leaves = [t.clone().requires_grad_(True) for t in (Q, K, H, V, gamma)]
    out = node_self_attention(*leaves)
    dout = torch.randn(out.shape, generator=torch.Generator().manual_seed(3)).to(DEV)
    out.backward(dout)
    ref_leaves = [t.double().clone().requires_grad_(True) for t in (Q, K, H, V, gamma)]
    _ref(*ref_leaves).backward(dout.double())
    for name, a, r in zip("QKHVg", leaves, ref_leaves):
        scale = (r.grad.abs().max().item() if r.grad.numel() else 0.0) + 1.0
        torch.testing.assert_close(a.grad.double(), r.grad, rtol=1e-4, atol=2e-5 * scale, msg=f"d{name}")


def test_large_scores_are_stable():
    """No 1/sqrt(dk) scaling in the reference: scores of several hundred must
    not overflow (online max subtraction)."""
    Q, K, H, V, gamma = _inputs(2, 200, 16, 128, seed=5, scale=6.0)
    out = node_attention_forward(Q, K, H, V, gamma)
    assert torch.isfinite(out).all()
    ref = _ref(*(t.double() for t in (Q, K, H, V, gamma)))
    torch.testing.assert_close(out.double(), ref, rtol=1e-4, atol=1e-4)


def test_large_n_rows_sampled():
    """N = 20k (a dense softmax would need 1.6 GB of scores per batch): check
    64 sampled query rows against fp64."""
    B, N, dk, dv = 1, 20000, 16, 128
    Q, K, H, V, gamma = _inputs(B, N, dk, dv, seed=11)
    out = node_attention_forward(Q, K, H, V, gamma)
    idx = torch.randperm(N, generator=torch.Generator().manual_seed(1))[:64].to(DEV)
    s = torch.softmax(Q[0, idx].double() @ K[0].double().T, -1)
    ref = gamma.double() * (s @ H[0].double()) + V[0, idx].double()
    # fp32 sums over 20k keys: the north-star fp32 tolerance (1e-4)
    torch.testing.assert_close(out[0, idx].double(), ref, rtol=1e-4, atol=1e-4)


def test_deterministic():
    Q, K, H, V, gamma = _inputs(2, 150, 16, 128, seed=2)
    grads = []
    for _ in range(2):
        leaves = [t.clone().requires_grad_(True) for t in (Q, K, H, V, gamma)]
        node_self_attention(*leaves).sum().backward()
        grads.append([t.grad for t in leaves])
    for a, b in zip(*grads):
        assert torch.equal(a, b)


def test_bad_widths_raise():
    Q, K, H, V, gamma = _inputs(1, 8, 72, 16, seed=0)  # input_dim > 512: dk > 64
    with pytest.raises(_lib.GrlError, match="key width"):
        node_attention_forward(Q, K, H, V, gamma)
    with pytest.raises(_lib.GrlError, match="attention shapes"):
        node_attention_forward(Q[..., :8], K[..., :8], H, V[..., :8], gamma)


@pytest.mark.parametrize("B,N,dk,dv", [(1, 74, 16, 128), (4, 1100, 16, 128), (64, 1024, 16, 128), (2, 300, 32, 256),
                                       (1, 2048, 16, 128), (2, 1000, 5, 100), (3, 4099, 16, 64), (2, 4127, 32, 32)])
def test_pipelined_forward_same_bits(B, N, dk, dv, monkeypatch, grl_option):
    """attn_fwd_x6p_kernel (block k+1's softmax inside block k's P.H MFMAs)
    against the unpipelined x6 forward (attn_pipe = 0): same products, same
    order of every sum -- out and the saved row stats bitwise, with key
    splits, partial last blocks and every value width."""
    from grl.ops import node_self_attention

    Q, K, H, V, gamma = _inputs(B, N, dk, dv, seed=7 * N + dk)
    res = {}
    for pipe in ("1", "0"):
        grl_option("attn_pipe", int(pipe))
        out = node_attention_forward(Q, K, H, V, gamma)
        leaves = [t.clone().requires_grad_(True) for t in (Q, K, H, V, gamma)]
        node_self_attention(*leaves).square().sum().backward()
        res[pipe] = (out, [t.grad for t in leaves])
    assert torch.equal(res["1"][0], res["0"][0])
    for a, b in zip(res["1"][1], res["0"][1]):
        assert torch.equal(a, b)


@pytest.mark.parametrize("B,N,dk,dv", [(1, 8192, 16, 128), (2, 5000, 16, 100), (3, 4099, 9, 128), (1, 6000, 1, 97),
                                       (200, 24, 16, 128)])  # many pages shorter than one query block
def test_fused_dq_backward(B, N, dk, dv, monkeypatch, grl_option):
    """dQ folded into the key-stationary dK kernel (attn_bwd_kq_x6_kernel:
    exact MFMA transpose of dS, per-workgroup slabs added in order) against
    fp64 and against the separate dQ kernel (attn_fused_dq = 0); dK / dH
    within the same tolerance, deterministic run to run."""
    lib = _lib.lib()
    assert lib.grl_node_attention_bwd_workspace_size(B, N, dk, dv) > lib.grl_node_attention_workspace_size(B, N, dk, dv)
    Q, K, H, V, gamma = _inputs(B, N, dk, dv, seed=N + 3 * dk)
    dout = torch.randn(B, N, dv, generator=torch.Generator().manual_seed(4)).to(DEV)
    grads = {}
    for fused in ("1", "0", "1"):
        grl_option("attn_fused_dq", int(fused))
        leaves = [t.clone().requires_grad_(True) for t in (Q, K, H, V, gamma)]
        node_self_attention(*leaves).backward(dout)
        g = [t.grad for t in leaves]
        if fused in grads:
            for a, b in zip(grads[fused], g):
                assert torch.equal(a, b)
        grads[fused] = g
    ref_leaves = [t.double().clone().requires_grad_(True) for t in (Q, K, H, V, gamma)]
    _ref(*ref_leaves).backward(dout.double())
    for name, a, c, r in zip("QKHVg", grads["1"], grads["0"], ref_leaves):
        scale = r.grad.abs().max().item() + 1.0
        torch.testing.assert_close(a.double(), r.grad, rtol=1e-4, atol=2e-5 * scale, msg=f"fused d{name}")
        torch.testing.assert_close(a.double(), c.double(), rtol=1e-4, atol=2e-5 * scale, msg=f"fused vs dQ kernel d{name}")


@pytest.mark.parametrize("B,N,dk,dv", [(1, 8192, 16, 128), (3, 4099, 9, 100), (2, 5000, 32, 128)])
def test_eight_wave_workgroups_same_bits(B, N, dk, dv, monkeypatch, grl_option):
    """The forward and dH kernels on 8-wave (256-row) workgroups compute every
    row exactly as on 4-wave ones (attn_fwd8 / attn_dh8 = 0): out and
    every gradient bitwise, partial last blocks and splits included."""
    Q, K, H, V, gamma = _inputs(B, N, dk, dv, seed=N + dv)
    res = {}
    grl_option("attn_dh16", 0)  # the 32x32x16 dH on both workgroup sizes
    for v in ("1", "0"):
        grl_option("attn_fwd8", int(v))
        grl_option("attn_dh8", int(v))
        leaves = [t.clone().requires_grad_(True) for t in (Q, K, H, V, gamma)]
        out = node_self_attention(*leaves)
        out.square().sum().backward()
        res[v] = [out.detach()] + [t.grad for t in leaves]
    for a, b in zip(res["1"], res["0"]):
        assert torch.equal(a, b)


@pytest.mark.parametrize("B,N,dk,dv", [(1, 8192, 16, 128), (3, 4099, 9, 100), (64, 1024, 16, 128), (4, 1100, 16, 128),
                                       (1, 20_000, 16, 128), (2, 4127, 16, 32)])
def test_dh_on_16x16x32_matches_fp64(B, N, dk, dv, grl_option):
    """attn_bwd_h16_kernel (dH in 16 x 16 tiles on v_mfma_f32_16x16x32_bf16,
    the six x6 products of S paired along K = 32): every gradient against
    float64, and dH within fp32 rounding of the 32x32x16 kernel -- unsplit
    and query-split grids (N = 1100 x 4, 20k), partial blocks, dk = 9,
    dv = 100 (zero-padded planes) and dv = 32 (its own 32-wide planes: the
    32x32x16 kernel runs)."""
    Q, K, H, V, gamma = _inputs(B, N, dk, dv, seed=5 * N + dk)
    dout = torch.randn(B, N, dv, generator=torch.Generator().manual_seed(4)).to(DEV)
    grads = {}
    for v in (1, 0):
        grl_option("attn_dh16", v)
        leaves = [t.clone().requires_grad_(True) for t in (Q, K, H, V, gamma)]
        node_self_attention(*leaves).backward(dout)
        grads[v] = [t.grad for t in leaves]
    ref_leaves = [t.double().clone().requires_grad_(True) for t in (Q, K, H, V, gamma)]
    _ref(*ref_leaves).backward(dout.double())
    for name, a, c, r in zip("QKHVg", grads[1], grads[0], ref_leaves):
        scale = r.grad.abs().max().item() + 1.0
        print(f"d{name}: scale {scale:.3e} err vs fp64 {float((a.double() - r.grad).abs().max()):.3e} "
              f"(32x32x16: {float((c.double() - r.grad).abs().max()):.3e})")
        torch.testing.assert_close(a.double(), r.grad, rtol=1e-4, atol=2e-5 * scale, msg=f"dh16 d{name}")
        torch.testing.assert_close(a.double(), c.double(), rtol=1e-5, atol=1e-6 * scale, msg=f"dh16 vs 32x32 d{name}")


@pytest.mark.parametrize("B,N,dk,dv", [(1, 8192, 16, 128), (3, 4099, 9, 100), (64, 1024, 16, 128), (4, 1100, 16, 128),
                                       (1, 20_000, 16, 128), (1, 6000, 1, 97), (200, 24, 16, 128)])
def test_kq_on_16x16x32_matches_fp64(B, N, dk, dv, grl_option):
    """attn_bwd_kq16_kernel (the fused dK / dQ pass in 16 x 16 tiles on
    v_mfma_f32_16x16x32_bf16: S's products paired along K = 32, dS^T by
    a round trip through the wave's LDS slots, dQ over the wave's keys): every
    gradient against float64 and within fp32 rounding of the 32x32x16 kernel
    -- unsplit and query-split grids, partial blocks, pages shorter than a
    query block, dk = 1 / 9, dv = 97 / 100; deterministic run to run."""
    Q, K, H, V, gamma = _inputs(B, N, dk, dv, seed=7 * N + dk)
    dout = torch.randn(B, N, dv, generator=torch.Generator().manual_seed(6)).to(DEV)
    grads = {}
    for v in (1, 0, 1):
        grl_option("attn_kq16", v)
        leaves = [t.clone().requires_grad_(True) for t in (Q, K, H, V, gamma)]
        node_self_attention(*leaves).backward(dout)
        g = [t.grad for t in leaves]
        if v in grads:
            for a, b in zip(grads[v], g):
                assert torch.equal(a, b)
        grads[v] = g
    ref_leaves = [t.double().clone().requires_grad_(True) for t in (Q, K, H, V, gamma)]
    _ref(*ref_leaves).backward(dout.double())
    for name, a, c, r in zip("QKHVg", grads[1], grads[0], ref_leaves):
        scale = r.grad.abs().max().item() + 1.0
        e16, e32 = float((a.double() - r.grad).abs().max()), float((c.double() - r.grad).abs().max())
        print(f"d{name}: scale {scale:.3e} err vs fp64 {e16:.3e} (32x32x16: {e32:.3e}) "
              f"apart {float((a - c).abs().max()):.3e}")
        torch.testing.assert_close(a.double(), r.grad, rtol=1e-4, atol=2e-5 * scale, msg=f"kq16 d{name}")
        # dQ sums dS over every key with cancellation (the keys' dS add to ~0 per query), so the two
        # kernels' roundings differ by more than dH's; the bar is the 32x32x16 kernel's own error
        assert e16 <= 2.0 * e32 + 1e-6 * scale, f"kq16 d{name}: {e16} vs {e32}"


RANGED = [(1, 20_000, 16, 128, (0, 7000, 13_003, 20_000)), (2, 3000, 16, 100, (0, 0, 1, 1500, 3000)),
          (1, 5000, 32, 128, (0, 2500, 5000)), (1, 1200, 64, 512, (0, 600, 1200)), (1, 9000, 4, 32, (0, 9000))]


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("B,N,dk,dv,cuts", RANGED)
def test_query_ranges_partition_the_attention(B, N, dk, dv, cuts, mode, monkeypatch, grl_option):
    """grl_node_attention_fwd_rows / _bwd_rows (a node-range shard's queries
    against every key, grl.dist sharded_node_attention): over a partition of
    the queries, each range's output rows match the float64 attention (the
    unranged forward's tolerance: 1e-5, and the fp32 1e-4 at 20k keys), the
    ranges' dQ rows are the whole dQ's, and the ranges' dK / dH partials add
    up (in range order) to the whole dK / dH -- within the unranged
    backward's tolerance per range (each range's partial is one more fp32
    rounding of the sum).  Rows outside a range stay zero."""
    from grl.ops import node_attention_backward

    _set_mode(mode, monkeypatch, grl_option)
    Q, K, H, V, gamma = _inputs(B, N, dk, dv, seed=N + 7)
    dout = torch.randn(B, N, dv, generator=torch.Generator().manual_seed(3)).to(DEV)
    Qd, Kd, Hd, Vd, gd = (t.double().requires_grad_(True) for t in (Q, K, H, V, gamma))
    ref = _ref(Qd, Kd, Hd, Vd, gd)
    ref.backward(dout.double())
    dQ_sum = torch.zeros_like(Q)
    dK_sum, dH_sum = torch.zeros_like(K), torch.zeros_like(H)
    for q0, q1 in zip(cuts[:-1], cuts[1:]):
        out, onorm, rmax, rsum = node_attention_forward(Q, K, H, V, gamma, stats=True, q_range=(q0, q1))
        # as test_forward_matches_fp64 (N <= 2048) / test_large_n_rows_sampled (the fp32 1e-4 beyond)
        tol = 1e-4 if N > 2048 and (N >= 20_000 or mode == "f32") else 1e-5
        torch.testing.assert_close(out[:, q0:q1].double(), ref[:, q0:q1].detach(), rtol=tol, atol=tol)
        assert not bool(out[:, :q0].any()) and not bool(out[:, q1:].any())
        dQ, dK, dH = node_attention_backward(Q, K, H, gamma, onorm, rmax, rsum, dout, q_range=(q0, q1))
        assert not bool(dQ[:, :q0].any()) and not bool(dQ[:, q1:].any())
        dQ_sum += dQ
        dK_sum += dK
        dH_sum += dH
    ranges = len(cuts) - 1
    for got, want in ((dQ_sum, Qd.grad), (dK_sum, Kd.grad), (dH_sum, Hd.grad)):
        scale = float(want.abs().max()) + 1.0  # test_backward_matches_fp64's bound, per range
        per = 1e-4 if mode == "f32" and N > 2048 else 2e-5  # the fp32-MFMA kernels' sums over >= 3k queries
        torch.testing.assert_close(got.double(), want, rtol=1e-4, atol=per * scale * ranges)


@pytest.mark.parametrize("kq16", [0, 1])
@pytest.mark.parametrize("B,N,budget_x", [(1, 20_000, 23), (2, 9000, 7), (1, 4500, 1)])
def test_fused_dq_key_chunks_are_bitwise(B, N, budget_x, kq16, monkeypatch, grl_option):
    """The fused dK/dQ pass in key chunks (the dQ slabs of budget_x key
    workgroups per launch, the attn_qslab_max option), each chunk's slabs added onto
    dQ in order: dQ, dK, dH bitwise the one-launch pass's (both kernels)."""
    from grl.ops import node_attention_backward

    grl_option("attn_kq16", kq16)
    Q, K, H, V, gamma = _inputs(B, N, 16, 128, seed=N)
    dout = torch.randn(B, N, 128, generator=torch.Generator().manual_seed(4)).to(DEV)
    out, onorm, rmax, rsum = node_attention_forward(Q, K, H, V, gamma, stats=True)
    whole = node_attention_backward(Q, K, H, gamma, onorm, rmax, rsum, dout)
    npad = -(-N // 32) * 32
    grl_option("attn_qslab_max", budget_x * B * npad * 16 * 4)
    chunked = node_attention_backward(Q, K, H, gamma, onorm, rmax, rsum, dout)
    for a, b in zip(whole, chunked):
        assert torch.equal(a, b)


def test_half_million_nodes_forward_backward():
    """B = 1, N = 500k (the fused pass's dQ slabs, 62 GB in one piece, run in
    key chunks): fwd + bwd run; out on sampled queries within 1e-5 of float64
    (their softmax statistics recomputed in float64 over every key), dQ within
    the fp32 1e-4 of its scale (sums over 500k keys); dK / dH equal the
    separate-dQ-kernel path's within 1e-5 of their scale."""
    import os

    from grl.ops import node_attention_backward

    N = 500_000
    Q, K, H, V, gamma = _inputs(1, N, 16, 128, seed=11)
    dout = torch.randn(1, N, 128, generator=torch.Generator().manual_seed(5)).to(DEV)
    out, onorm, rmax, rsum = node_attention_forward(Q, K, H, V, gamma, stats=True)
    dQ, dK, dH = node_attention_backward(Q, K, H, gamma, onorm, rmax, rsum, dout)
    rows = torch.tensor([0, 1, 31, 32, 4095, 123_457, 250_000, 499_968, N - 1], device=DEV)
    Kd, Hd = K[0].double(), H[0].double()
    s = Q[0, rows].double() @ Kd.T
    p = torch.softmax(s, -1)
    o = p @ Hd
    torch.testing.assert_close(out[0, rows].double(), gamma.double() * o + V[0, rows].double(), rtol=1e-5, atol=1e-5)
    dO = dout[0, rows].double() * gamma.double()
    dP = dO @ Hd.T
    D = (dO * o).sum(-1, keepdim=True)
    dQ_ref = (p * (dP - D)) @ Kd
    torch.testing.assert_close(dQ[0, rows].double(), dQ_ref, rtol=1e-4, atol=1e-4 * float(dQ_ref.abs().max()))
    with grl.options(attn_fused_dq=0):
        _, dK2, dH2 = node_attention_backward(Q, K, H, gamma, onorm, rmax, rsum, dout)
    for a, b in ((dK, dK2), (dH, dH2)):
        assert float((a - b).abs().max()) <= 1e-5 * max(1.0, float(b.abs().max()))
