"""CPU: the arithmetic behind the split-bf16 ("x6") fp32 GEMM and attention
kernels, restated in numpy.

Every finite fp32 v (|v| below the bf16 overflow threshold) is split as
v0 = bf16(v), v1 = bf16(v - v0), v2 = bf16(v - v0 - v1) with round-to-
nearest-even conversions; the kernels rely on (a) v == v0 + v1 + v2 exactly
and (b) the six products a_i b_j with i + j <= 2 reproducing a dot product to
fp32-rounding accuracy.  Both are checked here on random and adversarial
values, independent of the GPU."""
import numpy as np
import pytest


def bf16_rne(x: np.ndarray) -> np.ndarray:
    """fp32 -> bf16 (round to nearest even) -> fp32, as v_cvt_pk_bf16_f32."""
    u = x.astype(np.float32).view(np.uint32).astype(np.uint64)
    r = (u + 0x7FFF + ((u >> 16) & 1)) & 0xFFFF0000
    return r.astype(np.uint32).view(np.float32)


def split3(v: np.ndarray):
    v = v.astype(np.float32)
    v0 = bf16_rne(v)
    r1 = (v - v0).astype(np.float32)
    v1 = bf16_rne(r1)
    r2 = (r1 - v1).astype(np.float32)
    v2 = bf16_rne(r2)
    return v0, v1, v2


def _values(rng, n, lo=-96, hi=100):
    mant = rng.standard_normal(n).astype(np.float32)
    scale = np.float32(2.0) ** rng.integers(lo, hi, n).astype(np.float32)
    adversarial = np.array([1.0, -1.0, 1 + 2 ** -23, 1 - 2 ** -24, 3.4e38 / 512, 1.17549435e-38 * 2 ** 30,
                            0.0, -0.0, 0.1, 1 / 3, np.pi, 65504.0, 2 ** -95], dtype=np.float32)
    return np.concatenate([mant * scale, adversarial]).astype(np.float32)


def test_split_is_exact():
    """Exact for 2^-100 <= |v| < 3.39e38 (the third part stays a normal bf16)."""
    rng = np.random.default_rng(0)
    v = _values(rng, 200_000)
    v0, v1, v2 = split3(v)
    # each part is a bf16 value
    for p in (v0, v1, v2):
        assert np.array_equal(bf16_rne(p), p)
    # and they add up exactly (in float64, which holds the sum without rounding)
    recon = v0.astype(np.float64) + v1.astype(np.float64) + v2.astype(np.float64)
    assert np.array_equal(recon, v.astype(np.float64))
    # magnitudes: |v1| <= 2^-8 |v|, |v2| <= 2^-16 |v| (up to one ulp of slack at binade edges)
    nz = v != 0
    assert np.all(np.abs(v1[nz]) <= np.abs(v[nz]) * 2.0 ** -8 * (1 + 2 ** -7))
    assert np.all(np.abs(v2[nz]) <= np.abs(v[nz]) * 2.0 ** -16 * (1 + 2 ** -6))


def test_split_of_tiny_values_is_close():
    """Below 2^-100 the third part underflows into bf16 subnormals and loses
    low bits: the split is then off by at most one bf16 subnormal ulp (2^-133)."""
    rng = np.random.default_rng(1)
    v = (rng.standard_normal(100_000) * 2.0 ** -115).astype(np.float32)
    v0, v1, v2 = split3(v)
    recon = v0.astype(np.float64) + v1.astype(np.float64) + v2.astype(np.float64)
    assert np.all(np.abs(recon - v.astype(np.float64)) <= 2.0 ** -133)


@pytest.mark.parametrize("K", [16, 256, 1792])
def test_six_products_match_fp32_accuracy(K):
    """sum_k a_k b_k from the six products i + j <= 2 (each product exact in
    fp32, accumulated in fp32 like the MFMA accumulators) stays within the
    fp32 dot-product error bound K * 2^-24 * sum |a b| of the fp64 value, and
    is no worse than a plain fp32 fmaf chain by more than a small factor."""
    rng = np.random.default_rng(K)
    trials = 200
    a = rng.standard_normal((trials, K)).astype(np.float32)
    b = rng.standard_normal((trials, K)).astype(np.float32)
    ap, bp = split3(a), split3(b)
    acc = np.zeros(trials, dtype=np.float32)
    for k in range(K):  # k-outer, products in the kernels' order (small terms first)
        for i, j in ((2, 0), (1, 1), (0, 2), (1, 0), (0, 1), (0, 0)):
            acc = (acc + (ap[i][:, k] * bp[j][:, k]).astype(np.float32)).astype(np.float32)
    ref = np.sum(a.astype(np.float64) * b.astype(np.float64), axis=1)
    scale = np.sum(np.abs(a.astype(np.float64) * b.astype(np.float64)), axis=1)
    err_x6 = np.abs(acc.astype(np.float64) - ref) / scale
    plain = np.zeros(trials, dtype=np.float32)
    for k in range(K):
        plain = (plain + a[:, k] * b[:, k]).astype(np.float32)
    err_f32 = np.abs(plain.astype(np.float64) - ref) / scale
    assert err_x6.max() <= K * 2.0 ** -24
    # six accumulations per product instead of one: a few times the fp32 chain's error at most
    assert err_x6.mean() <= 4 * max(err_f32.mean(), 2.0 ** -24)


def test_integers_are_exact():
    """Small integers are single bf16 values (v1 = v2 = 0): integer GEMMs stay exact."""
    v = np.arange(-256, 257, dtype=np.float32)
    v0, v1, v2 = split3(v)
    assert np.array_equal(v0, v) and not v1.any() and not v2.any()
