"""Numerics of the exact three-term bf16 split the column-slice spectral kernel runs its GEMMs
with (csrc/tr_spectral_slice.hip: sl_split2 / sl_mfma6 / sl_mfma_lp), restated in numpy on the
fp32 bit patterns (CPU; the kernel itself is covered by tests/test_gpu_spectral.py).

  x1 = x with the low 16 bits cleared (top 8 significand bits), r = x - x1 (exact),
  x2 = r with the low 16 bits cleared, x3 = r - x2 (at most 8 significant bits: a bf16)
  a.b ~ a1b1 + a1b2 + a2b1 + a1b3 + a2b2 + a3b1   (dropped: a2b3 + a3b2 + a3b3 < 2^-20 |ab|)
"""
import numpy as np

MASK = np.uint32(0xFFFF0000)


def split3(x):
    x = np.asarray(x, dtype=np.float32)
    x1 = (x.view(np.uint32) & MASK).view(np.float32)
    r = (x - x1).astype(np.float32)
    x2 = (r.view(np.uint32) & MASK).view(np.float32)
    x3 = (r - x2).astype(np.float32)
    return x1, x2, x3


def _rand(n, seed):
    g = np.random.default_rng(seed)
    # wide exponent range, both signs, including values whose low bits are all set
    x = (g.standard_normal(n) * np.exp2(g.integers(-60, 60, n))).astype(np.float32)
    x[:8] = np.array([1.0, -1.0, 3.0000002, np.float32(1) - np.float32(2 ** -24), 1e-30, -7.5e30,
                      np.float32(0.1), 0.0], dtype=np.float32)
    return x


def test_split_is_exact_and_bf16():
    x = _rand(200000, 0)
    x1, x2, x3 = split3(x)
    # every piece is a bf16 (low 16 bits zero) and the pieces sum back to x exactly
    for p in (x1, x2, x3):
        assert not np.any(p.view(np.uint32) & np.uint32(0xFFFF))
    s = (x1.astype(np.float64) + x2.astype(np.float64)) + x3.astype(np.float64)
    assert np.array_equal(s, x.astype(np.float64))
    # magnitude bounds the error analysis uses
    ax = np.abs(x.astype(np.float64))
    assert np.all(np.abs(x2) <= ax * 2.0 ** -7)
    assert np.all(np.abs(x3) <= ax * 2.0 ** -14)


def test_six_term_product_error():
    a, b = _rand(100000, 1), _rand(100000, 2)
    a1, a2, a3 = (p.astype(np.float64) for p in split3(a))
    b1, b2, b3 = (p.astype(np.float64) for p in split3(b))
    six = a1 * b1 + a1 * b2 + a2 * b1 + a1 * b3 + a2 * b2 + a3 * b1
    exact = a.astype(np.float64) * b.astype(np.float64)
    nz = exact != 0
    rel = np.abs(six[nz] - exact[nz]) / np.abs(exact[nz])
    # the bound the kernel comment, the public header and DESIGN.md state: < 2^-20 |ab| worst case
    # (measured 2^-21.3 on this kind of sample), typically 2^-25 (below the fp32 product rounding)
    assert rel.max() < 2.0 ** -20
    assert np.median(rel) < 2.0 ** -24


def test_packed_lin_columns_sum_to_the_six_terms():
    """[b1 | b2] with A = a1, a2, a3 and [b3 | 0] with A = a1: columns c and c + 8 summed give the
    six terms plus a3b2 (sl_mfma_lp + sl_fold8)"""
    a, b = _rand(5000, 3), _rand(5000, 4)
    a1, a2, a3 = (p.astype(np.float64) for p in split3(a))
    b1, b2, b3 = (p.astype(np.float64) for p in split3(b))
    col_lo = a1 * b1 + a2 * b1 + a3 * b1 + a1 * b3
    col_hi = a1 * b2 + a2 * b2 + a3 * b2
    six = a1 * b1 + a1 * b2 + a2 * b1 + a1 * b3 + a2 * b2 + a3 * b1
    assert np.allclose(col_lo + col_hi - six, a3 * b2, rtol=0, atol=1e-300 + 1e-12 * np.abs(six).max())


def test_dot_product_matches_fp32_quality():
    """a W x D contraction at config 5's size: the split sum is as close to the exact dot product
    as a plain fp32 accumulation of fp32 products"""
    g = np.random.default_rng(5)
    n = 256 * 129
    a = np.abs(g.standard_normal(n)).astype(np.float32)
    b = (g.standard_normal(n) * 0.2).astype(np.float32)
    exact = float(np.dot(a.astype(np.float64), b.astype(np.float64)))
    a1, a2, a3 = split3(a)
    b1, b2, b3 = split3(b)
    acc = np.float32(0)
    terms = [(a1, b1), (a1, b2), (a2, b1), (a1, b3), (a2, b2), (a3, b1)]
    # fp32 accumulation of exact bf16 x bf16 products, 32 at a time (one MFMA k step)
    prods = sum(np.float64(1) * p.astype(np.float64) * q.astype(np.float64) for p, q in terms)
    for k in range(0, n, 32):
        acc = np.float32(acc + np.float32(prods[k:k + 32].sum()))
    ref32 = np.float32(0)
    for k in range(0, n, 32):
        ref32 = np.float32(ref32 + np.float32((a[k:k + 32] * b[k:k + 32]).astype(np.float32).sum()))
    scale = float(np.abs(a.astype(np.float64) * b.astype(np.float64)).sum())
    assert abs(float(acc) - exact) <= 2 * abs(float(ref32) - exact) + 1e-7 * scale


def split2_rne(x):
    """TR_SLICE_X2 (off by default): the X side as two round-to-nearest-even bf16 pieces"""
    x = np.asarray(x, dtype=np.float32)

    def rne_bf16(v):
        u = v.view(np.uint32).astype(np.uint64)
        r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16) << 16
        return r.astype(np.uint32).view(np.float32)

    x1 = rne_bf16(x)
    r = (x - x1).astype(np.float32)
    return x1, rne_bf16(r)


def test_two_piece_rne_split_bound():
    x = _rand(200000, 6)
    x = x[np.isfinite(x) & (np.abs(x) > 1e-30) & (np.abs(x) < 1e30)]
    x1, x2 = split2_rne(x)
    err = np.abs(x.astype(np.float64) - x1.astype(np.float64) - x2.astype(np.float64))
    # |x - x1| <= half an 8-bit ulp <= 2^-8 |x|, and the second rounding leaves at most 2^-8 of
    # that: <= 2^-16 |x| (measured worst case on this sample 2^-17, median 2^-19.4)
    assert np.all(err <= np.abs(x.astype(np.float64)) * 2.0 ** -16)
