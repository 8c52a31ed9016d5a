"""Hyperparameter optimisation: Mallet's
Dirichlet.learnParameters / learnSymmetricConcentration / digamma.

The product's host arithmetic (liblda_mi355x.so: lda_learn_*) against the
oracle's independent restatement (oracle/lda_oracle.c): identical fp64
operation order, so equal to the last bit; plus statistical sanity against
histograms drawn from known Dirichlet-multinomials (the fixed point recovers
the generating parameters).  Mallet itself is absent: parity unpinned beyond
the published algorithm.
"""
import ctypes as C

import numpy as np
import pytest
from scipy.special import digamma as sp_digamma

from ldagibbssampling_amd import capi


def _learn_parameters_product(alpha, hist, lens, shape=1.001, scale=1.0, iters=1):
    a = np.ascontiguousarray(alpha, dtype=np.float64).copy()
    h = np.ascontiguousarray(hist, dtype=np.int32)
    lens = np.ascontiguousarray(lens, dtype=np.int32)
    s = C.c_double()
    capi.check(capi.load().lda_learn_parameters(a, len(a), h, lens, len(lens) - 1, shape, scale,
                                                iters, C.byref(s)), "lda_learn_parameters")
    return a, s.value


def _learn_symmetric_product(count_hist, length_hist, dims, value):
    counts = np.ascontiguousarray(count_hist, dtype=np.int32)
    lens = np.nonzero(length_hist)[0].astype(np.int64)
    lc = np.ascontiguousarray(np.asarray(length_hist)[lens], dtype=np.int32)
    out = C.c_double()
    capi.check(capi.load().lda_learn_symmetric_concentration(counts, len(counts) - 1, lens, lc,
                                                             len(lens), dims, value, C.byref(out)),
               "lda_learn_symmetric_concentration")
    return out.value


def _dirmult_histograms(alpha, doc_lens, rng):
    """topicDocCounts / docLengthCounts of documents drawn from DirMult(alpha)."""
    K, L = len(alpha), int(max(doc_lens))
    hist = np.zeros((K, L + 1), np.int32)
    lens = np.zeros(L + 1, np.int32)
    for n in doc_lens:
        theta = rng.dirichlet(alpha)
        c = rng.multinomial(n, theta)
        lens[n] += 1
        for k in np.nonzero(c)[0]:
            hist[k, c[k]] += 1
    return hist, lens


def test_digamma(oracle):
    L = capi.load()
    for x in [1e-8, 1e-3, 0.1, 0.5, 1.0, 2.5, 9.4, 9.5, 10.0, 123.4, 1e6]:
        p = L.lda_digamma(x)
        assert p == oracle.digamma(x), x
        assert abs(p - sp_digamma(x)) <= 1e-9 * max(1.0, abs(sp_digamma(x))) or x < 1e-6, x


def test_learn_parameters_matches_oracle(oracle):
    rng = np.random.default_rng(1)
    alpha_true = rng.uniform(0.05, 1.5, size=12)
    hist, lens = _dirmult_histograms(alpha_true, rng.integers(5, 120, size=400), rng)
    a0 = np.full(12, 0.3)
    for iters in (1, 5):
        ap, sp = _learn_parameters_product(a0, hist, lens, iters=iters)
        ao, so = oracle.learn_parameters(a0, hist, lens, iters=iters)
        np.testing.assert_array_equal(ap, ao)
        assert sp == so


def test_learn_parameters_recovers_alpha():
    rng = np.random.default_rng(2)
    alpha_true = np.array([0.1, 0.3, 0.5, 1.0, 2.0, 0.2, 0.05, 0.8])
    hist, lens = _dirmult_histograms(alpha_true, rng.integers(50, 200, size=3000), rng)
    a, s = _learn_parameters_product(np.full(8, 1.0), hist, lens, iters=200)
    np.testing.assert_allclose(a, alpha_true, rtol=0.12)
    assert abs(s - alpha_true.sum()) < 0.1 * alpha_true.sum()


def test_learn_symmetric_matches_oracle_and_recovers(oracle):
    rng = np.random.default_rng(3)
    K, a_true = 20, 0.25
    hist, lens = _dirmult_histograms(np.full(K, a_true), rng.integers(10, 300, size=1500), rng)
    pooled = hist.sum(0)
    vp = _learn_symmetric_product(pooled, lens, K, 2.0)
    vo = oracle.learn_symmetric_concentration(pooled, lens, K, 2.0)
    assert vp == vo
    assert abs(vp / K - a_true) < 0.1 * a_true
    # topic sizes spread out (gaps > 20 take the digamma-difference branch)
    sizes = np.zeros(5001, np.int32)
    sizes[rng.integers(1, 5000, size=60)] += 1
    counts = np.bincount(rng.integers(1, 40, size=3000), minlength=41).astype(np.int32)
    assert _learn_symmetric_product(counts, sizes, 500, 5.0) == \
        oracle.learn_symmetric_concentration(counts, sizes, 500, 5.0)


def test_learn_errors_are_loud():
    L = capi.load()
    out = C.c_double()
    bad = np.array([5, 3], np.int64)          # lengths must ascend
    r = L.lda_learn_symmetric_concentration(np.ones(3, np.int32), 2, bad, np.ones(2, np.int32), 2,
                                            4, 1.0, C.byref(out))
    assert r == -1


@pytest.mark.slow
def test_mallet_oracle_optimisation_moves_hyperparameters(oracle):
    from ldagibbssampling_amd.corpus import synthetic_lda
    c = synthetic_lda(num_docs=300, num_types=800, num_topics=10, doc_len=None, mean_len=60,
                      min_len=5, max_len=200, seed=4)
    m = oracle.MalletModel(10, 10.0, 0.01, c.num_types, c.doc_off, c.words, seed=1, num_threads=2)
    m.set_optimize(20, burnin=40)
    m.estimate(100)
    a, b = m.hyper()
    assert not np.allclose(a, 1.0) and b != 0.01
    assert np.all(a > 0) and b > 0


def test_dead_topics_stay_finite(oracle):
    """A topic whose alpha has decayed below 1.1e-16 and then reappears in a
    document: Mallet's literal (a + i) - 1 cancels to 0 there (1/0 -> inf ->
    NaN alpha).  Both restatements add the integer offset first and floor
    alpha at 1e-300, so the update stays finite and positive."""
    K, L = 4, 10
    hist = np.zeros((K, L + 1), np.int32)
    lens = np.zeros(L + 1, np.int32)
    lens[10] = 50
    hist[0, 1] = 3
    hist[0, 2] = 1
    hist[1, 10] = 40
    for a0 in (1e-17, 1e-200, 1e-300):
        alpha = np.array([a0, 0.5, 1e-250, 0.3])
        ap, sp = _learn_parameters_product(alpha, hist, lens)
        ao, so = oracle.learn_parameters(alpha, hist, lens)
        np.testing.assert_array_equal(ap, ao)
        assert np.all(np.isfinite(ap)) and np.all(ap >= 1e-300) and np.isfinite(sp)


def _learn_symmetric_literal(counts, lens, dims, value):
    """Mallet's learnSymmetricConcentration with the numerator as the literal
    loop over every count 1..max (denominator: its own gap rule)."""
    top = int(np.nonzero(counts)[0].max())
    nz_len = np.nonzero(lens)[0]
    for _ in range(200):
        p = value / dims
        d = num = 0.0
        for c in range(1, top + 1):
            d += 1.0 / (p + (c - 1))
            num += counts[c] * d
        base = float(sp_digamma(value))
        d = den = 0.0
        prev = 0
        for n in nz_len:
            if n - prev > 20:
                d = float(sp_digamma(value + n)) - base
            else:
                for i in range(prev, n):
                    d += 1.0 / (value + i)
            den += d * lens[n]
            prev = n
        value = p * num / den
    return value


def test_learn_symmetric_sparse_counts(oracle):
    """optimizeBeta's countHistogram at scale is sparse at the top (cells of
    ~1e5 beside empty stretches): the numerator walks the non-zero counts with
    the denominator's gap rule.  Product == oracle to the bit, and within
    1e-12 of Mallet's literal loop."""
    rng = np.random.default_rng(7)
    counts = np.zeros(200_001, np.int32)
    counts[1:60] = rng.integers(100, 5000, 59)
    counts[rng.integers(60, 200_000, 300)] += 1
    sizes = np.zeros(2_000_001, np.int32)
    sizes[rng.integers(500_000, 2_000_000, 40)] += 1
    vp = _learn_symmetric_product(counts, sizes, 100_000, 1000.0)
    vo = oracle.learn_symmetric_concentration(counts, sizes, 100_000, 1000.0)
    assert vp == vo
    small = np.zeros(3001, np.int32)
    small[1:30] = rng.integers(10, 400, 29)
    small[rng.integers(30, 3000, 40)] += 1
    ssz = np.zeros(20001, np.int32)
    ssz[rng.integers(1000, 20000, 12)] += 1
    lit = _learn_symmetric_literal(small, ssz, 2000, 20.0)
    got = _learn_symmetric_product(small, ssz, 2000, 20.0)
    assert abs(got - lit) <= 1e-12 * abs(lit), (got, lit)
