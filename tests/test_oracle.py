"""CPU tests of the oracle itself (no GPU): pinned against published KATs
and independent math, then self-consistency of the cpu_exact semantics."""
import math

import numpy as np
import pytest

from ldagibbssampling_amd.corpus import synthetic_lda, synthetic_changelists


# Random123 kat_vectors, philox4x32 10 rounds (ctr, key -> out).
PHILOX_KAT = [
    ([0, 0, 0, 0], [0, 0], [0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8]),
    ([0xffffffff] * 4, [0xffffffff] * 2, [0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd]),
    ([0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344], [0xa4093822, 0x299f31d0],
     [0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1]),
]


@pytest.mark.parametrize("ctr,key,out", PHILOX_KAT)
def test_philox_kat(oracle, ctr, key, out):
    assert oracle.philox4x32_10(ctr, key) == out


def test_java_random_known_values(oracle):
    r = oracle.JavaRandom(42)
    assert r.nextInt() == -1170105035
    assert r.nextInt() == 234785527
    assert oracle.JavaRandom(0).nextInt() == -1155484576
    assert oracle.JavaRandom(0).nextDouble() == 0.730967787376657
    assert oracle.JavaRandom(42).nextDouble() == 0.7275636800328681
    r = oracle.JavaRandom(7)
    vals = [r.nextInt(10) for _ in range(1000)]
    assert min(vals) == 0 and max(vals) == 9


@pytest.mark.parametrize("z", [0.001, 0.01, 0.2, 1.0, 1.5, 2.0, 7.3, 100.0, 1e5])
def test_log_gamma_stirling_vs_lgamma(oracle, z):
    assert abs(oracle.log_gamma_stirling(z) - math.lgamma(z)) < 2e-5 * max(1.0, abs(math.lgamma(z)))


def test_u01_range(oracle):
    assert oracle.u01(0) == 0.0
    assert oracle.u01(0xFFFFFFFF) == 1.0 - 2.0 ** -24


def test_exact_counts_consistent(oracle):
    c = synthetic_lda(num_docs=50, num_types=300, num_topics=20, doc_len=None, mean_len=40,
                      min_len=1, max_len=120, seed=3)
    K = 20
    o = oracle.ExactSampler(K, c.num_types, c.doc_off, c.words, np.full(K, 0.1), 0.01, seed=9)
    o.sweep(4)
    z = o.z()
    nw, nwsum, nd, ndsum = o.counts(with_nd=True)
    ref_nw = np.zeros((c.num_types, K), np.int64)
    np.add.at(ref_nw, (c.words, z), 1)
    np.testing.assert_array_equal(nw, ref_nw)
    np.testing.assert_array_equal(nwsum, ref_nw.sum(0))
    np.testing.assert_array_equal(nd.sum(1), ndsum)
    assert o.sweep_index == 4
    assert z.min() >= 0 and z.max() < K


def test_exact_is_deterministic_and_seeded(oracle):
    c = synthetic_changelists(num_docs=100, num_types=200, seed=1)
    K = 16
    a = oracle.ExactSampler(K, c.num_types, c.doc_off, c.words, 0.5, 0.01, seed=5)
    b = oracle.ExactSampler(K, c.num_types, c.doc_off, c.words, 0.5, 0.01, seed=5)
    d = oracle.ExactSampler(K, c.num_types, c.doc_off, c.words, 0.5, 0.01, seed=6)
    for s in (a, b, d):
        s.sweep(3)
    np.testing.assert_array_equal(a.z(), b.z())
    assert not np.array_equal(a.z(), d.z())


def test_exact_sharded_equals_single(oracle):
    """AD-LDA: summing shard deltas reproduces the single-shard run exactly."""
    c = synthetic_lda(num_docs=60, num_types=200, num_topics=32, doc_len=None, mean_len=30,
                      min_len=0, max_len=80, seed=4)
    K, seed = 32, 11
    single = oracle.ExactSampler(K, c.num_types, c.doc_off, c.words, 0.1, 0.01, seed)
    cuts = [0, 25, 60]
    shards = [oracle.ExactSampler(K, c.num_types, c.doc_off[a:b + 1],
                                  c.words[c.doc_off[a]:c.doc_off[b]], 0.1, 0.01, seed,
                                  token_base=int(c.doc_off[a]))
              for a, b in zip(cuts[:-1], cuts[1:])]

    def reduce_apply():
        tot = sum(s.delta().astype(np.int64) for s in shards).astype(np.int32)
        for s in shards:
            s.delta()[:] = tot
            s.apply()

    reduce_apply()
    single.apply()
    for _ in range(3):
        for s in shards:
            s.sample()
        reduce_apply()
        single.sample()
        single.apply()
    np.testing.assert_array_equal(np.concatenate([s.z() for s in shards]), single.z())


def test_mallet_restatement_counts(oracle):
    c = synthetic_changelists(num_docs=300, num_types=500, seed=2)
    for threads in (1, 4):
        m = oracle.MalletModel(20, 10.0, 0.01, c.num_types, c.doc_off, c.words, seed=3,
                               num_threads=threads)
        m.estimate(5)
        z = m.z()
        nw, nwsum = m.counts()
        ref = np.zeros((c.num_types, 20), np.int64)
        np.add.at(ref, (c.words, z), 1)
        np.testing.assert_array_equal(nw, ref)
        np.testing.assert_array_equal(nwsum, ref.sum(0))


def test_mallet_init_uses_java_random(oracle):
    """addInstances: z = random.nextInt(K) in document order, Randoms(seed)."""
    c = synthetic_changelists(num_docs=30, num_types=50, seed=2)
    m = oracle.MalletModel(20, 10.0, 0.01, c.num_types, c.doc_off, c.words, seed=123)
    r = oracle.JavaRandom(123)
    np.testing.assert_array_equal(m.z(), [r.nextInt(20) for _ in range(c.num_tokens)])


def test_mallet_ll_improves(oracle):
    c = synthetic_lda(num_docs=200, num_types=400, num_topics=10, doc_len=50, seed=5)
    m = oracle.MalletModel(10, 1.0, 0.01, c.num_types, c.doc_off, c.words, seed=1)
    ll0 = m.log_likelihood()
    m.estimate(30)
    assert m.log_likelihood() > ll0 + 0.05 * abs(ll0)


def test_exact_and_mallet_ll_same_formula(oracle):
    """Both restatements score the same z with the same modelLogLikelihood."""
    c = synthetic_changelists(num_docs=80, num_types=120, seed=8)
    K = 20
    m = oracle.MalletModel(K, 10.0, 0.01, c.num_types, c.doc_off, c.words, seed=3)
    m.estimate(3)
    o = oracle.ExactSampler(K, c.num_types, c.doc_off, c.words, 10.0 / K, 0.01, 1, z_init=m.z())
    o.apply()
    assert abs(o.log_likelihood() - m.log_likelihood()) < 1e-9 * abs(m.log_likelihood())


def test_large_k_draw_samples_the_exact_conditional(oracle):
    """exact_draw_big (the large-K kernel's draw, k_sample_big) is an exact
    sampler of p_k ~ (nd_k + a_k)(nw_wk - [k=zo] + b) / (nwsum_k - [k=zo] + V b):
    its own entry enters the word part uncorrected and is fixed by the accept
    / re-draw step, and the doc part is summed in fixed point.  Chi-square of
    its draws against the float64 conditional, including own entries that hold
    most of the mass (c = 40, 200) and a word seen once (c = 1, O = 0, the
    re-draw always taken)."""
    K, V = 2048, 40
    rng = np.random.default_rng(7)
    o = oracle.ExactSampler(K, V, np.array([0, 4], np.int64), np.zeros(4, np.int32), 0.05, 0.01, 5,
                            kind="sparse")
    for c_own, nd_own, others in [(1, 0, 0), (40, 5, 3), (200, 20, 1), (2, 1, 0), (5, 0, 40)]:
        nw = np.zeros((V, K), np.int32)
        zo, w = 777, 3
        nw[w, zo] = c_own
        for t in rng.choice(K, others, replace=False):
            nw[w, t] += rng.integers(1, 30)
        nw[10:] = rng.integers(0, 2, size=(V - 10, K))
        nwsum = nw.sum(0).astype(np.int32)
        o.load_snapshot(nw, nwsum)
        nd = np.zeros(o.Kp, np.int32)
        nd[zo] = nd_own
        for t in rng.choice(K, 5, replace=False):
            nd[t] += rng.integers(1, 4)
        nwr = nw[w].astype(np.float64)
        ns = nwsum.astype(np.float64)
        nwr[zo] -= 1
        ns[zo] -= 1
        p = (nd[:K] + 0.05) * (nwr + 0.01) / (ns + V * 0.01)
        p /= p.sum()
        n = 30000
        x = rng.integers(0, 2**32, size=(n, 4), dtype=np.uint64).astype(np.uint32)
        cnt = np.bincount([o.big_draw(w, nd, zo, x[j]) for j in range(n)], minlength=K)
        m = p * n > 20
        chi = ((cnt[m] - n * p[m]) ** 2 / (n * p[m])).sum()
        dof = max(int(m.sum()) - 1, 1)
        # the null's chi2/dof has sd sqrt(2/dof); 1 + 5 sd (or 6 for dof 1)
        assert chi / dof < 1 + 5 * np.sqrt(2 / dof) + (6 if dof == 1 else 0), (c_own, chi, dof)
        assert abs(cnt[zo] / n - p[zo]) < 5 * np.sqrt(p[zo] * (1 - p[zo]) / n) + 1e-4


def test_counts_checksum_definition(oracle):
    """oracle.counts_checksum (the restatement lda_counts_checksum is checked
    against on the GPU) equals its definition written as a loop: the sum mod
    2^64 over nonzero cells of splitmix64's finaliser of (index << 32 |
    uint32 value), nw cells at w K + k, nwsum cells at V K + k; zero cells add
    nothing, so the hash does not depend on the row padding; one changed
    count changes it."""
    M = (1 << 64) - 1

    def mix(x):
        x ^= x >> 30
        x = (x * 0xBF58476D1CE4E5B9) & M
        x ^= x >> 27
        x = (x * 0x94D049BB133111EB) & M
        return x ^ (x >> 31)

    rng = np.random.default_rng(4)
    V, K = 37, 11
    nw = rng.integers(0, 5, size=(V, K)) * (rng.random((V, K)) < 0.4)
    nw[3, 4] = 70000                        # beyond 16 bits
    nwsum = nw.sum(0)
    want = 0
    for w in range(V):
        for k in range(K):
            if nw[w, k]:
                want = (want + mix(((w * K + k) << 32) | (int(nw[w, k]) & 0xFFFFFFFF))) & M
    for k in range(K):
        if nwsum[k]:
            want = (want + mix(((V * K + k) << 32) | (int(nwsum[k]) & 0xFFFFFFFF))) & M
    assert oracle.counts_checksum(nw, nwsum) == want
    nw2 = nw.copy()
    nw2[0, 0] += 1
    assert oracle.counts_checksum(nw2, nwsum) != want
