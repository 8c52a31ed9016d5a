"""GPU parity at BASELINE.json's workload sizes, bit for bit against cpu_exact.

- C2 and C3 (100k docs x 200 tokens, V = 50k, K = 128 / K = 1024): the
  bench's corpora (corpus.synthetic_lda_torch, seed 20261015), the dense
  sampler bench.py times, z / nw / nwsum compared with the (threaded) oracle
  after the Philox initialisation and after each sweep.
- Philox counter word 1 (the high half of the global token index): shards
  whose token_base is >= 2^32, so `gtok >> 32` is non-zero on both sides.
- The whole C4 corpus in ONE context (11M docs x 200 = 2.2e9 tokens, so
  token indices and offsets cross 2^31): conservation, recount and the
  likelihood at full size, and a bit-exact check of the last documents'
  draws (global indices > 2^31) against the oracle run on that slice with
  the GPU's global snapshot loaded.
"""
import numpy as np
import pytest

from ldagibbssampling_amd.corpus import Corpus

pytestmark = pytest.mark.gpu


def _bench_corpus(docs, V, K, seed=20261015):
    from ldagibbssampling_amd.corpus import synthetic_lda_torch
    return synthetic_lda_torch(docs, V, K, doc_len=200, seed=seed, device="cuda:0")


def _same(g, o):
    np.testing.assert_array_equal(g.z(), o.z())
    gnw, gns, _, gds = g.counts()
    onw, ons, _, ods = o.counts()
    np.testing.assert_array_equal(gnw, onw)
    np.testing.assert_array_equal(gns, ons)
    np.testing.assert_array_equal(gds, ods)


@pytest.mark.parametrize("K,sweeps", [(128, 2), (1024, 2)])
def test_c2_c3_workload_bit_exact(oracle, K, sweeps):
    """C2 (K = 128) and C3 (K = 1024) at their full size, as bench.py runs them."""
    from ldagibbssampling_amd.sampler import GibbsSampler
    c = _bench_corpus(100_000, 50_000, K)
    assert c.num_tokens == 20_000_000
    alpha = np.full(K, 0.1)               # bench.py: alphaSum = 0.1 K, beta = 0.01, seed 1
    g = GibbsSampler(K, c.num_types, c.doc_off, c.words, alpha, 0.01, seed=1)
    o = oracle.ExactSampler(K, c.num_types, c.doc_off, c.words, alpha, 0.01, 1)
    g.sweep(0)
    o.apply()
    _same(g, o)
    for _ in range(sweeps):
        g.sweep(1)
        o.sweep(1)
        _same(g, o)
    lg, lo = g.log_likelihood(), o.log_likelihood()
    assert abs(lg - lo) <= 1e-9 * abs(lo), (lg, lo)


def _ragged(D, V, seed):
    rng = np.random.default_rng(seed)
    lens = rng.integers(0, 400, size=D)
    lens[::13] = 0
    off = np.zeros(D + 1, dtype=np.int64)
    np.cumsum(lens, out=off[1:])
    p = 1.0 / np.arange(1, V + 1) ** 1.05
    p /= p.sum()
    return Corpus(off, rng.choice(V, size=int(off[-1]), p=p).astype(np.int32), V)


@pytest.mark.parametrize("kind,K", [("dense", 20), ("dense", 512), ("dense", 1024),
                                    ("sparse", 256), ("sparse", 2048)])
def test_token_base_above_2_32(oracle, kind, K):
    """A shard whose global token indices start above 2^32: the Philox
    counter's high word is non-zero in every draw (init and sampling)."""
    from ldagibbssampling_amd.sampler import GibbsSampler
    c = _ragged(150, 900, seed=K)
    base = (1 << 32) + 123_457
    alpha = np.full(K, 0.1)
    g = GibbsSampler(K, c.num_types, c.doc_off, c.words, alpha, 0.01, seed=9, token_base=base,
                     sampler=kind)
    o = oracle.ExactSampler(K, c.num_types, c.doc_off, c.words, alpha, 0.01, 9, token_base=base,
                            kind=kind)
    g.sweep(0)
    o.apply()
    _same(g, o)
    g.sweep(2)
    o.sweep(2)
    _same(g, o)
    # the high word matters: the same shard at token_base mod 2^32 draws differently
    lo = GibbsSampler(K, c.num_types, c.doc_off, c.words, alpha, 0.01, seed=9,
                      token_base=base & 0xFFFFFFFF, sampler=kind)
    lo.sweep(2)
    assert not np.array_equal(lo.z(), g.z())


def test_full_c4_single_context():
    """BASELINE C4's whole corpus (10M docs in the config; 11M here so the
    2.2e9 token indices cross 2^31) in one context on one MI355X."""
    import torch
    from oracle import oracle as O
    from ldagibbssampling_amd.sampler import GibbsSampler
    docs, V, K = 11_000_000, 100_000, 512
    c = _bench_corpus(docs, V, K)
    N = c.num_tokens
    assert N == 2_200_000_000 and N > 2**31
    alpha = np.full(K, 0.1)
    g = GibbsSampler(K, V, c.doc_off, c.words, alpha, 0.01, seed=3)
    g.sweep(0)
    ll0 = g.log_likelihood()
    nw0, nwsum0, _, _ = g.counts()
    assert int(nw0.sum(dtype=np.int64)) == N
    z0 = g.z()

    # the last 2000 documents: global token indices above 2^31
    tail_docs = 2000
    d_first = docs - tail_docs
    t_first = int(c.doc_off[d_first])
    assert t_first > 2**31
    t_off = c.doc_off[d_first:] - t_first
    t_words = c.words[t_first:]
    o_init = O.ExactSampler(K, V, t_off, t_words, alpha, 0.01, 3, token_base=t_first)
    np.testing.assert_array_equal(z0[t_first:], o_init.z())        # Philox init
    del o_init

    g.sweep(1)
    z1 = g.z()
    o = O.ExactSampler(K, V, t_off, t_words, alpha, 0.01, 3, z_init=z0[t_first:],
                       token_base=t_first)
    o.load_snapshot(nw0, nwsum0)
    o.sample()                       # sweep 0 of the slice against the global snapshot
    np.testing.assert_array_equal(z1[t_first:], o.z())
    del o, z0, nw0

    g.sweep(2)
    z = g.z()
    assert z.min() >= 0 and z.max() < K
    nw, nwsum, _, _ = g.counts()
    assert int(nw.sum(dtype=np.int64)) == N
    np.testing.assert_array_equal(nw.sum(0, dtype=np.int64), nwsum.astype(np.int64))
    w = torch.as_tensor(c.words, device="cuda:0")
    cell = w.long() * K + torch.as_tensor(z, device="cuda:0").long()
    rc = torch.bincount(cell, minlength=V * K).reshape(V, K)
    del cell, w
    assert torch.equal(rc, torch.as_tensor(nw, device="cuda:0").long())
    del rc
    ll = g.log_likelihood()
    assert np.isfinite(ll0) and np.isfinite(ll) and ll > ll0
    g.close()
    torch.cuda.empty_cache()


@pytest.mark.parametrize("K,alpha_sum,beta", [(20, 10.0, 0.01), (500, 100.0, 1.0)])
def test_c1_workload_bit_exact(oracle, K, alpha_sum, beta):
    """BASELINE.json configs[0] at its size: 2000 changelist-shaped documents
    (Poisson(8) paths, Zipf(1.1) over 5000 paths), 100 sweeps, bit-exact
    z / nw / nwsum against cpu_exact -- at C1's K = 20 (quarter-wave kernel)
    and at src/cmu_ron's K = 500 (full-wave k_sample<8>)."""
    from ldagibbssampling_amd.corpus import synthetic_changelists
    from ldagibbssampling_amd.sampler import GibbsSampler
    c = synthetic_changelists(num_docs=2000, num_types=5000, seed=20261015)
    alpha = np.full(K, alpha_sum / K)
    g = GibbsSampler(K, c.num_types, c.doc_off, c.words, alpha, beta, seed=1)
    o = oracle.ExactSampler(K, c.num_types, c.doc_off, c.words, alpha, beta, 1)
    g.sweep(100)
    o.sweep(100)
    np.testing.assert_array_equal(g.z(), o.z())
    gnw, gns, _, _ = g.counts()
    onw, ons, _, _ = o.counts()
    np.testing.assert_array_equal(gnw, onw)
    np.testing.assert_array_equal(gns, ons)
