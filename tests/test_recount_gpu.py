"""The dense samplers' two count-update modes against cpu_exact.

RECOUNT (the default): the sampler writes only z, then k_recount rebuilds
every word row of the shard from a word-sorted token index into the exchange
buffer, and the apply replaces nw / nwsum with the (summed) buffer.  DELTA
(LDA_RECOUNT=0): the sampler's per-chunk atomics into a delta that the apply
adds.  Both are integer counts of the same z, so both must be bit-exact
against cpu_exact, which keeps Mallet's delta form (sumTypeTopicCounts sums
the workers' local counts [M]; the order of integer adds is immaterial).

Covered: every dense kernel family (quarter-wave K <= 128, full-wave up to
1024), words split over several recount work items (more than
RECOUNT_ITEM_TOKENS = 1024 tokens of one word in one part), split sweeps
(parts 1..4, per-part indices), empty documents, counts above 65535 (int32
rows), lda_set_z, and sharded contexts summing their buffers.
"""
import os
from types import SimpleNamespace

import numpy as np
import pytest

from ldagibbssampling_amd.corpus import Corpus

pytestmark = pytest.mark.gpu


def _corpus(D, V, seed, max_len=400, zipf=1.05, heavy=None):
    rng = np.random.default_rng(seed)
    lens = rng.integers(0, max_len, size=D)
    lens[::13] = 0
    if heavy:
        lens[5] = heavy
    off = np.zeros(D + 1, dtype=np.int64)
    np.cumsum(lens, out=off[1:])
    p = 1.0 / np.arange(1, V + 1) ** zipf
    p /= p.sum()
    words = rng.choice(V, size=int(off[-1]), p=p).astype(np.int32)
    return Corpus(off, words, V)


def _sampler(corpus, K, seed, mode, **kw):
    from ldagibbssampling_amd.sampler import GibbsSampler
    old = os.environ.get("LDA_RECOUNT")
    os.environ["LDA_RECOUNT"] = "1" if mode == "recount" else "0"
    try:
        return GibbsSampler(K, corpus.num_types, corpus.doc_off, corpus.words, np.full(K, 0.1), 0.01,
                            seed=seed, **kw)
    finally:
        if old is None:
            os.environ.pop("LDA_RECOUNT")
        else:
            os.environ["LDA_RECOUNT"] = old


def _same(g, o):
    np.testing.assert_array_equal(g.z(), o.z())
    gnw, gns, _, _ = g.counts()
    onw, ons, _, _ = o.counts()
    np.testing.assert_array_equal(gnw, onw)
    np.testing.assert_array_equal(gns, ons)


@pytest.mark.parametrize("mode", ["recount", "delta"])
@pytest.mark.parametrize("K", [20, 128, 200, 512, 1024])
def test_modes_bit_exact(oracle, K, mode):
    # V = 60 with ~90k tokens: the frequent words hold several thousand
    # tokens, i.e. several recount items each (device-atomic rows)
    c = _corpus(D=400, V=60 if K <= 200 else 600, seed=K, heavy=3000)
    g = _sampler(c, K, 5 + K, mode, tokens_per_range=200)
    assert g.count_update()[0] == mode
    o = oracle.ExactSampler(K, c.num_types, c.doc_off, c.words, np.full(K, 0.1), 0.01, 5 + K)
    for n in (0, 1, 3):
        g.sweep(n)
        o.sweep(n)
        _same(g, o)
    if mode == "recount":
        assert np.all(g.recount_times(4) > 0)
        assert int(g.delta_tensor().abs().sum()) == 0      # the apply leaves the buffer zero


@pytest.mark.parametrize("parts", [2, 3, 4])
def test_recount_split_sweeps(oracle, parts):
    c = _corpus(D=300, V=80, seed=parts, heavy=2500)
    K = 128
    g = _sampler(c, K, 9, "recount", tokens_per_range=100)
    o = oracle.ExactSampler(K, c.num_types, c.doc_off, c.words, np.full(K, 0.1), 0.01, 9)
    g.sweep(1)
    o.sweep(1)
    g.set_exchange_parts(parts)
    for _ in range(2):
        for i in range(parts):
            g.sample_part(i)
        g.apply()
        o.sweep(1)
        _same(g, o)
    g.set_exchange_parts(1)       # the index is rebuilt for one part again
    g.sweep(2)
    o.sweep(2)
    _same(g, o)


def test_recount_wide_rows_and_set_z(oracle):
    """Counts above 65535 (the int32-row path of the 16-bit rows) through the
    recount, then lda_set_z re-seeding the counts."""
    rng = np.random.default_rng(3)
    D, L = 400, 400
    off = np.arange(D + 1, dtype=np.int64) * L
    words = np.where(rng.random(D * L) < 0.6, 0, rng.integers(1, 40, D * L)).astype(np.int32)
    c = Corpus(off, words, 40)
    K = 64
    g = _sampler(c, K, 21, "recount")
    o = oracle.ExactSampler(K, c.num_types, c.doc_off, c.words, np.full(K, 0.1), 0.01, 21)
    g.sweep(2)
    o.sweep(2)
    _same(g, o)
    z = rng.integers(0, K, D * L).astype(np.int32)
    z[words == 0] = 7                       # word 0's topic-7 cell: ~96k tokens
    g.set_z(z)
    o2 = oracle.ExactSampler(K, c.num_types, c.doc_off, c.words, np.full(K, 0.1), 0.01, 21, z_init=z)
    o2.sweep_index = g.sweep_index
    g.sweep(0)
    o2.sweep(0)
    _same(g, o2)
    assert g.counts()[0][0, 7] > 65535
    g.sweep(2)
    o2.sweep(2)
    _same(g, o2)


def test_recount_shards_sum(oracle):
    """Three shards in recount mode: each buffer holds its shard's counts;
    their sum replaces nw on every shard (the AD-LDA exchange)."""
    import torch
    c = _corpus(D=150, V=100, seed=4, heavy=2000)
    K = 100
    cuts = [0, 40, 101, 150]
    shards = []
    for a, b in zip(cuts[:-1], cuts[1:]):
        sub = SimpleNamespace(doc_off=c.doc_off[a:b + 1], words=c.words[c.doc_off[a]:c.doc_off[b]],
                              num_types=c.num_types)
        shards.append(_sampler(sub, K, 31, "recount", token_base=int(c.doc_off[a])))
    o = oracle.ExactSampler(K, c.num_types, c.doc_off, c.words, np.full(K, 0.1), 0.01, 31)

    def exchange():
        for s in shards:
            s.synchronize()
        ts = [s.delta_tensor() for s in shards]
        tot = sum(t.clone() for t in ts)
        for t in ts:
            t.copy_(tot)
        torch.cuda.synchronize()
        for s in shards:
            s.apply()

    exchange()
    o.sweep(0)
    for _ in range(3):
        for s in shards:
            s.sample()
        exchange()
        o.sweep(1)
    np.testing.assert_array_equal(np.concatenate([s.z() for s in shards]), o.z())
    onw, ons, _, _ = o.counts()
    for s in shards:
        np.testing.assert_array_equal(s.counts()[0], onw)
        np.testing.assert_array_equal(s.counts()[1], ons)


def test_auto_mode_switches_to_delta(oracle):
    """LDA_COUNT_AUTO (the default): the first recount_sweeps sweeps after the
    counts are seeded recount, later ones keep a delta; lda_set_z re-seeds.
    Bit-exact throughout."""
    c = _corpus(D=300, V=200, seed=8, heavy=1500)
    K = 64
    from ldagibbssampling_amd.sampler import GibbsSampler
    g = GibbsSampler(K, c.num_types, c.doc_off, c.words, np.full(K, 0.1), 0.01, seed=2)
    assert g.count_update() == ("auto", 0)     # < 2^20 tokens: no recount by default
    g.set_count_update("auto", 3)
    o = oracle.ExactSampler(K, c.num_types, c.doc_off, c.words, np.full(K, 0.1), 0.01, 2)
    g.sweep(0)
    o.sweep(0)
    modes = []
    for _ in range(6):
        modes.append(g.recount)           # the mode the next sweep will use
        g.sweep(1)
        o.sweep(1)
        _same(g, o)
    assert modes == [True, True, True, False, False, False]
    rc = g.recount_times(6)
    assert np.all(rc[:3] > 0)
    g.set_z(o.z())                        # re-seeded: recounts again
    assert g.recount is False             # the seeded counts are pending as a delta
    g.sweep(0)
    assert g.recount is True
    g.set_count_update("delta")
    assert g.recount is False
    g.sweep(2)
    o.sweep(2)
    _same(g, o)
