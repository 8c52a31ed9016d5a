"""GPU parity: the HIP sampler (through the C ABI) against cpu_exact.

Bar: bit-exact z, nw, nwsum, nd after 1..N sweeps (integer work); the fp64
log likelihood within 1e-9 relative (summation order differs); inference
theta within 1e-12 absolute (same integer samples, fp64 normalisation).
"""
import numpy as np
import pytest

from ldagibbssampling_amd.corpus import synthetic_lda, synthetic_changelists, Corpus

pytestmark = pytest.mark.gpu


def _ragged_corpus(D, V, seed, max_len=300, empty_every=17):
    rng = np.random.default_rng(seed)
    lens = rng.integers(0, max_len, size=D)
    lens[::empty_every] = 0                   # empty documents
    lens[3] = 1                               # single-token document
    if D > 10:
        lens[10] = 1500                       # spans many 64-token chunks
    off = np.zeros(D + 1, dtype=np.int64)
    np.cumsum(lens, out=off[1:])
    p = 1.0 / np.arange(1, V + 1) ** 1.05
    p /= p.sum()
    words = rng.choice(V, size=int(off[-1]), p=p).astype(np.int32)
    return Corpus(off, words, V)


def _pair(oracle, corpus, K, alpha, beta, seed, tokens_per_range=0, z_init=None, kind="dense"):
    from ldagibbssampling_amd.sampler import GibbsSampler
    g = GibbsSampler(K, corpus.num_types, corpus.doc_off, corpus.words, alpha, beta, seed=seed,
                     z_init=z_init, tokens_per_range=tokens_per_range, sampler=kind)
    o = oracle.ExactSampler(K, corpus.num_types, corpus.doc_off, corpus.words, alpha, beta, seed,
                            z_init=z_init, kind="sparse" if kind == "sparse" else "dense")
    return g, o


KINDS = ["dense", "sparse"]


def _assert_same_state(g, o, with_nd=True):
    np.testing.assert_array_equal(g.z(), o.z())
    gnw, gns, gnd, gds = g.counts(with_nd=with_nd)
    onw, ons, ond, ods = o.counts(with_nd=with_nd)
    np.testing.assert_array_equal(gnw, onw)
    np.testing.assert_array_equal(gns, ons)
    np.testing.assert_array_equal(gds, ods)
    if with_nd:
        np.testing.assert_array_equal(gnd, ond)


@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("K", [20, 64, 100, 128, 256, 512, 1000, 1024])
def test_sweeps_bit_exact(oracle, K, kind):
    corpus = _ragged_corpus(D=120, V=700, seed=K)
    alpha = np.full(K, 0.1)
    g, o = _pair(oracle, corpus, K, alpha, 0.01, seed=1234 + K, tokens_per_range=300, kind=kind)
    g.sweep(0)
    o.apply()
    _assert_same_state(g, o)                  # Philox initialisation
    for n in (1, 2):
        g.sweep(n)
        o.sweep(n)
        _assert_same_state(g, o)


@pytest.mark.parametrize("kind", KINDS)
def test_non_power_of_two_padding(oracle, kind):
    """K=300 pads to Kp=512 (C=8): padded topics never drawn."""
    corpus = _ragged_corpus(D=60, V=400, seed=300)
    K = 300
    g, o = _pair(oracle, corpus, K, np.full(K, 0.05), 0.01, seed=3, kind=kind)
    assert g.Kp == 512
    g.sweep(2)
    o.sweep(2)
    _assert_same_state(g, o)
    assert g.z().max() < K


@pytest.mark.parametrize("K", [1500, 2048, 4096])
def test_large_k_sparse_bit_exact(oracle, K):
    """K > 1024 (C = 32, 64): grouped doc-part partials, streamed word rounds,
    16-bit document counts in LDS."""
    corpus = _ragged_corpus(D=80, V=600, seed=K)
    alpha = np.full(K, 50.0 / K)
    g, o = _pair(oracle, corpus, K, alpha, 0.01, seed=K + 1, tokens_per_range=400, kind="sparse")
    g.sweep(0)
    o.apply()
    _assert_same_state(g, o)
    for n in (1, 3):
        g.sweep(n)
        o.sweep(n)
        _assert_same_state(g, o)
    lg, lo = g.log_likelihood(), o.log_likelihood()
    assert abs(lg - lo) <= 1e-9 * abs(lo), (lg, lo)


@pytest.mark.parametrize("D,L", [(0, 0), (2, 5)])
def test_large_k_ring_probe_with_empty_first_part(oracle, D, L):
    """The large-K sampler times its ring depths on sweeps 8-10 (big_rb_next).
    An empty shard launches nothing, and under the staleness schedule a tiny
    shard's part 0 is empty (D=2, L=5: parts [], [docs 0-1]); the probe then
    times the first launch that runs, or none, and decides only on three
    equal launches -- sweeps past the decision keep working, bit-exact."""
    K = 1500
    rng = np.random.default_rng(D + L)
    off = np.arange(D + 1, dtype=np.int64) * L
    corpus = Corpus(off, rng.integers(0, 40, size=D * L).astype(np.int32), 40)
    g, o = _pair(oracle, corpus, K, np.full(K, 0.05), 0.01, seed=9, kind="sparse")
    if D:
        g.set_sequential_sweeps(*oracle.staleness_schedule(4))
        o.set_sequential_sweeps(*oracle.staleness_schedule(4))
        o.apply()
        assert o._sweep_runs()[0] == []          # the first part is empty
        g.sweep(0)
    for _ in range(14):
        g.sweep(1)
    o.sweep(14)
    _assert_same_state(g, o)


def test_large_k_sparse_long_rows_and_inference(oracle):
    """Frequent words with > 128 nonzero topics (more rounds than the prefetch
    ring holds), then frozen-model inference at K=4096."""
    c = synthetic_lda(num_docs=150, num_types=300, num_topics=64, doc_len=None, mean_len=400,
                      min_len=1, max_len=1200, seed=4)
    train, held = c.subset(range(0, 120)), c.subset(range(120, 150))
    K = 4096
    g, o = _pair(oracle, train, K, np.full(K, 0.01), 0.05, seed=6, kind="sparse")
    g.sweep(4)
    o.sweep(4)
    _assert_same_state(g, o)
    assert (g.counts()[0] > 0).sum(1).max() > 128
    tg = g.infer(held.doc_off, held.words, n_iter=6, burn_in=2, thin=2, seed=8)
    to = o.infer(held.doc_off, held.words, n_iter=6, burn_in=2, thin=2, seed=8)
    np.testing.assert_allclose(tg, to, rtol=0, atol=1e-12)


@pytest.mark.parametrize("K", [1500, 4096])
def test_large_k_symmetric_and_asymmetric_alpha(oracle, K):
    """The large-K sampler has a symmetric-alpha instantiation (alpha in a
    register, an inv-only LDS table) and the general one; a run that switches
    symmetric -> asymmetric -> symmetric alpha (as the optimisation does after
    its burn-in) stays bit-exact through both, and so does inference."""
    corpus = _ragged_corpus(D=80, V=600, seed=K + 3)
    train = corpus.subset(range(0, 64))
    held = corpus.subset(range(64, 80))
    alpha = np.full(K, 20.0 / K)
    g, o = _pair(oracle, train, K, alpha, 0.01, seed=K + 5, tokens_per_range=300, kind="sparse")
    g.sweep(2)
    o.sweep(2)
    _assert_same_state(g, o)
    rng = np.random.default_rng(K)
    alpha2 = rng.uniform(0.5, 2.0, size=K) * (20.0 / K)
    # one topic differing in its fp32 value is enough to leave the symmetric path
    alpha3 = alpha.copy()
    alpha3[K - 1] *= 1.25
    for a in (alpha2, alpha3, np.full(K, 30.0 / K)):
        g.set_alpha_beta(a, 0.02)
        o.set_alpha_beta(a, 0.02)
        g.sweep(2)
        o.sweep(2)
        _assert_same_state(g, o)
        tg = g.infer(held.doc_off, held.words, n_iter=4, burn_in=1, thin=1, seed=3)
        to = o.infer(held.doc_off, held.words, n_iter=4, burn_in=1, thin=1, seed=3)
        np.testing.assert_allclose(tg, to, rtol=0, atol=1e-12)


def test_large_k_limits():
    from ldagibbssampling_amd.sampler import GibbsSampler
    from ldagibbssampling_amd.capi import LdaError
    off = np.array([0, 3], dtype=np.int64)
    w = np.array([1, 2, 3], np.int32)
    with pytest.raises(LdaError, match="SPARSE"):
        GibbsSampler(2000, 10, off, w, 0.1, 0.01, sampler="dense")
    with pytest.raises(LdaError):
        GibbsSampler(5000, 10, off, w, 0.1, 0.01, sampler="sparse")
    long_off = np.array([0, 70000], dtype=np.int64)
    with pytest.raises(LdaError, match="65535"):
        GibbsSampler(2048, 10, long_off, np.zeros(70000, np.int32), 0.1, 0.01, sampler="sparse")


@pytest.mark.parametrize("kind", KINDS)
def test_many_sweeps_and_loglik(oracle, kind):
    c = synthetic_lda(num_docs=300, num_types=2000, num_topics=128, doc_len=None, mean_len=80,
                      min_len=1, max_len=400, seed=7)
    K = 128
    g, o = _pair(oracle, c, K, np.full(K, 0.1), 0.01, seed=99, kind=kind)
    g.sweep(10)
    o.sweep(10)
    _assert_same_state(g, o)
    lg, lo = g.log_likelihood(), o.log_likelihood()
    assert abs(lg - lo) <= 1e-9 * abs(lo), (lg, lo)


@pytest.mark.parametrize("kind", KINDS)
def test_asymmetric_alpha_and_z_init(oracle, kind):
    c = synthetic_changelists(num_docs=400, num_types=900, seed=3)
    K = 20
    rng = np.random.default_rng(5)
    alpha = rng.uniform(0.05, 2.0, size=K)
    z0 = rng.integers(0, K, size=c.num_tokens).astype(np.int32)
    g, o = _pair(oracle, c, K, alpha, 0.001, seed=2**40 + 17, z_init=z0, kind=kind)
    g.sweep(5)
    o.sweep(5)
    _assert_same_state(g, o)
    # hyperparameters replaced mid-run (host-side optimisation hook)
    alpha2 = alpha * 1.5
    g.set_alpha_beta(alpha2, 0.002)
    o.set_alpha_beta(alpha2, 0.002)
    g.sweep(2)
    o.sweep(2)
    _assert_same_state(g, o)


@pytest.mark.parametrize("kind", KINDS)
def test_sharded_equals_single(oracle, kind):
    """AD-LDA over 3 shards (delta summed on the host) == one shard, bit for bit."""
    from ldagibbssampling_amd.sampler import GibbsSampler
    c = _ragged_corpus(D=90, V=500, seed=11)
    K, seed = 128, 77
    alpha = np.full(K, 0.2)
    single = GibbsSampler(K, c.num_types, c.doc_off, c.words, alpha, 0.01, seed=seed, sampler=kind)
    cuts = [0, 30, 61, 90]
    shards = [GibbsSampler(K, c.num_types, c.doc_off[a:b + 1], c.words[c.doc_off[a]:c.doc_off[b]],
                           alpha, 0.01, seed=seed, token_base=int(c.doc_off[a]), sampler=kind)
              for a, b in zip(cuts[:-1], cuts[1:])]
    import torch

    def allreduce():
        ts = [s.delta_tensor() for s in shards]
        tot = sum(t.clone() for t in ts)
        for t in ts:
            t.copy_(tot)
        torch.cuda.synchronize()

    for s in shards:
        s.synchronize()
    allreduce()
    for s in shards:
        s.apply()
    single.sweep(0)
    for _ in range(3):
        for s in shards:
            s.sample()
            s.synchronize()
        allreduce()
        for s in shards:
            s.apply()
        single.sweep(1)
    z = np.concatenate([s.z() for s in shards])
    np.testing.assert_array_equal(z, single.z())
    for s in shards:
        np.testing.assert_array_equal(s.counts()[0], single.counts()[0])
        np.testing.assert_array_equal(s.counts()[1], single.counts()[1])
    o = oracle.ExactSampler(K, c.num_types, c.doc_off, c.words, alpha, 0.01, seed, kind=kind)
    o.sweep(3)
    np.testing.assert_array_equal(single.z(), o.z())


@pytest.mark.parametrize("kind", KINDS)
def test_inference_matches_oracle(oracle, kind):
    c = synthetic_lda(num_docs=200, num_types=1500, num_topics=64, doc_len=None, mean_len=60,
                      min_len=2, max_len=200, seed=21)
    train, held = c.subset(range(0, 160)), c.subset(range(160, 200))
    K = 64
    g, o = _pair(oracle, train, K, np.full(K, 0.1), 0.01, seed=5, kind=kind)
    g.sweep(20)
    o.sweep(20)
    _assert_same_state(g, o, with_nd=False)
    tg = g.infer(held.doc_off, held.words, n_iter=30, burn_in=10, thin=5, seed=8)
    to = o.infer(held.doc_off, held.words, n_iter=30, burn_in=10, thin=5, seed=8)
    np.testing.assert_allclose(tg, to, rtol=0, atol=1e-12)
    np.testing.assert_allclose(tg.sum(1), 1.0, atol=1e-12)


def test_mallet_packed_layout(oracle):
    c = synthetic_changelists(num_docs=200, num_types=400, seed=9)
    K = 20
    g, _ = _pair(oracle, c, K, np.full(K, 0.5), 0.01, seed=1)
    g.sweep(3)
    rows, row_off, bits = g.mallet_packed()
    nw = g.counts()[0]
    assert bits == 5                                # K=20 -> topicMask 31
    for w in range(c.num_types):
        r = rows[row_off[w]:row_off[w + 1]]
        assert len(r) == min(K, nw[w].sum())
        assert np.all(np.diff(r.astype(np.int64)) <= 0)   # sorted descending
        live = r[r > 0]
        dense = np.zeros(K, np.int32)
        dense[live & 31] = live >> 5
        np.testing.assert_array_equal(dense, nw[w])


def test_errors_are_loud():
    from ldagibbssampling_amd.sampler import GibbsSampler
    from ldagibbssampling_amd.capi import LdaError
    off = np.array([0, 3], dtype=np.int64)
    with pytest.raises(LdaError):
        GibbsSampler(2000, 10, off, np.array([1, 2, 3], np.int32), 0.1, 0.01)   # K too large
    with pytest.raises(LdaError):
        GibbsSampler(8, 10, off, np.array([1, 2, 30], np.int32), 0.1, 0.01)    # word >= V
    g = GibbsSampler(8, 10, off, np.array([1, 2, 3], np.int32), 0.1, 0.01)
    with pytest.raises(LdaError):
        g.sample()                                       # pending delta after create
    g.sweep(1)
    assert g.z().shape == (3,)


def test_empty_corpus():
    from ldagibbssampling_amd.sampler import GibbsSampler
    off = np.zeros(4, dtype=np.int64)
    g = GibbsSampler(16, 10, off, np.zeros(0, np.int32), 0.1, 0.01)
    g.sweep(2)
    nw, nwsum, nd, ndsum = g.counts(with_nd=True)
    assert nw.sum() == 0 and nwsum.sum() == 0 and nd.sum() == 0 and ndsum.sum() == 0


def test_sparse_saturated_counts(oracle):
    """Entries whose count overflows the packed 20-bit field (>= 2^20 - 1) are
    read exactly from the dense row: one very frequent word."""
    from ldagibbssampling_amd.corpus import Corpus
    D, L = 40, 60000
    rng = np.random.default_rng(1)
    words = np.where(rng.random(D * L) < 0.97, 0, rng.integers(1, 50, D * L)).astype(np.int32)
    c = Corpus(np.arange(D + 1, dtype=np.int64) * L, words, 50)
    K = 2
    g, o = _pair(oracle, c, K, np.full(K, 0.1), 0.01, seed=3, kind="sparse")
    g.sweep(2)
    o.sweep(2)
    assert g.counts()[0].max() >= (1 << 20) - 1
    _assert_same_state(g, o, with_nd=False)


def test_large_k_saturated_counts(oracle):
    """The large-K sampler's saturated entries: a count >= 2^20 - 1
    does not fit the packed 20-bit field, and k_sample_big reads it from the
    dense row in three places -- the B-part term, the own-entry accept step
    (which reloads c of the selected entry) and the re-walk after a re-draw.
    K = 1500 (C = 32), one word holding 97% of 2.4M tokens, its tokens
    assigned in order so that topic 0 starts at exactly 2^20 - 1 (the first
    saturated value; the first sweep moves it below), topic 1 at 2^20 + 20000
    (saturated in every sweep: ~99% of the word's draws and own entries hit
    it) and topic 2 the rest; every other token starts at a random topic.
    Bit-exact against exact_draw_big for 4 sweeps."""
    D, L, K = 40, 60000, 1500
    rng = np.random.default_rng(11)
    words = np.where(rng.random(D * L) < 0.97, 0, rng.integers(1, 50, D * L)).astype(np.int32)
    c = Corpus(np.arange(D + 1, dtype=np.int64) * L, words, 50)
    sat = (1 << 20) - 1
    hot = np.flatnonzero(words == 0)
    n1 = sat + 20001
    assert len(hot) > sat + n1
    z0 = rng.integers(0, K, D * L).astype(np.int32)
    z0[hot[:sat]] = 0
    z0[hot[sat:sat + n1]] = 1
    z0[hot[sat + n1:]] = 2
    g, o = _pair(oracle, c, K, np.full(K, 0.1), 0.01, seed=5, z_init=z0, kind="sparse")
    g.sweep(0)
    o.apply()
    assert g.counts()[0][0, 0] == sat and g.counts()[0][0, 1] == n1
    for _ in range(4):
        g.sweep(1)
        o.sweep(1)
        _assert_same_state(g, o, with_nd=False)
        assert g.counts()[0][0, 1] >= sat          # the saturated path runs every sweep


@pytest.mark.parametrize("kind", ["dense", "sparse"])
def test_wide_rows_escape(oracle, kind):
    """Large counts (> 65535) through both draws: fp32 conversion of big counts
    in the dense word factors, exact escape reads in the sparse entries."""
    from ldagibbssampling_amd.corpus import Corpus
    D, L = 8, 40000
    rng = np.random.default_rng(2)
    words = np.where(rng.random(D * L) < 0.9, 0, rng.integers(1, 300, D * L)).astype(np.int32)
    c = Corpus(np.arange(D + 1, dtype=np.int64) * L, words, 300)
    K = 3
    g, o = _pair(oracle, c, K, np.full(K, 0.1), 0.01, seed=4, kind=kind)
    g.sweep(2)
    o.sweep(2)
    assert g.counts()[0].max() > 65535
    _assert_same_state(g, o, with_nd=False)


@pytest.mark.parametrize("K", [20, 512, 1024])
def test_dense_16bit_row_boundary(oracle, K):
    """Counts at the 16-bit row's edge: a cell of exactly 65535 (the largest
    count the 16-bit row holds; its own-token correction reads 65534) beside
    cells of 65536-65538 (the word's row is flagged wide and read from the
    int32 row), with counts crossing the boundary in both directions over the
    sweeps."""
    from ldagibbssampling_amd.corpus import Corpus
    D, L = 4, 50000
    rng = np.random.default_rng(K)
    n0, n1 = 65535 + 40, 65537 + 40          # tokens of word 0 and word 1
    words = np.concatenate([np.zeros(n0, np.int32), np.ones(n1, np.int32),
                            rng.integers(2, 300, D * L - n0 - n1).astype(np.int32)])
    z0 = np.concatenate([np.full(n0, 3), np.full(n1, 5),
                         rng.integers(0, K, D * L - n0 - n1)]).astype(np.int32)
    z0[:40] = 4                                # word 0: topic 3 holds exactly 65535
    z0[n0:n0 + 40] = 6                         # word 1: topic 5 holds 65537
    perm = rng.permutation(D * L)
    c = Corpus(np.arange(D + 1, dtype=np.int64) * L, words[perm], 300)
    # a tiny alpha and beta keep most tokens on their topic: the cells move a
    # few counts per sweep around the boundary
    g, o = _pair(oracle, c, K, np.full(K, 1e-3), 1e-4, seed=K + 5, z_init=z0[perm])
    g.sweep(0)
    o.apply()
    nw = g.counts()[0]
    assert nw[0, 3] == 65535 and nw[1, 5] == 65537
    _assert_same_state(g, o, with_nd=False)
    seen_lo = seen_hi = False
    for _ in range(4):
        g.sweep(1)
        o.sweep(1)
        _assert_same_state(g, o, with_nd=False)
        nw = g.counts()[0]
        seen_lo |= nw[1, 5] <= 65535
        seen_hi |= nw[0, 3] > 65535 or nw[1, 5] > 65535
    assert seen_hi


@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("K", [20, 512, 1024])
def test_range_tails_and_chunk_edges(oracle, K, kind):
    # one document per work range (tokens_per_range=1), so every range length
    # below occurs: fewer tokens than the prefetch depth P (the sampler then
    # prefetches past the range end from stale but valid word ids), and
    # documents ending just before, at and after the 64-token chunk edges
    lens = list(range(0, 10)) + [62, 63, 64, 65, 66, 126, 127, 128, 129, 130,
                                 190, 191, 192, 193, 194, 255, 256, 257]
    rng = np.random.default_rng(K)
    lens = np.array(lens * 2, dtype=np.int64)
    rng.shuffle(lens)
    off = np.zeros(len(lens) + 1, dtype=np.int64)
    np.cumsum(lens, out=off[1:])
    V = 300
    words = rng.integers(0, V, size=int(off[-1])).astype(np.int32)
    corpus = Corpus(off, words, V)
    alpha = np.full(K, 0.1)
    g, o = _pair(oracle, corpus, K, alpha, 0.01, seed=77 + K, tokens_per_range=1, kind=kind)
    g.sweep(0)
    o.apply()
    _assert_same_state(g, o)
    for n in (1, 2):
        g.sweep(n)
        o.sweep(n)
        _assert_same_state(g, o)


@pytest.mark.parametrize("kind", KINDS)
def test_inference_skips_types_without_training_tokens(oracle, kind):
    """Held-out tokens of in-vocabulary types that have no training tokens
    (Mallet allocates them an empty typeTopicCounts row, and its inferencer
    skips them): dropped on the GPU as in cpu_exact; a document made only of
    such tokens gets theta = alpha / alphaSum, as in cpu_mallet."""
    c = synthetic_lda(num_docs=120, num_types=800, num_topics=32, doc_len=None, mean_len=50,
                      min_len=2, max_len=120, seed=12)
    V = c.num_types + 50                       # 50 types never seen in training
    K = 32
    alpha = np.full(K, 0.1)
    from ldagibbssampling_amd.sampler import GibbsSampler
    g = GibbsSampler(K, V, c.doc_off, c.words, alpha, 0.01, seed=2, sampler=kind)
    o = oracle.ExactSampler(K, V, c.doc_off, c.words, alpha, 0.01, 2,
                            kind="sparse" if kind == "sparse" else "dense")
    g.sweep(5)
    o.sweep(5)
    rng = np.random.default_rng(3)
    unseen = np.arange(c.num_types, V, dtype=np.int32)
    docs = [rng.choice(unseen, 9),                                          # only unseen types
            np.concatenate([rng.integers(0, c.num_types, 30), rng.choice(unseen, 10)]),
            rng.integers(0, c.num_types, 25)]
    docs = [d.astype(np.int32) for d in docs]
    off = np.zeros(len(docs) + 1, np.int64)
    np.cumsum([len(d) for d in docs], out=off[1:])
    words = np.concatenate(docs)
    tg = g.infer(off, words, n_iter=20, burn_in=4, thin=4, seed=5)
    to = o.infer(off, words, n_iter=20, burn_in=4, thin=4, seed=5)
    np.testing.assert_allclose(tg, to, rtol=0, atol=1e-12)
    np.testing.assert_allclose(tg[0], alpha / alpha.sum(), rtol=0, atol=1e-15)
    # the mixed document equals the same document with its unseen tokens removed
    t_clean = g.infer(np.array([0, 30], np.int64), docs[1][:30], n_iter=20, burn_in=4, thin=4,
                      seed=5)
    m = oracle.MalletModel(K, alpha.sum(), 0.01, V, c.doc_off, c.words, seed=1)
    m.estimate(5)
    tm = m.infer(off[:2], docs[0], n_iter=20, burn_in=4, thin=4, seed=5)
    np.testing.assert_allclose(tm[0], alpha / alpha.sum(), rtol=0, atol=1e-15)
    np.testing.assert_array_equal(tg[1], t_clean[0])


@pytest.mark.parametrize("variant", [1, 2])
@pytest.mark.parametrize("K", [3, 12, 20, 48, 100, 128])
def test_dense_half_wave_variant(oracle, K, variant, monkeypatch):
    """The dense variants for K <= 128 -- two documents per wave (opt-in,
    LDA_DENSE_HALF=1, exact_draw_half) and four (=2, exact_draw_quarter, the
    default) --
    against their own oracle draws: ragged
    documents (empty, one token, 1500 tokens) over short work ranges, so the
    two halves switch ranges, chunks and documents at different steps and one
    half idles at the end; counts > 65535 (the int32-row path) at K = 3;
    inference (the frozen kernel)."""
    from ldagibbssampling_amd.sampler import GibbsSampler
    from ldagibbssampling_amd.corpus import Corpus
    monkeypatch.setenv("LDA_DENSE_HALF", str(variant))     # 1 half-wave, 2 quarter-wave
    if K == 3:
        rng = np.random.default_rng(2)
        D, L = 8, 40000
        words = np.where(rng.random(D * L) < 0.9, 0, rng.integers(1, 300, D * L)).astype(np.int32)
        corpus = Corpus(np.arange(D + 1, dtype=np.int64) * L, words, 300)
    else:
        corpus = _ragged_corpus(D=150, V=700, seed=K)
    alpha = np.full(K, 0.1)
    g = GibbsSampler(K, corpus.num_types, corpus.doc_off, corpus.words, alpha, 0.01, seed=77 + K,
                     tokens_per_range=100)
    o = oracle.ExactSampler(K, corpus.num_types, corpus.doc_off, corpus.words, alpha, 0.01, 77 + K,
                            half=variant)
    for n in (1, 2):
        g.sweep(n)
        o.sweep(n)
        _assert_same_state(g, o, with_nd=K != 3)
    if K == 3:
        assert g.counts()[0].max() > 65535
        return
    held = _ragged_corpus(D=30, V=700, seed=K + 1, empty_every=7)
    tg = g.infer(held.doc_off, held.words, n_iter=20, burn_in=5, thin=5, seed=3)
    to = o.infer(held.doc_off, held.words, n_iter=20, burn_in=5, thin=5, seed=3)
    np.testing.assert_allclose(tg, to, rtol=0, atol=1e-12)


@pytest.mark.parametrize("ring", ["short", "default", "auto"])
def test_large_k_sparse_very_long_rows(oracle, monkeypatch, ring):
    """Word rows far longer than the register rounds (K = 4096): rows of up
    to ~3500 entries, so a draw can land in the register rounds, in either of
    the batches whose running sums are kept, or past them (the re-read of
    the rest of the selected lane), and the sparse rows are padded to whole
    64-entry rounds.  ring: the sampler's ring, fixed at the short (6 rounds
    x 4 slots) or the default (12 x 2) one (LDA_SB_RB) or chosen by timing
    both (round 4): the same sums in the same order, so the same draws."""
    if ring != "auto":
        monkeypatch.setenv("LDA_SB_RB", ring)
    from ldagibbssampling_amd.corpus import Corpus
    rng = np.random.default_rng(12)
    D, L, V = 600, 300, 2000
    p = np.empty(V)
    p[:40] = np.geomspace(0.05, 0.002, 40)       # a few very frequent words
    p[40:] = (1.0 - p[:40].sum()) / (V - 40)
    words = rng.choice(V, size=D * L, p=p / p.sum()).astype(np.int32)
    c = Corpus(np.arange(D + 1, dtype=np.int64) * L, words, V)
    K = 4096
    g, o = _pair(oracle, c, K, np.full(K, 0.05), 0.01, seed=31, kind="sparse")
    g.sweep(2)
    o.sweep(2)
    _assert_same_state(g, o, with_nd=False)
    nnz = (g.counts()[0] > 0).sum(1)
    rounds = (nnz + 63) // 64
    assert rounds.max() > 10 + 8 * 3                 # past every kept batch
    assert ((rounds > 10) & (rounds <= 18)).any() and ((rounds > 18) & (rounds <= 26)).any()
    if ring == "auto":          # sweeps 8-10 probe both depths, 11-13 take the faster
        g.sweep(12)
        o.sweep(12)
        _assert_same_state(g, o, with_nd=False)
