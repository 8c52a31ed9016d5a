"""GPU statistics for hyperparameter optimisation: bit-exact integer
histograms (Mallet's docLengthCounts / topicDocCounts / countHistogram)
against numpy on the same state."""
import numpy as np
import pytest

from ldagibbssampling_amd.corpus import synthetic_lda

pytestmark = pytest.mark.gpu


def _nd(z, doc_off, K):
    D = len(doc_off) - 1
    nd = np.zeros((D, K), np.int64)
    doc = np.repeat(np.arange(D), np.diff(doc_off))
    np.add.at(nd, (doc, z), 1)
    return nd


@pytest.mark.parametrize("kind,K", [("dense", 20), ("dense", 512), ("sparse", 2048)])
def test_doc_topic_histograms(kind, K):
    from ldagibbssampling_amd.sampler import GibbsSampler
    c = synthetic_lda(num_docs=300, num_types=500, num_topics=min(K, 50), doc_len=None,
                      mean_len=70, min_len=0, max_len=600, seed=K)
    g = GibbsSampler(K, c.num_types, c.doc_off, c.words, 0.1, 0.01, seed=2, sampler=kind)
    g.sweep(2)
    lens = np.diff(c.doc_off)
    L = g.max_doc_length()
    assert L == lens.max()
    dl, td = g.doc_topic_histograms()
    g.doc_topic_histograms(dl, td)                        # accumulates
    nd = _nd(g.z(), c.doc_off, K)
    exp_dl = 2 * np.bincount(lens, minlength=L + 1)
    exp_td = np.zeros((K, L + 1), np.int64)
    for k in range(K):
        v = nd[:, k]
        exp_td[k] = 2 * np.bincount(v[v > 0], minlength=L + 1)
    np.testing.assert_array_equal(dl, exp_dl)
    np.testing.assert_array_equal(td, exp_td)
    with pytest.raises(Exception):
        g.doc_topic_histograms(max_len=L - 1)


@pytest.mark.parametrize("K", [100, 4096])
def test_count_histogram(K):
    from ldagibbssampling_amd.sampler import GibbsSampler
    c = synthetic_lda(num_docs=400, num_types=300, num_topics=20, doc_len=None, mean_len=300,
                      min_len=1, max_len=900, seed=5)
    g = GibbsSampler(K, c.num_types, c.doc_off, c.words, 0.1, 0.01, seed=3,
                     sampler="sparse" if K > 1024 else "dense")
    g.sweep(3)
    nw = g.counts()[0]
    top = int(np.bincount(c.words).max())
    h = g.count_histogram(top)
    v = nw[nw > 0]
    np.testing.assert_array_equal(h, np.bincount(v, minlength=top + 1))
    with pytest.raises(Exception):
        g.count_histogram(int(v.max()) - 1)


def test_count_histogram_large_cells():
    """Cells >= 4096 take the global-atomic bins (small ones go through LDS)."""
    from ldagibbssampling_amd.corpus import Corpus
    from ldagibbssampling_amd.sampler import GibbsSampler
    rng = np.random.default_rng(6)
    D, L = 20, 3000
    words = np.where(rng.random(D * L) < 0.6, 0, rng.integers(1, 40, D * L)).astype(np.int32)
    c = Corpus(np.arange(D + 1, dtype=np.int64) * L, words, 40)
    g = GibbsSampler(2, 40, c.doc_off, c.words, 0.1, 0.01, seed=1)
    g.sweep(2)
    nw = g.counts()[0]
    assert nw.max() >= 4096
    top = int(np.bincount(words).max())
    np.testing.assert_array_equal(g.count_histogram(top), np.bincount(nw[nw > 0], minlength=top + 1))


@pytest.mark.parametrize("K", [20, 300, 2048])
def test_row_stats(K):
    """Token-weighted mean nonzeros per word row (the sparse bytes model)."""
    from ldagibbssampling_amd.sampler import GibbsSampler
    c = synthetic_lda(num_docs=200, num_types=700, num_topics=30, doc_len=None, mean_len=80,
                      min_len=1, max_len=300, seed=K)
    g = GibbsSampler(K, c.num_types, c.doc_off, c.words, 0.1, 0.01, seed=1,
                     sampler="sparse" if K > 1024 else "dense")
    g.sweep(2)
    nw = g.counts()[0].astype(np.float64)
    tot, nnz = nw.sum(1), (nw > 0).sum(1)
    assert abs(g.row_stats() - (tot * nnz).sum() / tot.sum()) < 1e-9


@pytest.mark.parametrize("kind,K", [("dense", 64), ("sparse", 4096)])
def test_device_accumulated_histograms_and_async_ll(kind, K):
    """lda_doc_topic_histograms_accumulate over three sweeps + _take equal the
    sum of the per-sweep histograms; lda_log_likelihood_enqueue/_collect
    equal the blocking lda_log_likelihood_parts; a ticket is collected once."""
    import ctypes as C
    from ldagibbssampling_amd import capi
    from ldagibbssampling_amd.sampler import GibbsSampler
    c = synthetic_lda(num_docs=200, num_types=400, num_topics=30, doc_len=None, mean_len=60,
                      min_len=0, max_len=300, seed=K)
    g = GibbsSampler(K, c.num_types, c.doc_off, c.words, 0.1, 0.01, seed=5, sampler=kind)
    L = g.max_doc_length()
    lib = capi.load()
    dl_sum = np.zeros(L + 1, np.int32)
    td_sum = np.zeros(K * (L + 1), np.int32)
    tickets, exp_ll = [], []
    for _ in range(3):
        g.sweep(1)
        dl, td = g.doc_topic_histograms()
        dl_sum += dl
        td_sum += td.reshape(-1)
        capi.check(lib.lda_doc_topic_histograms_accumulate(g._h, L), "accumulate")
        t = C.c_int64()
        capi.check(lib.lda_log_likelihood_enqueue(g._h, C.byref(t)), "enqueue")
        tickets.append(t.value)
        exp_ll.append(g.log_likelihood_parts())
    dl_acc = np.zeros(L + 1, np.int32)
    td_acc = np.zeros(K * (L + 1), np.int32)
    capi.check(lib.lda_doc_topic_histograms_take(g._h, L, dl_acc, td_acc), "take")
    np.testing.assert_array_equal(dl_acc, dl_sum)
    np.testing.assert_array_equal(td_acc, td_sum)
    capi.check(lib.lda_doc_topic_histograms_take(g._h, L, dl_acc, td_acc), "take")   # zeroed: adds 0
    np.testing.assert_array_equal(dl_acc, dl_sum)
    for t, (ed, ew) in zip(tickets, exp_ll):
        a, b = C.c_double(), C.c_double()
        capi.check(lib.lda_log_likelihood_collect(g._h, t, C.byref(a), C.byref(b)), "collect")
        assert a.value == ed and b.value == ew
    a, b = C.c_double(), C.c_double()
    assert lib.lda_log_likelihood_collect(g._h, tickets[0], C.byref(a), C.byref(b)) == -4


@pytest.mark.parametrize("kind,K", [("dense", 100), ("sparse", 2048)])
def test_hyper_statistics_in_one_call(kind, K):
    """lda_hyper_statistics (one wait) equals _take + lda_count_histogram +
    lda_get_counts' nwsum, each output optional; the accumulated histograms
    are zeroed by it as by _take."""
    import ctypes as C
    from ldagibbssampling_amd import capi
    from ldagibbssampling_amd.sampler import GibbsSampler
    c = synthetic_lda(num_docs=150, num_types=300, num_topics=20, doc_len=None, mean_len=50,
                      min_len=0, max_len=200, seed=K + 1)
    mk = lambda: GibbsSampler(K, c.num_types, c.doc_off, c.words, 0.1, 0.01, seed=9, sampler=kind)
    a, b = mk(), mk()
    L = a.max_doc_length()
    M = int(np.bincount(c.words, minlength=c.num_types).max())
    lib = capi.load()
    for g in (a, b):
        for _ in range(2):
            g.sweep(1)
            capi.check(lib.lda_doc_topic_histograms_accumulate(g._h, L), "accumulate")
    dl, td = np.zeros(L + 1, np.int32), np.zeros(K * (L + 1), np.int32)
    capi.check(lib.lda_doc_topic_histograms_take(a._h, L, dl, td), "take")
    hist = a.count_histogram(M)
    nws = a.counts(with_nd=False)[1]
    dl2, td2 = np.zeros(L + 1, np.int32), np.zeros(K * (L + 1), np.int32)
    hist2, nws2 = np.zeros(M + 1, np.int32), np.zeros(K, np.int32)
    ptr = lambda x: x.ctypes.data_as(C.c_void_p)
    capi.check(lib.lda_hyper_statistics(b._h, L, ptr(dl2), ptr(td2), M, ptr(hist2), ptr(nws2)), "hyper")
    np.testing.assert_array_equal(dl2, dl)
    np.testing.assert_array_equal(td2, td)
    np.testing.assert_array_equal(hist2, hist)
    np.testing.assert_array_equal(nws2, nws[:K])
    # zeroed like _take; outputs optional
    capi.check(lib.lda_hyper_statistics(b._h, L, ptr(dl2), ptr(td2), 0, None, None), "hyper")
    np.testing.assert_array_equal(dl2, dl)
    capi.check(lib.lda_hyper_statistics(b._h, L, None, None, M, None, ptr(nws2)), "hyper")
    np.testing.assert_array_equal(nws2, nws[:K])
    assert lib.lda_hyper_statistics(b._h, L, ptr(dl2), None, 0, None, None) == -1
