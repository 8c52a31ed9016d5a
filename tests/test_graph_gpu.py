"""lda_sweep's graph-launched plain sweeps (k x (sampler, apply) captured once,
the sweep counter read from device memory) against cpu_exact and against the
same sweeps launched one by one (LDA_GRAPHS=0).  Bar: bit-exact z and counts,
across the events that change what a graph captured (beta, exchange parts),
batches longer than one graph (16 sweeps), the warm start and the recount."""
import numpy as np
import pytest

from ldagibbssampling_amd.corpus import synthetic_changelists

pytestmark = pytest.mark.gpu


def _state(s):
    nw, ns, _, _ = s.counts(with_nd=False)
    return s.z(), nw, ns


def _same(a, b):
    for x, y in zip(_state(a), _state(b)):
        np.testing.assert_array_equal(x, y)


def _make(corpus, K, seed, graphs, monkeypatch):
    from ldagibbssampling_amd.sampler import GibbsSampler
    monkeypatch.setenv("LDA_GRAPHS", "1" if graphs else "0")
    return GibbsSampler(K, corpus.num_types, corpus.doc_off, corpus.words, np.full(K, 0.2), 0.01, seed=seed,
                        tokens_per_range=256)


@pytest.mark.parametrize("K", [20, 100, 500])
def test_graph_sweeps_bit_exact(oracle, monkeypatch, K):
    c = synthetic_changelists(num_docs=600, num_types=900, seed=K)
    g = _make(c, K, 11, True, monkeypatch)
    n = _make(c, K, 11, False, monkeypatch)
    o = oracle.ExactSampler(K, c.num_types, c.doc_off, c.words, np.full(K, 0.2), 0.01, 11)
    for s in (g, n, o):
        s.sweep(1)
    _same(g, o)
    # 7, then 37 (two full graphs + 5), with a beta change between batches
    for s in (g, n, o):
        s.sweep(7)
    _same(g, o)
    for s in (g, n, o):
        s.set_alpha_beta(np.linspace(0.05, 0.5, K), 0.02)
        s.sweep(37)
    _same(g, o)
    _same(g, n)
    lg, lo = g.log_likelihood(), o.log_likelihood()
    assert abs(lg - lo) <= 1e-9 * abs(lo)


def test_graph_sweeps_across_parts_warm_start_and_recount(oracle, monkeypatch):
    """The exchange parts changed and restored (the graphs captured the old
    ranges), a warm start whose first sweeps are sequential parts, and the
    recount's sweeps: lda_sweep runs those one by one and the plain ones after
    them as graphs, with the same result as the one-by-one path."""
    c = synthetic_changelists(num_docs=800, num_types=1200, seed=3)
    K = 64
    g = _make(c, K, 5, True, monkeypatch)
    n = _make(c, K, 5, False, monkeypatch)
    for s in (g, n):
        s.set_warm_start(3, 6)
        s.set_count_update("recount", 0)
    g.sweep(9)
    n.sweep(9)
    _same(g, n)
    for s in (g, n):
        s.set_count_update("delta", 0)
        s.sweep(20)
    _same(g, n)
    for s in (g, n):
        s.set_exchange_parts(2)
        s.sweep(3)
        s.set_exchange_parts(1)
        s.sweep(21)
    _same(g, n)
    o = oracle.ExactSampler(K, c.num_types, c.doc_off, c.words, np.full(K, 0.2), 0.01, 5)
    o.set_warm_start(3, 6, 0, c.num_tokens)
    o.sweep(9 + 20 + 3 + 21)
    _same(g, o)


def test_graph_sweeps_follow_sweep_counter_and_stream(monkeypatch):
    """The sweep counter set between graph launches (lda_set_sweep, as a
    resumed checkpoint does) and a change of stream (lda_set_stream: the
    graphs are rebuilt for it) give the one-by-one path's state."""
    import torch
    c = synthetic_changelists(num_docs=500, num_types=800, seed=9)
    K = 48
    g = _make(c, K, 21, True, monkeypatch)
    n = _make(c, K, 21, False, monkeypatch)
    for s in (g, n):
        s.sweep(5)
        s.sweep_index = 2            # rewind the Philox sweep word
        s.sweep(7)
    assert g.sweep_index == n.sweep_index == 9
    _same(g, n)
    st = torch.cuda.Stream()
    for s in (g, n):
        s.set_stream(st.cuda_stream)
        s.sweep(19)
        s.synchronize()
    _same(g, n)
    for s in (g, n):
        s.set_stream(None)
        s.sweep(3)
    _same(g, n)


def test_graph_sweeps_stream_switch_without_synchronize(monkeypatch):
    """lda_set_stream between two lda_sweep calls with graph sweeps
    still in flight on the old stream.  The graphs captured for the old stream
    are destroyed only after their last launch has finished, and the new
    stream is ordered after the old one, so no caller synchronize is needed."""
    import torch
    c = synthetic_changelists(num_docs=500, num_types=800, seed=19)
    K = 100
    g = _make(c, K, 31, True, monkeypatch)
    n = _make(c, K, 31, False, monkeypatch)
    streams = [torch.cuda.Stream() for _ in range(3)]
    for s in (g, n):
        for i in range(6):
            s.set_stream(streams[i % 3].cuda_stream)     # no synchronize in between
            s.sweep(17)
        s.set_stream(None)
        s.sweep(2)
        s.synchronize()
    _same(g, n)
