"""Split sweeps (lda_set_exchange_parts / lda_sample_part): the
exchange of part i overlaps the sampling of part i+1.  A sweep cut into parts
is the same sweep: z and counts bit-exact against cpu_exact (which never
splits), for the dense, sparse and large-K sparse samplers, and the ABI's
ordering rules hold."""
import numpy as np
import pytest

from ldagibbssampling_amd.capi import LdaError
from ldagibbssampling_amd.corpus import synthetic_lda

pytestmark = pytest.mark.gpu


def _corpus(K, D=150, V=800, seed=5):
    return synthetic_lda(num_docs=D, num_types=V, num_topics=min(K, 100), doc_len=None,
                         mean_len=60, min_len=0, max_len=400, seed=seed)


@pytest.mark.parametrize("kind,K", [("dense", 20), ("dense", 512), ("dense", 1024),
                                    ("sparse", 300), ("sparse", 2048), ("sparse", 4096)])
@pytest.mark.parametrize("parts", [2, 3, 4])
def test_split_sweeps_bit_exact(oracle, kind, K, parts):
    from ldagibbssampling_amd.sampler import GibbsSampler
    c = _corpus(K, seed=K + parts)
    alpha = np.full(K, 50.0 / K)
    g = GibbsSampler(K, c.num_types, c.doc_off, c.words, alpha, 0.01, seed=77 + K,
                     tokens_per_range=200, sampler=kind)
    g.set_exchange_parts(parts, reserve_cus=8)
    assert g.exchange_parts == parts
    o = oracle.ExactSampler(K, c.num_types, c.doc_off, c.words, alpha, 0.01, 77 + K, kind=kind)
    g.sweep(0)
    o.apply()
    for sweep in range(3):
        # parts by hand (the trainer's order), then lda_sample (every part)
        if sweep == 1:
            g.sample()
        else:
            for i in range(parts):
                g.sample_part(i)
        g.apply()
        o.sample()
        o.apply()
        np.testing.assert_array_equal(g.z(), o.z())
    gnw, gns, _, _ = g.counts()
    onw, ons, _, _ = o.counts()
    np.testing.assert_array_equal(gnw, onw)
    np.testing.assert_array_equal(gns, ons)
    assert g.sweep_index == o.sweep_index == 3
    # back to one part: the delta of a dropped part is folded, not lost
    g.set_exchange_parts(1)
    g.sweep(1)
    o.sweep(1)
    np.testing.assert_array_equal(g.z(), o.z())


def test_split_sweep_ordering_rules(oracle):
    from ldagibbssampling_amd.sampler import GibbsSampler
    c = _corpus(64)
    g = GibbsSampler(64, c.num_types, c.doc_off, c.words, 0.1, 0.01, seed=3)
    g.set_exchange_parts(3)
    g.sweep(0)
    with pytest.raises(LdaError):
        g.sample_part(1)                  # parts in order
    g.sample_part(0)
    with pytest.raises(LdaError):
        g.apply()                         # not before the last part
    with pytest.raises(LdaError):
        g.sample()                        # not inside a split sweep
    with pytest.raises(LdaError):
        g.set_exchange_parts(2)           # nor re-cut it
    g.sample_part(1)
    g.sample_part(2)
    with pytest.raises(LdaError):
        g.sample_part(0)                  # the delta is pending
    g.apply()
    with pytest.raises(LdaError):
        g.set_exchange_parts(5)
    # every part's buffer is a distinct device buffer of the same size
    ptrs = {g.delta_buffer(i) for i in range(3)}
    assert len(ptrs) == 3 and len({n for _, n in ptrs}) == 1
    o = oracle.ExactSampler(64, c.num_types, c.doc_off, c.words, 0.1, 0.01, 3)
    o.sweep(1)
    np.testing.assert_array_equal(g.z(), o.z())
