"""No C++ exception crosses the C ABI: a failed host
allocation inside an entry point comes back as LDA_ERR_OUT_OF_MEMORY with a
message, and the library keeps working afterwards.  The allocation failure is
forced by the test hook lda_debug_fail_host_alloc(n) (the n-th caller-sized
host buffer on this thread throws std::bad_alloc)."""
import ctypes as C

import numpy as np
import pytest

from ldagibbssampling_amd import capi


def test_host_only_entry_reports_oom():
    L = capi.load()
    K, max_len = 4, 6
    params = np.full(K, 0.5)
    obs = np.zeros(K * (max_len + 1), dtype=np.int32)
    obs[1::max_len + 1] = 3
    lens = np.zeros(max_len + 1, dtype=np.int32)
    lens[2] = 5
    out = C.c_double()
    L.lda_debug_fail_host_alloc(1)
    st = L.lda_learn_parameters(params, K, obs, lens, max_len, 1.001, 1.0, 1, C.byref(out))
    assert st == -3, st                                   # LDA_ERR_OUT_OF_MEMORY, not an abort
    assert b"bad_alloc" in L.lda_last_error()
    st = L.lda_learn_parameters(params, K, obs, lens, max_len, 1.001, 1.0, 1, C.byref(out))
    assert st == 0 and out.value > 0                      # the hook fired once


@pytest.mark.gpu
def test_mallet_packed_reports_oom():
    from ldagibbssampling_amd.corpus import synthetic_lda
    from ldagibbssampling_amd.sampler import GibbsSampler
    c = synthetic_lda(num_docs=50, num_types=300, num_topics=20, doc_len=None, mean_len=30,
                      min_len=1, max_len=80, seed=2)
    g = GibbsSampler(20, c.num_types, c.doc_off, c.words, 0.5, 0.01, seed=1)
    g.sweep(2)
    L = capi.load()
    L.lda_debug_fail_host_alloc(1)
    with pytest.raises(capi.LdaError) as e:
        g.mallet_packed()
    assert e.value.status == -3
    rows, row_off, bits = g.mallet_packed()               # works again
    assert row_off[-1] == len(rows)
