"""Per-path draw counts of the large-K sampler (a build with -DSB_X_COUNT,
loaded through LDA_MI355X_LIB) on the C5 workload shape: after `burnin`
sweeps, one traced sampling pass counts tokens, A draws in the alpha part,
A draws in the document part, own-entry hits and re-draws.
    LDA_MI355X_LIB=variants/xcount/liblda_mi355x.so python tools/count_paths.py DOCS BURNIN..."""
import ctypes as C
import json
import sys

import numpy as np

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from ldagibbssampling_amd.corpus import synthetic_lda_torch  # noqa: E402
from ldagibbssampling_amd.sampler import GibbsSampler  # noqa: E402

docs = int(sys.argv[1])
marks = [int(x) for x in sys.argv[2:]] or [0, 30]
K, V = 4096, 262_144
c = synthetic_lda_torch(docs, V, K, doc_len=200, seed=20261015, doc_seed=20261015, device="cuda:0")
g = GibbsSampler(K, V, c.doc_off, c.words, np.full(K, 0.1), 0.01, seed=1, sampler="sparse")
L = g._L
L.lda_debug_sample_trace.restype = C.c_int32
L.lda_debug_sample_trace.argtypes = [C.c_void_p, C.c_void_p]
g.sweep(0)
done = 0
out = []
for m in marks:
    g.sweep(m - done)
    done = m
    tr = np.zeros(8 * g.N, dtype=np.float32)
    st = L.lda_debug_sample_trace(g._h, tr.ctypes.data)
    assert st == 0, st
    cnt = tr[:8].view(np.uint32)[:5].astype(np.int64)
    g.apply()
    done += 1
    n = max(int(cnt[0]), 1)
    rec = {"sweep": m, "tokens": int(cnt[0]), "a_alpha": int(cnt[1]) / n, "a_doc": int(cnt[2]) / n,
           "own_hit": int(cnt[3]) / n, "redraw": int(cnt[4]) / n}
    print(json.dumps(rec), flush=True)
    out.append(rec)
g.close()
