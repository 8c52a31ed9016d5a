"""Sweep time of small corpora (the reference's own scale) against the work
granule: BASELINE C1 (changelist-shaped, K=20), the perplexity-test corpus,
and the reference's training settings (K=100 / K=500) on the C1 corpus.
Usage: python tools/small_corpus.py [tpr ...]   (0 = the library default)"""
import sys, time
import numpy as np
sys.path.insert(0, '.')
from ldagibbssampling_amd.corpus import synthetic_changelists, synthetic_lda
from ldagibbssampling_amd.sampler import GibbsSampler

tprs = [int(x) for x in sys.argv[1:]] or [0]
cases = [
    ("C1 changelists K=20", synthetic_changelists(), 20, 10.0, 0.01, 100),
    ("C1 changelists K=100 (src/cmu)", synthetic_changelists(), 100, 10.0, 0.001, 200),
    ("C1 changelists K=500 (src/cmu_ron)", synthetic_changelists(), 500, 100.0, 1.0, 200),
    ("perplexity corpus K=100", synthetic_lda(num_docs=2200, num_types=3000, num_topics=100, doc_len=None,
                                              mean_len=80, min_len=10, max_len=300, seed=20261015, k_true=50),
     100, 10.0, 0.01, 200),
]
for name, c, K, asum, beta, sweeps in cases:
    for tpr in tprs:
        g = GibbsSampler(K, c.num_types, c.doc_off, c.words, np.full(K, asum / K), beta, seed=1,
                         tokens_per_range=tpr)
        g.sweep(5)
        g.synchronize()
        t = time.perf_counter()
        g.sweep(sweeps)
        g.synchronize()
        dt = (time.perf_counter() - t) / sweeps
        print(f"{name}: N={c.num_tokens} tpr={tpr}: {dt*1e6:.1f} us/sweep, {c.num_tokens/dt:.3g} tok/s", flush=True)
