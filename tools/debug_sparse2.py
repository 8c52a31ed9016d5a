import sys
import numpy as np
sys.path.insert(0, ".")
sys.path.insert(0, "tests")
from oracle import oracle as O
from ldagibbssampling_amd.sampler import GibbsSampler
from test_parity_gpu import _ragged_corpus

K = 20
c = _ragged_corpus(D=120, V=700, seed=K)
alpha = np.full(K, 0.1)
seed = 1234 + K
o = O.ExactSampler(K, c.num_types, c.doc_off, c.words, alpha, 0.01, seed, kind="sparse")
o.apply(); z0 = o.z().copy(); o.sweep(1); zo_ = o.z()
for tpr in (300, 256, 1000, 0, 100000):
    g = GibbsSampler(K, c.num_types, c.doc_off, c.words, alpha, 0.01, seed=seed, tokens_per_range=tpr, sampler="sparse")
    g.sweep(1)
    zg = g.z()
    bad = np.nonzero(zg != zo_)[0]
    print("tpr", tpr, "mismatches", len(bad), bad[:12])
    if tpr == 300:
        for d in (11, 12, 103, 104, 105):
            a, b = c.doc_off[d], c.doc_off[d + 1]
            print("doc", d, "old", z0[a:b].tolist(), "\n   orc", zo_[a:b].tolist(), "\n   gpu", zg[a:b].tolist(), "\n   words", c.words[a:b].tolist())
