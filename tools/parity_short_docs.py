#!/usr/bin/env python3
"""Large-K parity on documents of at most 250 tokens (measurement variants
whose per-wave document counts are bytes, SB_ND8, cannot hold the longer
documents of tests/test_parity_gpu.py): the library at LDA_MI355X_LIB against
cpu_exact for 3 sweeps and frozen-model inference, K = 1500 and 4096.
    LDA_MI355X_LIB=variants/nd8a/liblda_mi355x.so python tools/parity_short_docs.py"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from ldagibbssampling_amd.corpus import Corpus  # noqa: E402
from ldagibbssampling_amd.sampler import GibbsSampler  # noqa: E402
from oracle import oracle as O  # noqa: E402  (the checker)


def corpus(D, V, seed):
    rng = np.random.default_rng(seed)
    lens = rng.integers(0, 251, size=D)
    lens[::17] = 0
    off = np.zeros(D + 1, dtype=np.int64)
    np.cumsum(lens, out=off[1:])
    p = 1.0 / np.arange(1, V + 1) ** 1.05
    p /= p.sum()
    return Corpus(off, rng.choice(V, size=int(off[-1]), p=p).astype(np.int32), V)


for K in (1500, 4096):
    c = corpus(400, 800, K)
    train, held = c.subset(range(0, 360)), c.subset(range(360, 400))
    a = np.full(K, 30.0 / K)
    g = GibbsSampler(K, c.num_types, train.doc_off, train.words, a, 0.01, seed=K, sampler="sparse",
                     tokens_per_range=300)
    o = O.ExactSampler(K, c.num_types, train.doc_off, train.words, a, 0.01, K, kind="sparse")
    for n in (1, 2):
        g.sweep(n)
        o.sweep(n)
        assert np.array_equal(g.z(), o.z()), (K, "z")
        gn, gs, _, _ = g.counts()
        on, os_, _, _ = o.counts()
        assert np.array_equal(gn, on) and np.array_equal(gs, os_), (K, "counts")
    tg = g.infer(held.doc_off, held.words, n_iter=6, burn_in=2, thin=2, seed=8)
    to = o.infer(held.doc_off, held.words, n_iter=6, burn_in=2, thin=2, seed=8)
    assert np.abs(tg - to).max() <= 1e-12, (K, "infer")
    print(f"K={K}: {train.num_tokens} tokens x 3 sweeps + inference bit-exact", flush=True)
    g.close()
print("parity_short_docs ok")
