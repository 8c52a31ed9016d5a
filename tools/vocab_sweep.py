"""Dense sampler rate at K = 512 against the vocabulary size (C4 documents,
1.25M x 200 tokens): with V small the 16-bit table (V KiB) sits in L2, so the
rate at small V is the kernel's compute ceiling and the drop towards
V = 100k is what the row gather costs.  Prints one line per V."""
import sys
import time

import numpy as np
import torch

from ldagibbssampling_amd.corpus import synthetic_lda_torch
from ldagibbssampling_amd.sampler import GibbsSampler

K = 512
docs = int(sys.argv[1]) if len(sys.argv) > 1 else 1_250_000
for V in (2000, 8000, 30000, 100000):
    c = synthetic_lda_torch(docs, V, K, doc_len=200, seed=20261015, device="cuda:0")
    g = GibbsSampler(K, V, c.doc_off, c.words, np.full(K, 0.1), 0.01, seed=1, sampler="dense")
    g.sweep(3)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    g.sweep(10)
    g.synchronize()
    dt = time.perf_counter() - t0
    ks = g.sample_times(10)
    print(f"V={V} table={V * K * 2 / 1e6:.1f} MB  {c.num_tokens * 10 / dt / 1e9:.3f} G tok/s  "
          f"kernel {np.mean(ks):.3f} ms", flush=True)
    g.close()
    del c
