"""Token-weighted row statistics of the C4 bench corpus (design study for
narrower row encodings): cells >= 255 per row read, rows with none."""
import json
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from ldagibbssampling_amd.corpus import synthetic_lda_torch
from ldagibbssampling_amd.sampler import GibbsSampler

K, V = 512, 100_000
c = synthetic_lda_torch(1_250_000, V, K, doc_len=200, seed=20261015, device="cuda:0")
g = GibbsSampler(K, V, c.doc_off, c.words, np.full(K, 0.1), 0.01, seed=1)
tot = np.bincount(c.words, minlength=V).astype(np.float64)
w = tot / tot.sum()
out = {}
done = 0
for target in (5, 30):
    g.sweep(target - done)
    done = target
    nw = g.counts()[0]
    big = (nw >= 255).sum(1)
    huge = (nw > 65535).sum(1)
    nnz = (nw > 0).sum(1)
    sectors = np.zeros(V)          # distinct 64-byte (32-cell) sectors holding a cell >= 255
    for s in range(0, K, 32):
        sectors += (nw[:, s:s + 32] >= 255).any(1)
    out[target] = dict(escapes_per_token=float((w * big).sum()),
                       escape_sectors_per_token=float((w * sectors).sum()),
                       frac_tokens_no_escape=float(w[big == 0].sum()),
                       nnz_per_token=float((w * nnz).sum()),
                       wide_rows_token_frac=float(w[huge > 0].sum()),
                       est_bytes_u8_escape=float(512 + 64 * (w * sectors).sum()))
    print(target, json.dumps(out[target]), flush=True)
