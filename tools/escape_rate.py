#!/usr/bin/env python3
"""Escapes per rank of the compact exchange at N ranks' biases, with 2 and 4
cells per packed word (lda_set_exchange_cells), on one rank's shard of a
BASELINE workload: after sweep s the shard's delta buffer is
packed as a rank of an N-rank group would pack it (lda_exchange_pack with
world = N; nothing is all-reduced or unpacked, the sweep's apply then folds
the delta as usual) and its escape count read, with the pack's time.
    python tools/escape_rate.py [c5|c4shard] [N] > out.jsonl"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from ldagibbssampling_amd.corpus import synthetic_lda_torch  # noqa: E402
from ldagibbssampling_amd.sampler import GibbsSampler  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c5"
world = int(sys.argv[2]) if len(sys.argv) > 2 else 8
docs, V, K, kind = {"c5": (1_250_000, 262_144, 4096, "sparse"),
                    "c4shard": (1_250_000, 100_000, 512, "dense")}[cfg]
c = synthetic_lda_torch(docs, V, K, doc_len=200, seed=20261015, doc_seed=20261015, device="cuda:0")
g = GibbsSampler(K, V, c.doc_off, c.words, np.full(K, 0.1 * K / K), 0.01, seed=1, sampler=kind)
g.set_count_update("delta")           # the buffer holds the sweep's changes (what ranks exchange)
g.sweep(0)
marks = {1, 2, 5, 10, 20, 30}
for s in range(1, max(marks) + 1):
    g.sample()
    if s in marks:
        rec = {"workload": cfg, "sweep": s, "world": world, "tokens": int(g.N)}
        for cells in (2, 4):
            g.set_exchange_cells(cells)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            pk, es = g.exchange_pack(0, world, g.N)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            m = int(es[0])
            rec[f"cells{cells}"] = {"escapes": m, "packed_bytes": 4 * int(pk.numel()),
                                    "gathered_bytes_all_ranks": 4 * world * (1 + 3 * m) if m else 0,
                                    "pack_ms": 1e3 * dt}
        print(json.dumps(rec), flush=True)
    g.apply()
g.close()
