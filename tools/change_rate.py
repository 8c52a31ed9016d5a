#!/usr/bin/env python3
"""Fraction of tokens whose topic changes in each sweep (the delta path's
atomics are proportional to it; the recount's cost is not), on a bench
workload drawn as bench.py draws it.

  python tools/change_rate.py CONFIG [SWEEPS] [DOCS]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402


def main():
    import torch
    import bench
    from ldagibbssampling_amd.corpus import synthetic_lda_torch
    from ldagibbssampling_amd.sampler import GibbsSampler
    name = sys.argv[1]
    sweeps = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    cfg = bench.CONFIGS[name]
    docs = int(sys.argv[3]) if len(sys.argv) > 3 else cfg["docs"]
    K, V, L = cfg["K"], cfg["V"], cfg["doc_len"]
    c = synthetic_lda_torch(docs, V, K, doc_len=L, seed=20261015, doc_seed=20261015, device="cuda:0")
    g = GibbsSampler(K, V, c.doc_off, c.words, np.full(K, 0.1), 0.01, seed=1)
    g.sweep(0)
    z0 = g.z()
    rates = []
    for s in range(sweeps):
        g.sweep(1)
        z1 = g.z()
        rates.append(float((z1 != z0).mean()))
        z0 = z1
    print(json.dumps({"config": name, "docs": docs, "K": K, "tokens": int(c.num_tokens),
                      "changed_fraction_per_sweep": rates}))


if __name__ == "__main__":
    main()
