#!/usr/bin/env python3
"""Latency of one-document inference (the reference's predict loop calls
TopicInferencer.getSampledDistribution(inst, 100, 10, 10) once per test
instance: src/cmu_ron/TrainAndPredict.java:144, src/cmu/TrainAndPredict.java:114)
through lda_infer, after training on (a) the C1 changelist corpus at
src/cmu_ron's K = 500 and (b) a C4-vocabulary corpus (V = 100k, K = 512).
Prints one JSON line: ms per call (median of 50) for 1-document and
16-document calls.   PYTHONPATH=$PWD python tools/infer_latency.py"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def bench(g, held, reps=50):
    out = {}
    for nd in (1, 16):
        off = held.doc_off[:nd + 1] - held.doc_off[0]
        words = held.words[held.doc_off[0]:held.doc_off[nd]]
        g.infer(off, words, 100, 10, 10, seed=1)            # warm
        ts = []
        for r in range(reps):
            t0 = time.perf_counter()
            g.infer(off, words, 100, 10, 10, seed=r)
            ts.append(time.perf_counter() - t0)
        out[f"{nd}_docs_ms"] = 1e3 * float(np.median(ts))
    return out


def main():
    import torch  # noqa: F401
    from ldagibbssampling_amd.corpus import synthetic_changelists, synthetic_lda_torch
    from ldagibbssampling_amd.sampler import GibbsSampler
    res = {}
    c = synthetic_changelists(num_docs=2000, num_types=5000, seed=3)
    train, held = c.subset(range(0, 1800)), c.subset(range(1800, 2000))
    g = GibbsSampler(500, c.num_types, train.doc_off, train.words, 100.0 / 500, 1.0, seed=2)
    g.sweep(50)
    res["c1_K500"] = bench(g, held)
    g.close()
    c4 = synthetic_lda_torch(20000, 100_000, 512, doc_len=200, seed=20261015, device="cuda:0")
    train, held = c4.subset(range(0, 19000)), c4.subset(range(19000, 20000))
    g = GibbsSampler(512, 100_000, train.doc_off, train.words, 0.1, 0.01, seed=2)
    g.sweep(10)
    res["c4vocab_K512"] = bench(g, held)
    g.close()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
