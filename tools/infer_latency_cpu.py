#!/usr/bin/env python3
"""cpu_mallet's TopicInferencer (oracle/, the Mallet 2.0.7 restatement) per
one-document call at the reference's scale: C1 changelist corpus, K = 500
(src/cmu_ron), getSampledDistribution(inst, 100, 10, 10)
(src/cmu_ron/TrainAndPredict.java:144).  Compare with tools/infer_latency.py
(the GPU's lda_infer).   python tools/infer_latency_cpu.py"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import oracle as O  # noqa: E402  (the CPU baseline)
from ldagibbssampling_amd.corpus import synthetic_changelists  # noqa: E402


def main():
    c = synthetic_changelists(num_docs=2000, num_types=5000, seed=20261015)
    K = 500
    m = O.MalletModel(K, 100.0, 1.0, c.num_types, c.doc_off, c.words, seed=1, num_threads=4)
    m.estimate(200)
    held = synthetic_changelists(num_docs=200, num_types=5000, seed=7)
    lat = []
    for d in range(held.num_docs):
        off = np.array([0, held.doc_off[d + 1] - held.doc_off[d]], np.int64)
        w = held.words[held.doc_off[d]:held.doc_off[d + 1]]
        t = time.perf_counter()
        m.infer(off, w, n_iter=100, burn_in=10, thin=10, seed=d)
        lat.append(time.perf_counter() - t)
    lat = np.array(lat) * 1e3
    print(json.dumps({"cpu_mallet_one_doc_ms": {"mean": float(lat.mean()), "median": float(np.median(lat)),
                                                "p90": float(np.percentile(lat, 90))},
                      "workload": "C1 changelist corpus, K=500, 200 training sweeps, 200 held-out "
                                  "one-document calls, getSampledDistribution(100, 10, 10)"}))


if __name__ == "__main__":
    main()
