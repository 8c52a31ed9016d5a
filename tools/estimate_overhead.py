#!/usr/bin/env python3
"""Where the time of ParallelTopicModel.estimate() goes at the reference's own
scale (C1 changelist corpus, src/cmu_ron's K = 500, Sigma alpha 100, beta 1):
1000 iterations with the LL/token log and the alpha/beta optimisation each
switched on or off, and the sampler kernels' own time (lda_sample_times).
Prints one JSON line.   PYTHONPATH=$PWD python tools/estimate_overhead.py"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(c, K, asum, beta, iters, ll, opt):
    from ldagibbssampling_amd import topic_model as tm
    m = tm.ParallelTopicModel(K, asum, beta)
    m.addInstances(tm.InstanceList.fromCorpus(c))
    m.setRandomSeed(1)
    m.setTopicDisplay(0, 0)
    m.setOptimizeInterval(20 if opt else 0)
    m.setNumThreads(4)
    if hasattr(m, "setPrintLogLikelihood"):
        m.setPrintLogLikelihood(bool(ll))
    m.setNumIterations(10)
    m.estimate()                         # shards built, kernels warm
    m.setNumIterations(iters)
    t = time.perf_counter()
    m.estimate()
    return time.perf_counter() - t


def main():
    import torch  # noqa: F401
    from ldagibbssampling_amd.corpus import synthetic_changelists
    c = synthetic_changelists()
    K, asum, beta, iters = 500, 100.0, 1.0, 1000
    out = {"corpus": f"C1 changelists: {c.num_docs} docs, {c.num_tokens} tokens", "K": K,
           "iterations": iters}
    for ll in (0, 1):
        for opt in (0, 1):
            s = run(c, K, asum, beta, iters, ll, opt)
            out[f"ll{ll}_opt{opt}_us_per_iteration"] = 1e6 * s / iters
    print(json.dumps(out))


if __name__ == "__main__":
    main()
