#!/usr/bin/env python3
"""cpu_mallet's held-out perplexity per seed at the reference's OWN training
settings (tests/test_perplexity.py::test_heldout_perplexity_reference_settings):

  src/cmu/TrainAndPredict.java:259-263      K=100, alphaSum=10,  beta=0.001
  src/cmu_ron/TrainAndPredict.java:160-165  K=500, alphaSum=100, beta=1

each with setOptimizeInterval(20), Mallet's default burn-in 200,
setNumThreads(4) and 1000 sweeps.  The Mallet 2.0.7 restatement trains on the
CPU; its final z is loaded into cpu_exact with ITS learned alpha/beta and
scored with the document-completion estimator of the GPU leg (the inference
draw of the kernel the library picks at that K: quarter-wave for K <= 128,
full-wave k_sample<C> above), exactly as the test scores the GPU model.

  python tools/ppl_mallet_ref_seeds.py K alpha_sum beta first_seed last_seed [jobs] > out.json

The output is the committed fixture tests/golden/mallet_ppl_ref_k{K}.json.
Seeds run `jobs` at a time (default 2: each model uses 4 threads).
"""
import json
import os
import sys
import time
from concurrent.futures import ProcessPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

SWEEPS, OPT_INTERVAL, BURNIN, THREADS = 1000, 20, 200, 4


def one_seed(args):
    K, alpha_sum, beta, seed = args
    from oracle import oracle  # noqa: E402  (the checker)
    from test_perplexity import _corpus_split, score_state  # noqa: E402
    t = time.time()
    c, train, held_obs, held_sc = _corpus_split(K)
    m = oracle.MalletModel(K, alpha_sum, beta, c.num_types, train.doc_off, train.words,
                           seed=seed, num_threads=THREADS)
    m.set_optimize(OPT_INTERVAL, burnin=BURNIN)
    m.estimate(SWEEPS)
    a_m, b_m = m.hyper()
    ppl = score_state(oracle, K, c.num_types, train, m.z(), held_obs, held_sc,
                      alpha=a_m, beta=b_m)
    print(f"K={K} seed {seed}: {ppl:.4f} alphaSum {a_m.sum():.5g} beta {b_m:.5g} "
          f"({time.time() - t:.1f} s)", file=sys.stderr, flush=True)
    return seed, ppl, float(a_m.sum()), float(b_m)


def main():
    K, alpha_sum, beta = int(sys.argv[1]), float(sys.argv[2]), float(sys.argv[3])
    s0, s1 = int(sys.argv[4]), int(sys.argv[5])
    jobs = int(sys.argv[6]) if len(sys.argv) > 6 else 2
    out = {"K": K, "alpha_sum": alpha_sum, "beta": beta, "sweeps": SWEEPS, "threads": THREADS,
           "optimize_interval": OPT_INTERVAL, "burnin": BURNIN,
           "estimator": "document completion, inference(100, 10, 10, seed 7) with the learned "
                        "alpha/beta, the draw of the library's kernel at this K",
           "seeds": [], "perplexity": [], "alpha_sum_learned": [], "beta_learned": []}
    with ProcessPoolExecutor(jobs) as ex:
        for seed, ppl, asum, b in ex.map(one_seed, [(K, alpha_sum, beta, s)
                                                   for s in range(s0, s1 + 1)]):
            out["seeds"].append(seed)
            out["perplexity"].append(ppl)
            out["alpha_sum_learned"].append(asum)
            out["beta_learned"].append(b)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
