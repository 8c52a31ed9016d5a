#!/usr/bin/env python3
"""cpu_mallet's held-out perplexity per seed (tests/test_perplexity.py's
corpus, split and estimator), on the CPU: the Mallet 2.0.7 restatement trains
1000 sweeps with 4 threads (setNumThreads(4), src/cmu_ron/TrainAndPredict.java:164),
then its z is loaded into cpu_exact and scored with the same document-
completion estimator the GPU leg uses (the inference draw of the default
quarter-wave kernel, which cpu_exact restates bit for bit).

  python tools/ppl_mallet_seeds.py K first_seed last_seed > out.json

K > 1024 (round 6): scored with the large-K sparse sampler's inference draw
(exact_draw_big), the kernel the GPU leg runs there.

The output is the committed fixture tests/golden/mallet_ppl_k{K}.json that
tests/test_perplexity.py compares the GPU sampler against (the GPU test does
not retrain cpu_mallet: 96 seeds take ~16 CPU-minutes).
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from oracle import oracle  # noqa: E402  (the checker)
from test_perplexity import ALPHA_SUM, BETA, LARGE_K, _corpus_split, score_state  # noqa: E402


def main():
    K, s0, s1 = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
    c, train, held_obs, held_sc = _corpus_split(K)
    out = {"K": K, "alpha_sum": ALPHA_SUM, "beta": BETA, "sweeps": 1000, "threads": 4,
           "estimator": "document completion, lda_infer(100, 10, 10, seed 7), " + (
               "large-K sparse draw (exact_draw_big)" if K > LARGE_K else
               "quarter-wave draw" if K <= 128 else "full-wave dense draw"),
           "seeds": [], "perplexity": []}
    for seed in range(s0, s1 + 1):
        t = time.time()
        m = oracle.MalletModel(K, ALPHA_SUM, BETA, c.num_types, train.doc_off, train.words,
                               seed=seed, num_threads=4)
        m.estimate(1000)
        ppl = score_state(oracle, K, c.num_types, train, m.z(), held_obs, held_sc)
        out["seeds"].append(seed)
        out["perplexity"].append(ppl)
        print(f"K={K} seed {seed}: {ppl:.4f} ({time.time() - t:.1f} s)", file=sys.stderr, flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
