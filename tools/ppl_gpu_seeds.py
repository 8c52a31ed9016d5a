#!/usr/bin/env python3
"""Held-out perplexity per seed on the GPU for the dense kernels that can
serve K <= 128 (LDA_DENSE_HALF: 2 = quarter-wave, the default; 0 = full-wave
k_sample<C>), with tests/test_perplexity.py's corpus, split and estimator.

  python tools/ppl_gpu_seeds.py K first_seed last_seed [kernels] [warm] > out.json

kernels: comma list of LDA_DENSE_HALF values (default "2,0"); warm: "P,S"
for lda_set_warm_start(P, S) (default "1,0": off).
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402

from oracle import oracle  # noqa: E402  (the checker: doc_completion_loglik)
from test_perplexity import ALPHA_SUM, BETA, _corpus_split, _perplexity  # noqa: E402


def main():
    from ldagibbssampling_amd.sampler import GibbsSampler
    K, s0, s1 = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
    kernels = (sys.argv[4] if len(sys.argv) > 4 else "2,0").split(",")
    warm = [int(x) for x in (sys.argv[5] if len(sys.argv) > 5 else "1,0").split(",")]
    c, train, held_obs, held_sc = _corpus_split(K)
    alpha = np.full(K, ALPHA_SUM / K)
    out = {"K": K, "alpha_sum": ALPHA_SUM, "beta": BETA, "sweeps": 1000,
           "estimator": "document completion, lda_infer(100, 10, 10, seed 7)",
           "seeds": list(range(s0, s1 + 1)), "warm_start": warm, "perplexity": {}}
    for v in kernels:
        os.environ["LDA_DENSE_HALF"] = v
        vals = []
        t = time.time()
        for seed in out["seeds"]:
            g = GibbsSampler(K, c.num_types, train.doc_off, train.words, alpha, BETA, seed=seed)
            g.set_warm_start(*warm)
            g.sweep(1000)
            vals.append(_perplexity(g, held_obs, held_sc, oracle))
            g.close()
        out["perplexity"]["quarter" if v == "2" else ("full" if v == "0" else "half")] = vals
        print(f"K={K} LDA_DENSE_HALF={v}: {len(vals)} seeds in {time.time() - t:.1f} s, "
              f"mean {np.mean(vals):.3f} median {np.median(vals):.3f}", file=sys.stderr, flush=True)
    os.environ["LDA_DENSE_HALF"] = "2"
    print(json.dumps(out))


if __name__ == "__main__":
    main()
