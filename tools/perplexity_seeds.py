#!/usr/bin/env python3
"""Held-out perplexity over many seeds (tests/test_perplexity.py's corpus and
estimator): the GPU sampler under each dense kernel (LDA_DENSE_HALF 0 =
full-wave, 2 = quarter-wave) and the cpu_mallet restatement, to tell a
local-optimum outlier of one seed from a bias of a kernel's draw.

  python tools/perplexity_seeds.py K seeds... > out.json
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from oracle import oracle  # noqa: E402  (the checker: cpu_mallet, doc_completion_loglik)
from test_perplexity import _corpus_split, _perplexity  # noqa: E402


def main():
    from ldagibbssampling_amd.sampler import GibbsSampler
    K = int(sys.argv[1])
    seeds = [int(s) for s in sys.argv[2:]] or list(range(1, 11))
    c, train, held_obs, held_sc = _corpus_split(K)
    alpha_sum, beta = 10.0, 0.01
    alpha = np.full(K, alpha_sum / K)
    res = {"K": K, "seeds": seeds, "gpu": {}, "mallet": []}
    for v in ("0", "2"):
        os.environ["LDA_DENSE_HALF"] = v
        out = []
        for seed in seeds:
            g = GibbsSampler(K, c.num_types, train.doc_off, train.words, alpha, beta, seed=seed)
            g.sweep(1000)
            out.append(_perplexity(g, held_obs, held_sc, oracle))
            print(f"v{v} seed {seed}: {out[-1]:.3f}", file=sys.stderr, flush=True)
        res["gpu"][v] = out
    os.environ["LDA_DENSE_HALF"] = "2"
    for seed in seeds:
        m = oracle.MalletModel(K, alpha_sum, beta, c.num_types, train.doc_off, train.words,
                               seed=seed, num_threads=4)
        m.estimate(1000)
        gm = GibbsSampler(K, c.num_types, train.doc_off, train.words, alpha, beta, seed=seed,
                          z_init=m.z())
        gm.sweep(0)
        res["mallet"].append(_perplexity(gm, held_obs, held_sc, oracle))
        print(f"mallet seed {seed}: {res['mallet'][-1]:.3f}", file=sys.stderr, flush=True)
    for k, v in list(res["gpu"].items()) + [("mallet", res["mallet"])]:
        print(f"{k}: mean {np.mean(v):.3f} median {np.median(v):.3f}", file=sys.stderr)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
