#!/usr/bin/env python3
"""Which sampler semantics learn the hyperparameters cpu_mallet learns?

At the reference's settings (optimizeInterval 20, burn-in 200, 1000 sweeps;
tests/test_perplexity.py corpus) the GPU model learned alphaSum ~3.7% lower
and beta ~8-10% higher than cpu_mallet (4 threads).  This runs Mallet's
estimate() schedule over cpu_exact (the GPU's bit-exact semantics, the
restatement in tests/test_topic_model_gpu.py::_oracle_estimate) with a given
number of sequential parts per sweep -- P = 1 is the plain snapshot sweep
after the 4 x 50 warm start, P > 1 keeps every sweep in P sequential parts
(lda_set_warm_start(P, 1000)) -- and prints the learned alphaSum / beta and
the held-out perplexity per seed.

  python tools/hyper_dynamics.py K alpha_sum beta parts seed0 seed1 [jobs] > out.json
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


def run(args):
    K, alpha_sum, beta, parts, seed = args
    from oracle import oracle
    from test_perplexity import _corpus_split, score_state
    t0 = time.time()
    c, train, held_obs, held_sc = _corpus_split(K)
    V = c.num_types
    alpha = np.full(K, alpha_sum / K)
    o = oracle.ExactSampler(K, V, train.doc_off, train.words, alpha, beta, seed,
                            half=2 if K <= 128 else 0)
    if isinstance(parts, tuple):
        # two sequential parts of unequal size: part 0 takes the first
        # fraction f of each of the 64 blocks (the warm start's layout)
        f = parts[1]
        o.set_warm_start(2, 1000)
        off = o.doc_off - o.doc_off[0]
        N = int(off[-1])

        def runs():
            r = [[], []]
            prev = 0
            for b in range(64):
                for i, frac in enumerate((f, 1.0)):
                    tgt = int(N * (b + frac) / 64)
                    nxt = o.D if (b == 63 and i == 1) else int(np.searchsorted(off, tgt, side="left"))
                    nxt = min(max(nxt, prev), o.D)
                    if nxt > prev:
                        r[i].append((prev, nxt))
                    prev = nxt
            return r
        o._warm_runs = runs
    else:
        o.set_warm_start(4, 50) if parts == 1 else o.set_warm_start(parts, 1000)
    lens = np.diff(train.doc_off)
    L = int(lens.max())
    dl = np.zeros(L + 1, np.int32)
    td = np.zeros((K, L + 1), np.int32)
    totals = np.bincount(train.words, minlength=V)
    doc = np.repeat(np.arange(train.num_docs), lens)
    for it in range(1, 1001):
        o.sweep(1)
        if it > 200 and it % 10 == 0:
            nd = np.zeros((train.num_docs, K), np.int64)
            np.add.at(nd, (doc, o.z()), 1)
            dl += np.bincount(lens, minlength=L + 1).astype(np.int32)
            for k in range(K):
                v = nd[:, k]
                td[k] += np.bincount(v[v > 0], minlength=L + 1).astype(np.int32)
        if it > 200 and it % 20 == 0:
            alpha, alpha_sum = oracle.learn_parameters(alpha, td, dl, 1.001, 1.0, 1)
            dl[:] = 0
            td[:] = 0
            nw, nwsum = o.counts()[:2]
            counts = np.bincount(nw[nw > 0], minlength=int(totals.max()) + 1).astype(np.int32)
            sizes = np.bincount(nwsum, minlength=int(nwsum.max()) + 1).astype(np.int32)
            beta = oracle.learn_symmetric_concentration(counts, sizes, V, beta * V) / V
            o.set_alpha_beta(alpha, beta)
    ppl = score_state(oracle, K, V, train, o.z(), held_obs, held_sc, alpha=alpha, beta=beta)
    print(f"K={K} P={parts} seed {seed}: ppl {ppl:.3f} alphaSum {alpha.sum():.4f} beta {beta:.6f} "
          f"({time.time() - t0:.0f} s)", file=sys.stderr, flush=True)
    return seed, ppl, float(alpha.sum()), float(beta)


def main():
    K, asum, beta = int(sys.argv[1]), float(sys.argv[2]), float(sys.argv[3])
    # parts: "P" (P equal sequential parts) or "2:f" (two parts, the first a fraction f)
    parts = (2, float(sys.argv[4][2:])) if sys.argv[4].startswith("2:") else int(sys.argv[4])
    s0, s1 = int(sys.argv[5]), int(sys.argv[6])
    jobs = int(sys.argv[7]) if len(sys.argv) > 7 else 8
    out = {"K": K, "alpha_sum": asum, "beta": beta, "parts": parts, "seeds": [], "perplexity": [],
           "alpha_sum_learned": [], "beta_learned": []}
    with ProcessPoolExecutor(jobs) as ex:
        for seed, ppl, a, b in ex.map(run, [(K, asum, beta, parts, s) for s in range(s0, s1 + 1)]):
            out["seeds"].append(seed)
            out["perplexity"].append(ppl)
            out["alpha_sum_learned"].append(a)
            out["beta_learned"].append(b)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
