#!/usr/bin/env python3
"""Cost of Mallet's hyperparameter optimisation at benchmark scale (VERDICT r1
item 7): the native ParallelTopicModel (liblda_topic_model.so) runs
estimate() on the C4 shard (1.25M docs x 200 tokens, V = 100k, K = 512) with
setOptimizeInterval(20) and burn-in 0, and again with optimisation off; the
difference per optimisation is set against the 20 sweeps between two of them.

  python tools/opt_cost.py [--docs N] [--iters 40]
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(L, corpus, K, iters, interval, seed=1):
    from ldagibbssampling_amd.topic_model import _check
    h = C.c_void_p()
    _check(L.ldatm_create(C.byref(h), K, 0.1 * K, 0.01), "create")
    _check(L.ldatm_set_alphabet(h, corpus.num_types, None), "alphabet")
    off = np.ascontiguousarray(corpus.doc_off, np.int64)
    _check(L.ldatm_add_instances(h, corpus.num_docs, off, corpus.words.ctypes.data, None), "add")
    _check(L.ldatm_set_random_seed(h, seed), "seed")
    _check(L.ldatm_set_num_iterations(h, iters), "iters")
    _check(L.ldatm_set_burnin_period(h, 0), "burnin")
    _check(L.ldatm_set_optimize_interval(h, interval), "interval")
    _check(L.ldatm_set_print_log_likelihood(h, 0), "ll")
    _check(L.ldatm_set_topic_display(h, 0, 0), "display")
    _check(L.ldatm_set_num_iterations(h, 1), "warm")
    _check(L.ldatm_estimate(h), "warm-up estimate")        # shards built, kernels warm
    _check(L.ldatm_set_num_iterations(h, iters), "iters")
    t0 = time.perf_counter()
    _check(L.ldatm_estimate(h), "estimate")
    dt = time.perf_counter() - t0
    a = np.zeros(K)
    s, b = C.c_double(), C.c_double()
    _check(L.ldatm_get_hyper(h, a.ctypes.data, C.byref(s), C.byref(b)), "hyper")
    L.ldatm_destroy(h)
    return dt, s.value, b.value


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--docs", type=int, default=1_250_000)
    ap.add_argument("--iters", type=int, default=40)
    args = ap.parse_args()
    import torch  # noqa: F401  (one HIP runtime per process: torch's)
    from ldagibbssampling_amd.corpus import synthetic_lda_torch
    from ldagibbssampling_amd.topic_model import load_tm
    L = load_tm()
    K, V = 512, 100_000
    c = synthetic_lda_torch(args.docs, V, K, doc_len=200, seed=20261015, device="cuda:0")
    off_s, _, _ = run(L, c, K, args.iters, 0)
    on_s, asum, beta = run(L, c, K, args.iters, 20)
    n_opt = args.iters // 20
    per_opt = (on_s - off_s) / max(n_opt, 1)
    sweep_s = off_s / args.iters
    print(json.dumps({
        "workload": f"C4 shard: {args.docs} docs x 200, V={V}, K={K}",
        "iterations": args.iters, "optimisations": n_opt,
        "estimate_s_optimize_off": off_s, "estimate_s_optimize_20": on_s,
        "seconds_per_optimisation": per_opt, "seconds_per_sweep": sweep_s,
        "optimisation_share_of_20_sweeps": per_opt / (per_opt + 20 * sweep_s),
        "alpha_sum_after": asum, "beta_after": beta}))


if __name__ == "__main__":
    main()
