#!/usr/bin/env python3
"""Generate the committed golden fixtures under tests/golden/.

Run from the repo root:  python tests/golden/make_golden.py
Everything is produced by the CPU oracle (oracle/, test infrastructure) and
the corpus helpers; the reference itself has no fixtures, tests or runnable
sampler, so these pin the build's own definitions:
  exact_*.npz   cpu_exact: inputs, z after sweeps {1, 10, 100}, sha256 of
                nw/nwsum/nd, LL per checkpoint (bit-exact contract of the GPU)
  mallet_ll.json cpu_mallet (Mallet 2.0.7 restatement) LL/token traces
  inverse_docs_sample.txt.gz + inverse_docs_expected.json
                50 docs in the reference's corpus format
                (src/ron/GenerateInverseDocs.java:40-58) and the alphabet /
                word ids the cmu_ron InstanceImporter pipeline must produce
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from ldagibbssampling_amd.corpus import (Corpus, synthetic_changelists, synthetic_lda,  # noqa: E402
                                         write_inverse_docs)
from oracle import oracle as O  # noqa: E402

CASES = {
    # name: (corpus builder, K, alpha, beta, seed, checkpoints)
    "k4_tiny": (lambda: synthetic_lda(50, 100, 4, doc_len=None, mean_len=20, min_len=0,
                                      max_len=60, seed=1), 4, 0.5, 0.1, 11, (1, 10, 100)),
    "k20_changelists": (lambda: synthetic_changelists(200, 500, seed=2), 20, 0.5, 0.01, 12,
                        (1, 10, 100)),
    "k128_ragged": (lambda: synthetic_lda(100, 400, 128, doc_len=None, mean_len=70, min_len=0,
                                          max_len=300, seed=3), 128, 0.1, 0.01, 13, (1, 10)),
    "k1000_wide": (lambda: synthetic_lda(40, 300, 1000, doc_len=None, mean_len=90, min_len=1,
                                         max_len=250, seed=4), 1000, 0.05, 0.01, 14, (1, 3)),
    # the sparse draw (LDA_SAMPLER_SPARSE): C <= 16 fma-chain doc partials and
    # C = 32 / 64 16-lane row-scan group partials (k_sample_sparse_big)
    "k128_sparse": (lambda: synthetic_lda(100, 400, 128, doc_len=None, mean_len=70, min_len=0,
                                          max_len=300, seed=7), 128, 0.1, 0.01, 17, (1, 10),
                    "sparse"),
    "k2048_sparse": (lambda: synthetic_lda(60, 500, 64, doc_len=None, mean_len=120, min_len=1,
                                           max_len=400, seed=8), 2048, 0.02, 0.01, 18, (1, 5),
                     "sparse"),
    "k4096_sparse": (lambda: synthetic_lda(40, 300, 64, doc_len=None, mean_len=150, min_len=1,
                                           max_len=500, seed=9), 4096, 0.01, 0.05, 19, (1, 4),
                     "sparse"),
}
# dense K <= 128 runs the quarter-wave kernel by default (LDA_DENSE_HALF
# unset = 2, exact_draw_quarter); the cases above pin the full-wave
# k_sample<C> draw (half = 0, LDA_DENSE_HALF=0), these the default one
for _n in ("k4_tiny", "k20_changelists", "k128_ragged"):
    CASES[_n + "_quarter"] = CASES[_n] + ("dense", 2)


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def exact_case(name):
    build, K, alpha, beta, seed, checkpoints = CASES[name][:6]
    kind = CASES[name][6] if len(CASES[name]) > 6 else "dense"
    half = CASES[name][7] if len(CASES[name]) > 7 else 0
    c = build()
    o = O.ExactSampler(K, c.num_types, c.doc_off, c.words, alpha, beta, seed, kind=kind, half=half)
    o.apply()
    out = {"doc_off": c.doc_off, "words": c.words, "K": K, "V": c.num_types, "alpha": alpha,
           "beta": beta, "seed": seed, "checkpoints": np.array(checkpoints), "kind": kind,
           "half": half}
    out["z_0"] = o.z().astype(np.int16 if K < 32768 else np.int32)
    done = 0
    meta = {}
    for cp in checkpoints:
        o.sweep(cp - done)
        done = cp
        nw, nwsum, nd, _ = o.counts(with_nd=True)
        out[f"z_{cp}"] = o.z().astype(np.int16)
        meta[str(cp)] = {"nw_sha256": sha(nw), "nwsum_sha256": sha(nwsum), "nd_sha256": sha(nd),
                         "log_likelihood": o.log_likelihood()}
    out["meta"] = np.array(json.dumps(meta))
    np.savez_compressed(os.path.join(HERE, f"exact_{name}.npz"), **out)


def mallet_traces():
    c = synthetic_changelists(300, 600, seed=5)
    res = {"corpus": "synthetic_changelists(300, 600, seed=5)", "K": 20, "alpha_sum": 10.0,
           "beta": 0.01, "traces": {}}
    for threads in (1, 4):
        for seed in (1, 2, 3):
            m = O.MalletModel(20, 10.0, 0.01, c.num_types, c.doc_off, c.words, seed=seed,
                              num_threads=threads)
            tr = []
            for _ in range(5):
                m.estimate(10)
                tr.append(m.log_likelihood() / c.num_tokens)
            res["traces"][f"T{threads}_seed{seed}"] = {"ll_per_token_every_10": tr,
                                                       "z_sha256": sha(m.z())}
    with open(os.path.join(HERE, "mallet_ll.json"), "w") as f:
        json.dump(res, f, indent=1)


def hyper():
    """Dirichlet estimators on fixed histograms, and the Mallet restatement's
    optimisation schedule (optimizeInterval 10, burn-in 20) on a small corpus."""
    rng = np.random.default_rng(10)
    hist = rng.integers(0, 40, size=(12, 61)).astype(np.int32)
    hist[:, 0] = 0
    hist[3] = 0                                     # a topic in no document
    lens = rng.integers(0, 30, size=61).astype(np.int32)
    lens[0] = 0
    a0 = rng.uniform(0.05, 1.0, size=12)
    a1, s1 = O.learn_parameters(a0, hist, lens, 1.001, 1.0, 1)
    a5, s5 = O.learn_parameters(a0, hist, lens, 1.001, 1.0, 5)
    counts = np.bincount(rng.integers(1, 200, size=5000), minlength=201).astype(np.int32)
    sizes = np.zeros(3001, np.int32)
    sizes[rng.integers(1, 3000, size=40)] += 1
    sym = O.learn_symmetric_concentration(counts, sizes, 700, 7.0)
    c = synthetic_changelists(300, 600, seed=5)
    m = O.MalletModel(20, 10.0, 0.01, c.num_types, c.doc_off, c.words, seed=4, num_threads=2)
    m.set_optimize(10, burnin=20)
    m.estimate(60)
    a_m, b_m = m.hyper()
    res = {"learn_parameters": {"hist": hist.tolist(), "lens": lens.tolist(), "alpha0": a0.tolist(),
                                "alpha_1": a1.tolist(), "sum_1": s1, "alpha_5": a5.tolist(),
                                "sum_5": s5},
           "learn_symmetric_concentration": {"counts": counts.tolist(), "sizes": sizes.tolist(),
                                             "dims": 700, "value0": 7.0, "value": sym},
           "mallet_optimised": {"corpus": "synthetic_changelists(300, 600, seed=5)", "K": 20,
                                "alpha_sum": 10.0, "beta": 0.01, "seed": 4, "threads": 2,
                                "optimize_interval": 10, "burnin": 20, "iterations": 60,
                                "alpha": a_m.tolist(), "beta_out": b_m,
                                "z_sha256": sha(m.z())}}
    with open(os.path.join(HERE, "hyper.json"), "w") as f:
        json.dump(res, f)


def inverse_docs():
    c = synthetic_changelists(50, 300, seed=6)
    # mixed case on purpose: the pipeline lower-cases (InstanceImporter.java:35)
    alphabet = [t.replace("File", "FILE") if i % 3 == 0 else t for i, t in enumerate(c.alphabet)]
    c = Corpus(c.doc_off, c.words, c.num_types, alphabet, c.targets)
    write_inverse_docs(os.path.join(HERE, "inverse_docs_sample.txt.gz"), c)
    expected = {"targets": c.targets, "alphabet": [t.lower() for t in alphabet],
                "doc_off": c.doc_off.tolist(), "words": c.words.tolist()}
    with open(os.path.join(HERE, "inverse_docs_expected.json"), "w") as f:
        json.dump(expected, f)


if __name__ == "__main__":
    # python tests/golden/make_golden.py [case | mallet | hyper | inverse ...]  (default: all)
    O.build()
    want = set(sys.argv[1:])
    for n in CASES:
        if not want or n in want:
            exact_case(n)
    if not want or "mallet" in want:
        mallet_traces()
    if not want or "hyper" in want:
        hyper()
    if not want or "inverse" in want:
        inverse_docs()
    print("golden fixtures written to", HERE)
