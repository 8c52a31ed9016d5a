#!/usr/bin/env python3
"""Per-seed held-out perplexity statistics: mean, median and the trapped-seed
rate of each sampler, each with a 95% bootstrap CI, and the differences to
cpu_mallet (tools/ppl_gpu_seeds.py and tools/ppl_mallet_seeds.py outputs).

A seed is TRAPPED when its perplexity exceeds the pooled median of all
samplers by more than 2% (the posterior's 5-12%-worse local optima).

  python tools/ppl_stats.py gpu_kK.json mallet_kK.json > stats_kK.json
"""
import json
import sys

import numpy as np

TRAP = 1.02


def boot_ci(x, stat, n=4000, seed=0):
    rng = np.random.default_rng(seed)
    x = np.asarray(x)
    s = np.array([stat(x[rng.integers(0, len(x), len(x))]) for _ in range(n)])
    return [float(np.percentile(s, 2.5)), float(np.percentile(s, 97.5))]


def boot_diff_ci(x, y, stat, n=4000, seed=1):
    rng = np.random.default_rng(seed)
    x, y = np.asarray(x), np.asarray(y)
    s = np.array([stat(x[rng.integers(0, len(x), len(x))]) / stat(y[rng.integers(0, len(y), len(y))]) - 1
                  for _ in range(n)])
    return [float(np.percentile(s, 2.5)), float(np.percentile(s, 97.5))]


def summarize(samples):
    pooled = np.median(np.concatenate([np.asarray(v) for v in samples.values()]))
    thr = TRAP * pooled
    out = {"trap_threshold": float(thr), "samplers": {}}
    for name, v in samples.items():
        v = np.asarray(v)
        good = v[v <= thr]
        out["samplers"][name] = {
            "n": int(len(v)),
            "mean": float(v.mean()), "mean_ci": boot_ci(v, np.mean),
            "median": float(np.median(v)), "median_ci": boot_ci(v, np.median),
            "trapped": int((v > thr).sum()), "trapped_rate": float((v > thr).mean()),
            "trapped_rate_ci": boot_ci(v, lambda s: float((s > thr).mean())),
            "untrapped_mean": float(good.mean()) if len(good) else None,
        }
    ref = np.asarray(samples["mallet"])
    for name, v in samples.items():
        if name == "mallet":
            continue
        v = np.asarray(v)
        s = out["samplers"][name]
        s["vs_mallet"] = {
            "mean_rel": float(v.mean() / ref.mean() - 1), "mean_rel_ci": boot_diff_ci(v, ref, np.mean),
            "median_rel": float(np.median(v) / np.median(ref) - 1),
            "median_rel_ci": boot_diff_ci(v, ref, np.median),
            "untrapped_mean_rel": (float(v[v <= thr].mean() / ref[ref <= thr].mean() - 1)
                                   if (v <= thr).any() and (ref <= thr).any() else None),
            "fisher_one_sided_p_more_trapped": fisher_greater(int((v > thr).sum()), len(v),
                                                              int((ref > thr).sum()), len(ref)),
        }
    return out


def fisher_greater(a, n1, b, n2):
    """One-sided Fisher exact p that sample 1's trapped rate exceeds sample 2's."""
    from scipy.stats import fisher_exact
    return float(fisher_exact([[a, n1 - a], [b, n2 - b]], alternative="greater")[1])


def main():
    g = json.load(open(sys.argv[1]))
    m = json.load(open(sys.argv[2]))
    samples = dict(g["perplexity"])
    samples["mallet"] = m["perplexity"]
    out = {"K": g["K"], "seeds_gpu": [g["seeds"][0], g["seeds"][-1]],
           "seeds_mallet": [m["seeds"][0], m["seeds"][-1]], **summarize(samples)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
