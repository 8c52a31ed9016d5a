"""Held-out perplexity: the GPU sampler vs the Mallet 2.0.7 restatement
(cpu_mallet), 1000 sweeps, optimizeInterval = 0 on both.

Estimator (the same for both trained states): document completion.  10% of
the documents are held out; each held-out document's first floor(L/2) tokens
are observed, theta is inferred against the frozen model with the GPU
TopicInferencer analogue (lda_infer: 100 iterations, burn-in 10, thinning 10
-- the reference's getSampledDistribution(inst, 100, 10, 10),
src/cmu_ron/TrainAndPredict.java:144), and the other half is scored:
perplexity = exp(-sum log sum_k theta_dk phi_kw / N_scored).

The posterior is multimodal: at K=20 about 30% of seeds end in a local
optimum 5-12% worse (cpu_mallet: 28 of 96 seeds), so a few seeds measure
which seeds fell in, not the sampler.  Sampling every document against one
snapshot from the random start falls in more often (41-44 of 96 seeds for
the full- and quarter-wave kernels, profiles/r03/ppl/stats_k20.json), so the
GPU leg trains with the product's warm start: sweeps 0..49 in 4 sequential
parts (lda_set_warm_start; ParallelTopicModel's default).  The GPU leg runs
SEEDS = 1..96 here; cpu_mallet's 96 per-seed values are the committed
fixture tests/golden/mallet_ppl_k{K}.json (tools/ppl_mallet_seeds.py: the
restatement trained on the CPU with 4 threads, scored by cpu_exact with the
same estimator and the GPU default kernel's inference draw).  Bars, each
against cpu_mallet (profiles/r03/ppl/ has the per-seed evidence and
bootstrap CIs, tools/ppl_stats.py):
  1. mean over the 96 seeds within 1% (north_star's tolerance);
  2. median not worse by more than 0.5% (and not better by more than 1%): a
     +1% shift of the typical (untrapped) chain fails this bar with
     certainty (the median's bootstrap CI is ~+-0.1%); a sampler that mixes
     better than the reference is not a parity failure, so the bar is
     one-sided at 0.5% and two-sided only at north_star's 1%;
  3. trapped-seed rate (perplexity > 1.02 x the pooled median) not larger
     than cpu_mallet's at one-sided Fisher p < 0.01: a mean shift carried by
     more trapped seeds is caught here or by bar 1.
Parity with Mallet itself is unpinned (Mallet cannot run in this image);
cpu_mallet is its restatement.
"""
import json
import os

import numpy as np
import pytest

pytestmark = [pytest.mark.gpu, pytest.mark.slow]

ALPHA_SUM, BETA = 10.0, 0.01


def score_state(oracle, K, V, train, z, held_obs, held_sc, alpha=None, beta=None):
    """Perplexity of a trained state z, scored on the CPU by cpu_exact (the
    bit-exact restatement of the GPU's inference draw: quarter-wave for
    K <= 128, the full-wave kernel above) with the estimator of _perplexity:
    the fixture path for cpu_mallet's states.  alpha/beta default to the
    plain test's symmetric ones; the reference-settings fixture passes the
    model's learned ones."""
    alpha = np.full(K, ALPHA_SUM / K) if alpha is None else np.asarray(alpha, dtype=np.float64)
    beta = BETA if beta is None else float(beta)
    # K > 1024 runs the large-K sparse sampler (k_sample_big), whose frozen
    # draw cpu_exact restates as exact_draw_big
    e = oracle.ExactSampler(K, V, train.doc_off, train.words, alpha, beta, 1,
                            z_init=z, half=2 if K <= 128 else 0,
                            kind="sparse" if K > LARGE_K else "dense")
    e.sweep(0)
    theta = e.infer(held_obs.doc_off, held_obs.words, n_iter=100, burn_in=10, thin=10, seed=7)
    nw, nwsum, _, _ = e.counts()
    ll = oracle.doc_completion_loglik(K, V, nw, nwsum, beta, theta, held_sc.doc_off, held_sc.words)
    return float(np.exp(-ll / held_sc.num_tokens))


def _perplexity(sampler, held_obs, held_sc, oracle):
    theta = sampler.infer(held_obs.doc_off, held_obs.words, n_iter=100, burn_in=10, thin=10, seed=7)
    nw, nwsum, _, _ = sampler.counts()
    ll = oracle.doc_completion_loglik(sampler.K, sampler.V, nw, nwsum, sampler.beta, theta,
                                      held_sc.doc_off, held_sc.words)
    return float(np.exp(-ll / held_sc.num_tokens))


SEEDS = range(1, 97)
LARGE_K = 1024        # above: the large-K sparse sampler (the dense kernels stop at 1024)
WARM = (4, 50)        # the training loop's default warm start (ParallelTopicModel.setWarmStart)
TRAP = 1.02
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def mallet_fixture(K):
    """cpu_mallet's per-seed perplexities (and the seeds) for the plain test."""
    path = os.path.join(GOLDEN, f"mallet_ppl_k{K}.json")
    if not os.path.exists(path):
        pytest.skip(f"no cpu_mallet fixture {path} (tools/ppl_mallet_seeds.py makes it)")
    with open(path) as f:
        d = json.load(f)
    assert (d["K"], d["alpha_sum"], d["beta"], d["sweeps"]) == (K, ALPHA_SUM, BETA, 1000)
    return np.asarray(d["perplexity"]), list(d.get("seeds", SEEDS))


def parity_bars(pg, pm):
    """(mean rel diff, median rel diff, one-sided Fisher p of more trapped
    seeds) of the GPU values pg against cpu_mallet's pm."""
    from scipy.stats import fisher_exact
    pg, pm = np.asarray(pg), np.asarray(pm)
    thr = TRAP * np.median(np.concatenate([pg, pm]))
    a, b = int((pg > thr).sum()), int((pm > thr).sum())
    p = fisher_exact([[a, len(pg) - a], [b, len(pm) - b]], alternative="greater")[1]
    return pg.mean() / pm.mean() - 1, np.median(pg) / np.median(pm) - 1, float(p), a, b


@pytest.mark.parametrize("K", [20, 100, 2048, 4096])
def test_heldout_perplexity_within_1pct(oracle, K):
    """K = 20 / 100: the quarter-wave / full-wave dense kernels over 96 seeds.
    K = 2048 / 4096 (round 6, VERDICT r5 missing #2): the large-K sparse
    sampler k_sample_big (C = 32 / 64), whose round-5 draw -- the exact
    fixed-point doc part and the own-entry accept / re-draw --
    had only a per-draw chi-square test behind it; 16 seeds each against the
    committed cpu_mallet fixture (tools/ppl_mallet_seeds.py, scored with the
    large-K inference draw), the same three bars."""
    from ldagibbssampling_amd.sampler import GibbsSampler
    c, train, held_obs, held_sc = _corpus_split(K)
    alpha = np.full(K, ALPHA_SUM / K)
    pm, seeds = mallet_fixture(K)
    pg = []
    for seed in seeds:
        g = GibbsSampler(K, c.num_types, train.doc_off, train.words, alpha, BETA, seed=seed,
                         sampler="sparse" if K > LARGE_K else "dense")
        g.set_warm_start(*WARM)
        g.sweep(1000)
        pg.append(_perplexity(g, held_obs, held_sc, oracle))
        g.close()
    dmean, dmed, p, a, b = parity_bars(pg, pm)
    print(f"K={K}: gpu mean {np.mean(pg):.3f} median {np.median(pg):.3f} trapped {a}/{len(pg)} | "
          f"cpu_mallet mean {pm.mean():.3f} median {np.median(pm):.3f} trapped {b}/{len(pm)} | "
          f"mean {dmean:+.3%} median {dmed:+.3%} Fisher p {p:.3f}")
    print("GPU_PER_SEED " + json.dumps({"K": K, "seeds": seeds, "perplexity": pg}))
    assert abs(dmean) <= 0.01
    assert -0.01 <= dmed <= 0.005
    assert p >= 0.01


def _corpus_split(K):
    from ldagibbssampling_amd.corpus import synthetic_lda, document_completion_split
    c = synthetic_lda(num_docs=2200, num_types=3000, num_topics=K, doc_len=None, mean_len=80,
                      min_len=10, max_len=300, seed=20261015, k_true=min(K, 50))
    rng = np.random.default_rng(0)
    perm = rng.permutation(c.num_docs)
    n_held = c.num_docs // 10
    train = c.subset(np.sort(perm[n_held:]))
    held_obs, held_sc = document_completion_split(c.subset(np.sort(perm[:n_held])))
    return c, train, held_obs, held_sc


REF_SEEDS = range(1, 49)
# learned hyperparameters: the mean over the seeds of the GPU model's learned
# alphaSum and beta within 3% of cpu_mallet's mean.  Both learn them from
# their own chains with the same Minka fixed points (lda_dirichlet.cpp /
# oracle, identical fp64 code on identical histograms, test_hyper.py), so a
# difference in the means is a difference in the chains' statistics: the
# seed-to-seed spread is ~0.2% (alphaSum) and ~1.5% (beta), so the means
# of 48 seeds carry ~0.05% / ~0.3% of noise and 3% is many standard errors;
# yet the staleness of the sweep moves them by more: snapshot sweeps learned
# beta +8..10% and alphaSum -3.7%, two equal sequential parts beta -9% and
# alphaSum +3%, the emulation of Mallet's 4 threads within ~0.6%
# (profiles/r04/hyper/).
HYPER_TOL = 0.03


def mallet_ref_fixture(K, alpha_sum, beta):
    with open(os.path.join(GOLDEN, f"mallet_ppl_ref_k{K}.json")) as f:
        d = json.load(f)
    assert (d["K"], d["alpha_sum"], d["beta"], d["sweeps"], d["threads"], d["optimize_interval"],
            d["burnin"]) == (K, alpha_sum, beta, 1000, 4, 20, 200)
    return d


@pytest.mark.parametrize("K,alpha_sum,beta", [
    (100, 10.0, 0.001),     # src/cmu/TrainAndPredict.java:259-263
    (500, 100.0, 1.0),      # src/cmu_ron/TrainAndPredict.java:160-165
])
def test_heldout_perplexity_reference_settings(oracle, K, alpha_sum, beta):
    """The reference's own training configuration -- the one the Java drop-in
    (GpuParallelTopicModel) runs: hyperparameter optimisation on
    (setOptimizeInterval(20), Mallet's default burn-in 200), setNumThreads(4),
    1000 sweeps, the native ParallelTopicModel's default sweep schedule (the
    warm start, then sweeps with the staleness of Mallet's 4 worker threads,
    lda_staleness_schedule: without it the model learned beta ~9% higher and
    alphaSum ~4% lower than cpu_mallet, and at K = 500 trapped 8 of 48
    chains).  48
    seeds of the native ParallelTopicModel on the GPU against the committed
    48-seed cpu_mallet fixture (tests/golden/mallet_ppl_ref_k{K}.json,
    tools/ppl_mallet_ref_seeds.py); each model is scored with its own learned
    alpha/beta.  The bars of test_heldout_perplexity_within_1pct (mean 1%,
    median 0.5%, trapped-seed rate by one-sided Fisher), plus the learned
    alphaSum and beta (HYPER_TOL)."""
    from ldagibbssampling_amd import topic_model as tm
    c, train, held_obs, held_sc = _corpus_split(K)
    alphabet = tm.Alphabet(range(c.num_types))
    held_il = tm.InstanceList.fromCorpus(held_obs, alphabet)
    train_il = tm.InstanceList.fromCorpus(train, alphabet)
    fx = mallet_ref_fixture(K, alpha_sum, beta)
    assert fx["seeds"] == list(REF_SEEDS)
    pg, asum, bet = [], [], []
    for seed in REF_SEEDS:
        m = tm.ParallelTopicModel(K, alpha_sum, beta)
        m.addInstances(train_il)
        m.setRandomSeed(seed)
        m.setTopicDisplay(0, 0)
        m.setOptimizeInterval(20)
        m.setNumThreads(4)
        m.setNumIterations(1000)
        m.estimate()
        theta = m.getInferencer().getSampledDistributions(held_il, 100, 10, 10, seed=7)
        nw, nwsum = m.typeTopicCounts()
        ll = oracle.doc_completion_loglik(K, c.num_types, nw, nwsum, m.beta, theta,
                                          held_sc.doc_off, held_sc.words)
        pg.append(float(np.exp(-ll / held_sc.num_tokens)))
        asum.append(float(m.alphaSum))
        bet.append(float(m.beta))
        m.close()
    pm = np.asarray(fx["perplexity"])
    dmean, dmed, p, a, b = parity_bars(pg, pm)
    da = np.mean(asum) / np.mean(fx["alpha_sum_learned"]) - 1
    db = np.mean(bet) / np.mean(fx["beta_learned"]) - 1
    print(f"K={K} (alphaSum {alpha_sum}, beta {beta}, optimizeInterval 20): gpu mean "
          f"{np.mean(pg):.3f} median {np.median(pg):.3f} trapped {a}/{len(pg)} | cpu_mallet mean "
          f"{pm.mean():.3f} median {np.median(pm):.3f} trapped {b}/{len(pm)} | mean {dmean:+.3%} "
          f"median {dmed:+.3%} Fisher p {p:.3f} | learned alphaSum {np.mean(asum):.4f} vs "
          f"{np.mean(fx['alpha_sum_learned']):.4f} ({da:+.2%}), beta {np.mean(bet):.6f} vs "
          f"{np.mean(fx['beta_learned']):.6f} ({db:+.2%})")
    print("GPU_PER_SEED " + json.dumps({"K": K, "perplexity": pg, "alpha_sum_learned": asum,
                                         "beta_learned": bet}))
    assert abs(dmean) <= 0.01
    assert -0.01 <= dmed <= 0.005
    assert p >= 0.01
    assert abs(da) <= HYPER_TOL and abs(db) <= HYPER_TOL
