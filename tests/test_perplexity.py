"""Held-out perplexity: the GPU sampler vs the Mallet 2.0.7 restatement
(cpu_mallet), 1000 sweeps, seeds {1, 2, 3}, optimizeInterval = 0 on both.

Estimator (the same for both trained states): document completion.  10% of
the documents are held out; each held-out document's first floor(L/2) tokens
are observed, theta is inferred against the frozen model with the GPU
TopicInferencer analogue (lda_infer: 100 iterations, burn-in 10, thinning 10
— the reference's getSampledDistribution(inst, 100, 10, 10),
src/cmu_ron/TrainAndPredict.java:144), and the other half is scored:
perplexity = exp(-sum log sum_k theta_dk phi_kw / N_scored).
The Mallet state is evaluated by loading its z into a GPU context.

Tolerance: |median_gpu - median_mallet| <= 1% of median_mallet over seeds
1..12 (BASELINE.json north_star).  The median, not the mean of a few seeds:
the posterior is multimodal, and about one seed in six ends in a local
optimum 5-12% worse in EVERY implementation -- cpu_mallet seeds 10 and 12,
the full-wave kernel's 4 and 10, the quarter-wave kernel's 1, 4, 6 and 10 at
K=20 (profiles/r02/quarter/ppl_k20.json, tools/perplexity_seeds.py) -- so a
three-seed mean measures which seeds fell into one, not the sampler.  Parity with Mallet itself is unpinned (Mallet cannot run in
this image); cpu_mallet is its restatement.
"""
import numpy as np
import pytest

pytestmark = [pytest.mark.gpu, pytest.mark.slow]

ALPHA_SUM, BETA = 10.0, 0.01


def score_state(oracle, K, V, train, z, held_obs, held_sc):
    """Perplexity of a trained state z, scored on the CPU by cpu_exact (the
    bit-exact restatement of the GPU's quarter-wave inference draw) with the
    estimator of _perplexity: the fixture path for cpu_mallet's states."""
    e = oracle.ExactSampler(K, V, train.doc_off, train.words, np.full(K, ALPHA_SUM / K), BETA, 1,
                            z_init=z, half=2)
    e.sweep(0)
    theta = e.infer(held_obs.doc_off, held_obs.words, n_iter=100, burn_in=10, thin=10, seed=7)
    nw, nwsum, _, _ = e.counts()
    ll = oracle.doc_completion_loglik(K, V, nw, nwsum, BETA, theta, held_sc.doc_off, held_sc.words)
    return float(np.exp(-ll / held_sc.num_tokens))


def _perplexity(sampler, held_obs, held_sc, oracle):
    theta = sampler.infer(held_obs.doc_off, held_obs.words, n_iter=100, burn_in=10, thin=10, seed=7)
    nw, nwsum, _, _ = sampler.counts()
    ll = oracle.doc_completion_loglik(sampler.K, sampler.V, nw, nwsum, sampler.beta, theta,
                                      held_sc.doc_off, held_sc.words)
    return float(np.exp(-ll / held_sc.num_tokens))


@pytest.mark.parametrize("K,alpha_sum,beta", [(20, 10.0, 0.01), (100, 10.0, 0.01)])
def test_heldout_perplexity_within_1pct(oracle, K, alpha_sum, beta):
    from ldagibbssampling_amd.corpus import synthetic_lda, document_completion_split
    from ldagibbssampling_amd.sampler import GibbsSampler
    c = synthetic_lda(num_docs=2200, num_types=3000, num_topics=K, doc_len=None, mean_len=80,
                      min_len=10, max_len=300, seed=20261015, k_true=min(K, 50))
    rng = np.random.default_rng(0)
    perm = rng.permutation(c.num_docs)
    n_held = c.num_docs // 10
    train = c.subset(np.sort(perm[n_held:]))
    held_obs, held_sc = document_completion_split(c.subset(np.sort(perm[:n_held])))
    alpha = np.full(K, alpha_sum / K)
    pg, pm = [], []
    for seed in range(1, 13):
        g = GibbsSampler(K, c.num_types, train.doc_off, train.words, alpha, beta, seed=seed)
        g.sweep(1000)
        pg.append(_perplexity(g, held_obs, held_sc, oracle))
        m = oracle.MalletModel(K, alpha_sum, beta, c.num_types, train.doc_off, train.words,
                               seed=seed, num_threads=4)
        m.estimate(1000)
        gm = GibbsSampler(K, c.num_types, train.doc_off, train.words, alpha, beta, seed=seed,
                          z_init=m.z())
        gm.sweep(0)
        pm.append(_perplexity(gm, held_obs, held_sc, oracle))
    mg, mm = float(np.median(pg)), float(np.median(pm))
    print(f"K={K}: gpu {pg} median {mg:.3f} | cpu_mallet {pm} median {mm:.3f} | "
          f"rel diff {(mg - mm) / mm:+.4%}")
    assert abs(mg - mm) <= 0.01 * mm


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


@pytest.mark.parametrize("K,alpha_sum,beta", [
    (100, 10.0, 0.001),     # src/cmu/TrainAndPredict.java:259
    (500, 100.0, 1.0),      # src/cmu_ron/TrainAndPredict.java:160
])
def test_heldout_perplexity_reference_settings(oracle, K, alpha_sum, beta):
    """The reference's own training configuration, hyperparameter optimisation
    on (setOptimizeInterval(20), Mallet's default burn-in 200, 4 threads,
    1000 sweeps): the native ParallelTopicModel on the GPU vs cpu_mallet.
    Each model is scored with its own learned alpha/beta."""
    from ldagibbssampling_amd import topic_model as tm
    from ldagibbssampling_amd.sampler import GibbsSampler
    c, train, held_obs, held_sc = _corpus_split(K)
    alphabet = tm.Alphabet(range(c.num_types))
    held_il = tm.InstanceList.fromCorpus(held_obs, alphabet)
    pg, pm, hyper = [], [], []
    for seed in (1, 2, 3):
        m = tm.ParallelTopicModel(K, alpha_sum, beta)
        m.addInstances(tm.InstanceList.fromCorpus(train, alphabet))
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
        mm = oracle.MalletModel(K, alpha_sum, beta, c.num_types, train.doc_off, train.words,
                                seed=seed, num_threads=4)
        mm.set_optimize(20, burnin=200)
        mm.estimate(1000)
        a_m, b_m = mm.hyper()
        gm = GibbsSampler(K, c.num_types, train.doc_off, train.words, a_m, b_m, seed=seed,
                          z_init=mm.z())
        gm.sweep(0)
        pm.append(_perplexity(gm, held_obs, held_sc, oracle))
        hyper.append((float(m.alphaSum), float(m.beta), float(a_m.sum()), float(b_m)))
    # medians: one seed in a local optimum must not decide (see above)
    mg, mmn = float(np.median(pg)), float(np.median(pm))
    print(f"K={K} (alphaSum {alpha_sum}, beta {beta}, optimizeInterval 20): gpu {pg} median "
          f"{mg:.3f} | cpu_mallet {pm} median {mmn:.3f} | rel diff {(mg - mmn) / mmn:+.4%} | "
          f"learned (alphaSum, beta) gpu/mallet {hyper}")
    assert abs(mg - mmn) <= 0.01 * mmn
