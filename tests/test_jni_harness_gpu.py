"""The Java drop-in's native call, compiled and run on the GPU.

cmu_gpu.GpuParallelTopicModel.estimate() (integration/java/) pins its arrays
and calls ldaj_estimate (integration/jni/lda_jni_core.c) through the JNI glue.
tests/jni/estimate_harness.c makes that same call with the Java method's
marshalling (typeTopicCounts rows of min(K, typeTotal), LL buffers, options,
the sweep-counter field).  Checked here against the oracle-driven restatement
of Mallet's estimate() schedule (test_topic_model_gpu._oracle_estimate's
schedule from a given state):
  - z, alpha, alphaSum, beta, tokensPerTopic, the packed typeTopicCounts rows
    and the LL/token trace of a first estimate() from Mallet's own topics;
  - updateModel (src/cmu_ron/TrainAndPredict.java:173-177): documents (and
    types) added, a second estimate() from the written-back state, whose
    Philox stream continues (its z differs from a replay from sweep 0);
  - K > 1024 goes to the large-K sparse sampler without being asked.
"""
import os
import subprocess
import tempfile

import numpy as np
import pytest

from ldagibbssampling_amd.corpus import Corpus, synthetic_lda

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HARNESS = os.path.join(ROOT, "tests", "jni", "bin", "estimate_harness")
FAKE = os.path.join(ROOT, "tests", "jni", "bin", "fake_env")


def _run(K, V, corpus, z, alpha, hyper, sweep, options, seed, prog=HARNESS):
    assert os.path.exists(prog), "build() compiles tests/jni/bin/estimate_harness and fake_env"
    D = corpus.num_docs
    with tempfile.TemporaryDirectory() as d:
        fin, fout = os.path.join(d, "in.bin"), os.path.join(d, "out.bin")
        with open(fin, "wb") as f:
            f.write(np.array([K, V, D], np.int32).tobytes())
            f.write(np.asarray(corpus.doc_off, np.int64).tobytes())
            f.write(np.asarray(corpus.words, np.int32).tobytes())
            f.write(np.asarray(z, np.int32).tobytes())
            f.write(np.asarray(alpha, np.float64).tobytes())
            f.write(np.asarray(hyper, np.float64).tobytes())
            f.write(np.array([sweep], np.int64).tobytes())
            f.write(np.asarray(options, np.int32).tobytes())
            f.write(np.array([seed], np.int64).tobytes())
        r = subprocess.run([prog, fin, fout], capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stderr
        buf = open(fout, "rb").read()
    N = corpus.num_tokens
    out, p = {}, 0

    def take(name, dt, n):
        nonlocal p
        a = np.frombuffer(buf, dt, n, p)
        p += a.nbytes
        out[name] = a.copy()
        return out[name]

    take("z", np.int32, N)
    take("alpha", np.float64, K)
    take("hyper", np.float64, 3)
    out["sweep"] = int(take("sweep", np.int64, 1)[0])
    ro = take("row_off", np.int64, V + 1)
    take("rows", np.int32, int(ro[-1]))
    take("tpt", np.int32, K)
    n = int(take("n_ll", np.int32, 1)[0])
    take("ll_iter", np.int32, n)
    take("ll_value", np.float64, n)
    assert p == len(buf)
    return out


def _oracle_schedule(oracle, corpus, V, K, z0, alpha, alpha_sum, beta, seed, sweep0, iters,
                     interval, burnin, save, symmetric=False, kind="dense", threads=1):
    """Mallet's estimate() over cpu_exact from a given state (the test-side
    restatement: sweeps, statistics, optimizeAlpha / optimizeBeta, LL/10).
    threads: the options' numThreads, whose staleness the sweeps past the
    warm start emulate (lda_staleness_schedule)."""
    o = oracle.ExactSampler(K, V, corpus.doc_off, corpus.words, alpha, beta, seed, z_init=z0,
                            kind=kind)
    o.set_warm_start(4, 50)       # the native model's default warm start, keyed by the sweep counter
    o.set_sequential_sweeps(*oracle.staleness_schedule(threads))
    o.sweep_index = sweep0
    lens = np.diff(corpus.doc_off)
    L = int(lens.max())
    dl = np.zeros(L + 1, np.int32)
    td = np.zeros((K, L + 1), np.int32)
    totals = np.bincount(corpus.words, minlength=V)
    doc = np.repeat(np.arange(corpus.num_docs), lens)
    alpha = np.asarray(alpha, np.float64).copy()
    ll = []
    for it in range(1, iters + 1):
        o.sweep(1)
        opt = it > burnin and interval != 0
        if opt and it % save == 0:
            nd = np.zeros((corpus.num_docs, K), np.int64)
            np.add.at(nd, (doc, o.z()), 1)
            dl += np.bincount(lens, minlength=L + 1).astype(np.int32)
            for k in range(K):
                v = nd[:, k]
                td[k] += np.bincount(v[v > 0], minlength=L + 1).astype(np.int32)
        if opt and it % interval == 0:
            if symmetric:
                s = oracle.learn_symmetric_concentration(td.sum(0), dl, K, alpha_sum)
                alpha_sum, alpha = s, np.full(K, s / K)
            else:
                alpha, alpha_sum = oracle.learn_parameters(alpha, td, dl, 1.001, 1.0, 1)
            dl[:] = 0
            td[:] = 0
            nw, nwsum = o.counts()[:2]
            counts = np.bincount(nw[nw > 0], minlength=int(totals.max()) + 1).astype(np.int32)
            sizes = np.bincount(nwsum, minlength=int(nwsum.max()) + 1).astype(np.int32)
            beta = oracle.learn_symmetric_concentration(counts, sizes, V, beta * V) / V
            o.set_alpha_beta(alpha, beta)
        if it % 10 == 0:
            ll.append((it, o.log_likelihood() / corpus.num_tokens))
    return o, alpha, alpha_sum, beta, ll


def _packed(nw, K, row_off):
    """typeTopicCounts rows from dense counts, Mallet's layout."""
    mask = K - 1 if K & (K - 1) == 0 else (1 << K.bit_length()) - 1
    bits = bin(mask).count("1")
    rows = np.zeros(int(row_off[-1]), np.int32)
    for w in range(nw.shape[0]):
        ks = np.nonzero(nw[w])[0]
        cells = np.sort((nw[w, ks].astype(np.int64) << bits) | ks)[::-1]
        rows[row_off[w]:row_off[w] + len(cells)] = cells
    return rows


def _check(out, o, alpha, alpha_sum, beta, ll, K, V, iters):
    np.testing.assert_array_equal(out["z"], o.z())
    np.testing.assert_array_equal(out["alpha"], alpha)
    assert out["hyper"][0] == alpha_sum and out["hyper"][1] == beta
    assert out["hyper"][2] == beta * V
    nw, nwsum = o.counts()[:2]
    np.testing.assert_array_equal(out["tpt"], nwsum)
    np.testing.assert_array_equal(out["rows"], _packed(nw, K, out["row_off"]))
    assert list(out["ll_iter"]) == [i for i, _ in ll]
    np.testing.assert_allclose(out["ll_value"], [v for _, v in ll], rtol=1e-9)


def test_estimate_then_update_model(oracle):
    c = synthetic_lda(num_docs=260, num_types=700, num_topics=12, doc_len=None, mean_len=50,
                      min_len=1, max_len=160, seed=11)
    first = c.subset(range(0, 200))
    V1, K, seed = 680, 16, 3                    # types 680..699 appear only in the update
    first = Corpus(first.doc_off, np.minimum(first.words, V1 - 1).astype(np.int32), V1)
    rng = np.random.default_rng(8)
    z0 = rng.integers(0, K, first.num_tokens).astype(np.int32)   # Mallet's addInstances draws
    alpha0 = np.full(K, 8.0 / K)
    hyper0 = np.array([8.0, 0.05, 0.05 * V1])
    iters, interval, burnin, save = 40, 10, 10, 5
    opts = [iters, burnin, interval, save, 0, 4, 0]             # numThreads 4 -> the GPUs here
    out1 = _run(K, V1, first, z0, alpha0, hyper0, 0, opts, seed)
    o, alpha, alpha_sum, beta, ll = _oracle_schedule(oracle, first, V1, K, z0, alpha0, 8.0, 0.05,
                                                     seed, 0, iters, interval, burnin, save, threads=4)
    _check(out1, o, alpha, alpha_sum, beta, ll, K, V1, iters)
    assert out1["sweep"] == iters
    assert not np.allclose(alpha, alpha0) and beta != 0.05

    # updateModel: more documents (and types), Mallet's random topics for them,
    # the written-back state for the rest, and the sweep counter field
    V2 = c.num_types
    both = Corpus(np.concatenate([first.doc_off, c.doc_off[201:261] - c.doc_off[200]
                                  + first.doc_off[-1]]),
                  np.concatenate([first.words, c.words[c.doc_off[200]:c.doc_off[260]]]), V2)
    z_new = rng.integers(0, K, both.num_tokens - first.num_tokens).astype(np.int32)
    z1 = np.concatenate([out1["z"], z_new])
    iters2 = 20
    opts2 = [iters2, burnin, interval, save, 0, 4, 0]
    out2 = _run(K, V2, both, z1, out1["alpha"], [out1["hyper"][0], out1["hyper"][1],
                                                 out1["hyper"][1] * V2], out1["sweep"], opts2, seed)
    o2, alpha2, alpha_sum2, beta2, ll2 = _oracle_schedule(
        oracle, both, V2, K, z1, out1["alpha"], out1["hyper"][0], out1["hyper"][1], seed,
        iters, iters2, interval, burnin, save, threads=4)
    _check(out2, o2, alpha2, alpha_sum2, beta2, ll2, K, V2, iters2)
    assert out2["sweep"] == iters + iters2
    # without the carried counter the second estimate() would replay sweep 0's uniforms
    replay = _run(K, V2, both, z1, out1["alpha"], [out1["hyper"][0], out1["hyper"][1],
                                                   out1["hyper"][1] * V2], 0, opts2, seed)
    assert not np.array_equal(replay["z"], out2["z"])


def test_large_k_selects_sparse_sampler(oracle):
    c = synthetic_lda(num_docs=80, num_types=500, num_topics=40, doc_len=None, mean_len=60,
                      min_len=1, max_len=200, seed=5)
    K, seed = 2048, 9
    rng = np.random.default_rng(1)
    z0 = rng.integers(0, K, c.num_tokens).astype(np.int32)
    alpha0 = np.full(K, 50.0 / K)
    hyper0 = np.array([50.0, 0.01, 0.01 * c.num_types])
    out = _run(K, c.num_types, c, z0, alpha0, hyper0, 5, [12, 200, 0, 10, 0, 1, 0], seed)
    o, alpha, alpha_sum, beta, ll = _oracle_schedule(oracle, c, c.num_types, K, z0, alpha0, 50.0,
                                                     0.01, seed, 5, 12, 0, 200, 10, kind="sparse")
    _check(out, o, alpha, alpha_sum, beta, ll, K, c.num_types, 12)


def test_checkpoint_resume_equals_uninterrupted(oracle):
    """Checkpoint/resume (src/cmu_ron/TrainAndPredict.java:179-200): Mallet's
    ObjectOutputStream saves the fields estimate() wrote back (topicSequence,
    alpha, alphaSum, beta, betaSum) and the sweep-counter field of the
    drop-in; a model read back and trained on continues the chain exactly:
    estimate(15) -> save -> load -> estimate(25) == estimate(40).  (With
    optimisation off: Mallet restarts its iteration counter, and so its
    optimisation schedule, in every estimate() call.)"""
    c = synthetic_lda(num_docs=150, num_types=600, num_topics=10, doc_len=None, mean_len=40,
                      min_len=1, max_len=120, seed=21)
    K, V, seed = 24, c.num_types, 17
    z0 = np.random.default_rng(4).integers(0, K, c.num_tokens).astype(np.int32)
    alpha0 = np.full(K, 6.0 / K)
    hyper0 = np.array([6.0, 0.02, 0.02 * V])
    whole = _run(K, V, c, z0, alpha0, hyper0, 0, [40, 200, 0, 10, 0, 2, 0], seed)
    part = _run(K, V, c, z0, alpha0, hyper0, 0, [15, 200, 0, 10, 0, 2, 0], seed)
    with tempfile.TemporaryDirectory() as d:   # the saved fields, written and read back
        path = os.path.join(d, "model.npz")
        np.savez(path, z=part["z"], alpha=part["alpha"], hyper=part["hyper"],
                 sweep=np.int64(part["sweep"]))
        st = np.load(path)
        resumed = _run(K, V, c, st["z"], st["alpha"], st["hyper"], int(st["sweep"]),
                       [25, 200, 0, 10, 0, 2, 0], seed)
    np.testing.assert_array_equal(resumed["z"], whole["z"])
    np.testing.assert_array_equal(resumed["rows"], whole["rows"])
    np.testing.assert_array_equal(resumed["tpt"], whole["tpt"])
    assert resumed["sweep"] == whole["sweep"] == 40
    o, *_ = _oracle_schedule(oracle, c, V, K, z0, alpha0, 6.0, 0.02, seed, 0, 40, 0, 200, 10, threads=2)
    np.testing.assert_array_equal(whole["z"], o.z())


def test_estimate_ending_between_statistics_and_optimisation(oracle):
    """An estimate() that ends after a statistics sweep but before the next
    optimisation (iterations 35: statistics at 15..35 every 5, optimisation at
    20 and 30), then a second estimate() of the same model.  Mallet 2.0.7's
    estimate() builds new WorkerRunnables and calls initializeAlphaStatistics
    on each, so the statistics of sweep 35 die with the first call's runnables
    and the second call starts its schedule (iteration 1.., burn-in again)
    with empty histograms; the oracle schedule restates exactly that."""
    c = synthetic_lda(num_docs=220, num_types=600, num_topics=12, doc_len=None, mean_len=45,
                      min_len=1, max_len=150, seed=19)
    V, K, seed = c.num_types, 16, 6
    rng = np.random.default_rng(12)
    z0 = rng.integers(0, K, c.num_tokens).astype(np.int32)
    alpha0 = np.full(K, 8.0 / K)
    hyper0 = np.array([8.0, 0.05, 0.05 * V])
    iters, interval, burnin, save = 35, 10, 10, 5
    out1 = _run(K, V, c, z0, alpha0, hyper0, 0, [iters, burnin, interval, save, 0, 2, 0], seed)
    o, alpha, alpha_sum, beta, ll = _oracle_schedule(oracle, c, V, K, z0, alpha0, 8.0, 0.05, seed, 0,
                                                     iters, interval, burnin, save, threads=2)
    _check(out1, o, alpha, alpha_sum, beta, ll, K, V, iters)
    iters2 = 20
    out2 = _run(K, V, c, out1["z"], out1["alpha"], out1["hyper"], out1["sweep"],
                [iters2, burnin, interval, save, 0, 2, 0], seed)
    o2, alpha2, alpha_sum2, beta2, ll2 = _oracle_schedule(
        oracle, c, V, K, out1["z"], out1["alpha"], out1["hyper"][0], out1["hyper"][1], seed,
        iters, iters2, interval, burnin, save, threads=2)
    _check(out2, o2, alpha2, alpha_sum2, beta2, ll2, K, V, iters2)
    assert out2["sweep"] == iters + iters2


def test_jni_glue_through_a_fake_jnienv_equals_the_harness():
    """integration/jni/lda_jni.c itself (tests/jni/fake_env.c: HotSpot-like
    copying arrays, every pin released exactly once, outputs copied back with
    mode 0 and inputs released with JNI_ABORT) gives the harness's z, alpha,
    hyper, sweep counter, packed rows, tokensPerTopic and LL trace bit for bit,
    at numThreads 4 with optimisation and at K > 1024."""
    for K, opts in ((20, [40, 10, 10, 10, 0, 4, 0]), (1500, [12, 200, 0, 10, 0, 1, 0])):
        c = synthetic_lda(num_docs=60, num_types=200, num_topics=20, doc_len=None, mean_len=30,
                          min_len=1, max_len=80, seed=K)
        rng = np.random.default_rng(K)
        z0 = rng.integers(0, K, size=c.num_tokens).astype(np.int32)
        alpha0 = np.full(K, 0.1)
        hyper0 = [0.1 * K, 0.01, 0.01 * c.num_types]
        a = _run(K, c.num_types, c, z0, alpha0, hyper0, 3, opts, 11)
        b = _run(K, c.num_types, c, z0, alpha0, hyper0, 3, opts, 11, prog=FAKE)
        for key in a:
            np.testing.assert_array_equal(np.asarray(a[key]), np.asarray(b[key]), err_msg=key)
