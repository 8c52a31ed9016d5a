"""GPU parity over randomly drawn configurations (seeded, so every run draws
the same 256 cases): the HIP sampler through the C ABI against cpu_exact,
bit-exact z, nw, nwsum and nd after every step.

The hand-written cases in test_parity_gpu.py pin one feature each; these mix
them the way a caller can: every kernel family (quarter-wave K <= 128, dense
C <= 16, sparse C <= 16, large-K C = 32 / 64), symmetric and asymmetric
alpha over three decades, beta over three, ragged corpora with empty and
long documents and one word holding a large share of the tokens, a global
token base above 2^32 (the Philox counters of a later shard), an initial z,
work-range sizes, split sweeps, the count-update modes, warm-start and
staleness (sequential) schedules, an alpha / beta change between sweeps,
and then inference (lda_infer: theta within 1e-12) on held-out documents
with random iteration, burn-in and thinning counts.  Each case is small
enough for the oracle to finish in about a second.
"""
import numpy as np
import pytest

from ldagibbssampling_amd.corpus import Corpus

CASES = 256
K_CHOICES = [2, 7, 20, 33, 64, 100, 128, 200, 300, 512, 777, 1024, 1100, 2048, 3000, 4096]


def _case(i):
    """The i-th configuration: (corpus, K, kind, alpha, beta, options)."""
    rng = np.random.default_rng(7_000_003 + 97 * i)
    K = int(K_CHOICES[i % len(K_CHOICES)])
    kind = "sparse" if K > 1024 else ("dense" if rng.random() < 0.6 else "sparse")
    D = int(rng.integers(1, 260))
    V = int(rng.integers(1, 2500))
    mean = float(rng.choice([3.0, 20.0, 80.0, 200.0]))
    lens = rng.poisson(mean, size=D)
    lens[rng.random(D) < 0.1] = 0                          # empty documents
    if D > 3 and rng.random() < 0.5:
        lens[int(rng.integers(0, D))] = int(rng.integers(300, 1500))   # a long document
    if lens.sum() == 0:
        lens[0] = 1
    off = np.zeros(D + 1, dtype=np.int64)
    np.cumsum(lens, out=off[1:])
    n = int(off[-1])
    p = 1.0 / np.arange(1, V + 1) ** float(rng.uniform(0.6, 1.4))
    p /= p.sum()
    words = rng.choice(V, size=n, p=p).astype(np.int32)
    if n and rng.random() < 0.3:
        words[rng.random(n) < float(rng.uniform(0.2, 0.7))] = int(rng.integers(0, V))   # a hot word
    corpus = Corpus(off, words, V)
    alpha_sum = float(10 ** rng.uniform(-1, 2))
    if rng.random() < 0.5:
        alpha = np.full(K, alpha_sum / K)
    else:
        a = rng.gamma(0.5, 1.0, size=K) + 1e-3
        alpha = a / a.sum() * alpha_sum
    beta = float(10 ** rng.uniform(-3, 0))
    opts = {
        "seed": int(rng.integers(0, 2**63)),
        "token_base": int(rng.choice([0, 0, 2**32 + int(rng.integers(0, 2**20)), int(rng.integers(0, 2**40))])),
        "tokens_per_range": int(rng.choice([0, 0, 16, 100, 512])),
        "z_init": rng.random() < 0.25,
        "parts": int(rng.choice([1, 1, 2, 3, 4])),
        "count": str(rng.choice(["auto", "delta", "recount"])) if kind == "dense" else "auto",
        "schedule": str(rng.choice(["snapshot", "snapshot", "warm", "staleness"])),
        "threads": int(rng.choice([2, 3, 4])),
        "sweeps": [int(x) for x in rng.integers(1, 4, size=2)],
        "rehyper": rng.random() < 0.4,
        "zseed": int(rng.integers(0, 2**31)),
        "infer": [int(rng.integers(1, 25)), int(rng.integers(0, 8)), int(rng.integers(1, 6))],
    }
    return corpus, K, kind, alpha, beta, opts


def _state_equal(g, o, what):
    np.testing.assert_array_equal(g.z(), o.z(), err_msg=what)
    gnw, gns, gnd, gds = g.counts(with_nd=True)
    onw, ons, ond, ods = o.counts(with_nd=True)
    np.testing.assert_array_equal(gnw, onw, err_msg=what)
    np.testing.assert_array_equal(gns, ons, err_msg=what)
    np.testing.assert_array_equal(gnd, ond, err_msg=what)
    np.testing.assert_array_equal(gds, ods, err_msg=what)


@pytest.mark.gpu
@pytest.mark.parametrize("i", range(CASES))
def test_random_configuration_bit_exact(oracle, i):
    from ldagibbssampling_amd.sampler import GibbsSampler
    corpus, K, kind, alpha, beta, o_ = _case(i)
    z0 = None
    if o_["z_init"] and corpus.num_tokens:
        z0 = np.random.default_rng(o_["zseed"]).integers(0, K, size=corpus.num_tokens).astype(np.int32)
    what = (f"case {i}: K={K} {kind} D={corpus.num_docs} N={corpus.num_tokens} V={corpus.num_types} "
            f"{ {k: v for k, v in o_.items() if k not in ('seed', 'zseed')} }")
    g = GibbsSampler(K, corpus.num_types, corpus.doc_off, corpus.words, alpha, beta, seed=o_["seed"],
                     z_init=z0, token_base=o_["token_base"], tokens_per_range=o_["tokens_per_range"],
                     sampler=kind)
    o = oracle.ExactSampler(K, corpus.num_types, corpus.doc_off, corpus.words, alpha, beta, o_["seed"],
                            z_init=z0, token_base=o_["token_base"], kind=kind)
    try:
        if o_["count"] != "auto":
            g.set_count_update(o_["count"])
        if o_["schedule"] == "snapshot":
            g.set_warm_start(1, 0)
            o.set_warm_start(1, 0)
            if o_["parts"] > 1:
                g.set_exchange_parts(o_["parts"])     # same sweep, split buffers
        elif o_["schedule"] == "warm":
            g.set_warm_start(max(o_["parts"], 2), 2)      # 2..LDA_MAX_EXCHANGE_PARTS parts
            o.set_warm_start(max(o_["parts"], 2), 2)
        else:
            parts, fr = oracle.staleness_schedule(o_["threads"])
            g.set_warm_start(2, 1)
            o.set_warm_start(2, 1)
            g.set_sequential_sweeps(parts, fr)
            o.set_sequential_sweeps(parts, fr)
        g.sweep(0)
        o.apply()
        _state_equal(g, o, what + " after init")
        n1, n2 = o_["sweeps"]
        g.sweep(n1)
        o.sweep(n1)
        _state_equal(g, o, what + f" after {n1} sweeps")
        if o_["rehyper"]:
            rng = np.random.default_rng(o_["zseed"] + 1)
            alpha2 = alpha * float(rng.uniform(0.5, 2.0))
            beta2 = beta * float(rng.uniform(0.5, 2.0))
            g.set_alpha_beta(alpha2, beta2)
            o.set_alpha_beta(alpha2, beta2)
        g.sweep(n2)
        o.sweep(n2)
        _state_equal(g, o, what + f" after {n1 + n2} sweeps")
        lg, lo = g.log_likelihood(), o.log_likelihood()
        assert abs(lg - lo) <= 1e-9 * max(abs(lo), 1.0), (what, lg, lo)
        # held-out documents: the first few of the corpus plus one of unseen
        # and out-of-range-free random types
        rng = np.random.default_rng(o_["zseed"] + 2)
        dh = min(corpus.num_docs, 12)
        hoff = np.concatenate([corpus.doc_off[:dh + 1], [corpus.doc_off[dh] + 17]]).astype(np.int64)
        hw = np.concatenate([corpus.words[:corpus.doc_off[dh]],
                             rng.integers(0, corpus.num_types, size=17)]).astype(np.int32)
        it, burn, thin = o_["infer"]
        burn = min(burn, it - 1)
        tg = g.infer(hoff, hw, n_iter=it, burn_in=burn, thin=thin, seed=o_["zseed"])
        to = o.infer(hoff, hw, n_iter=it, burn_in=burn, thin=thin, seed=o_["zseed"])
        np.testing.assert_allclose(tg, to, rtol=0, atol=1e-12, err_msg=what + " inference")
    finally:
        g.close()


def test_random_cases_cover_every_kernel_family():
    """The draw above reaches every sampler family and option at least once
    (checked on the CPU: the case list is data)."""
    seen = set()
    for i in range(CASES):
        corpus, K, kind, alpha, beta, o_ = _case(i)
        fam = ("big" if K > 1024 else "sparse" if kind == "sparse" else
               "quarter" if K <= 128 else "dense")
        seen.add(fam)
        seen.add(o_["schedule"])
        seen.add(o_["count"])
        if o_["token_base"] >= 2**32:
            seen.add("base>2^32")
        if o_["parts"] > 1 and o_["schedule"] == "snapshot":
            seen.add("split")
        if o_["z_init"]:
            seen.add("z_init")
        if o_["rehyper"]:
            seen.add("rehyper")
        if (np.diff(corpus.doc_off) == 0).any():
            seen.add("empty doc")
    want = {"big", "sparse", "quarter", "dense", "snapshot", "warm", "staleness", "auto", "delta",
            "recount", "base>2^32", "split", "z_init", "rehyper", "empty doc"}
    assert want <= seen, want - seen
