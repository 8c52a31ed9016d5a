"""Parity at BASELINE.json's full single-GPU sizes, through properties that
hold at any size (the oracle cannot sweep 2.5e8 tokens in seconds; the
bit-exact oracle comparisons run at small sizes in test_parity_gpu.py):

- conservation: sum(nw) == N, nwsum == the column sums of nw, z in [0, K);
- the counts equal a recount of z (word-topic histogram on the GPU);
- determinism: a second context with the same seed reproduces z bit for bit;
- sharding invariance: two shards (global token_base, summed deltas) == one
  context, z bit for bit (AD-LDA's all-reduce, here on one GPU);
- the model log likelihood is finite and rises from the random init.

Workloads: the C4 shard (1.25M docs x 200 tokens, V = 100k, K = 512, dense
sampler: the bench's headline) and the C5 shard (V = 262144, K = 4096,
large-K sparse sampler), corpora drawn as bench.py draws them.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _corpus(docs, V, K):
    from ldagibbssampling_amd.corpus import synthetic_lda_torch
    return synthetic_lda_torch(docs, V, K, doc_len=200, seed=20261015, device="cuda:0")


def _recount(words, z, V, K):
    import torch
    w = torch.as_tensor(words, device="cuda:0").long()
    zt = torch.as_tensor(z, device="cuda:0").long()
    return torch.bincount(w * K + zt, minlength=V * K).reshape(V, K)


def _sweeps(kind, docs, V, K, sweeps):
    import torch
    from ldagibbssampling_amd.sampler import GibbsSampler
    c = _corpus(docs, V, K)
    N = c.num_tokens
    alpha = np.full(K, 0.1)
    g = GibbsSampler(K, V, c.doc_off, c.words, alpha, 0.01, seed=5, sampler=kind)
    g.sweep(0)
    ll0 = g.log_likelihood()
    g.sweep(sweeps)
    z = g.z()
    assert z.min() >= 0 and z.max() < K
    nw, nwsum, _, _ = g.counts()
    assert int(nw.sum(dtype=np.int64)) == N
    np.testing.assert_array_equal(nw.sum(0, dtype=np.int64), nwsum.astype(np.int64))
    rc = _recount(c.words, z, V, K)
    assert torch.equal(rc, torch.as_tensor(nw, device="cuda:0").long())
    del rc, nw
    ll1 = g.log_likelihood()
    assert np.isfinite(ll0) and np.isfinite(ll1) and ll1 > ll0
    g.close()

    # determinism: same seed, a fresh context
    g2 = GibbsSampler(K, V, c.doc_off, c.words, alpha, 0.01, seed=5, sampler=kind)
    g2.sweep(sweeps)
    np.testing.assert_array_equal(g2.z(), z)
    g2.close()

    # sharding invariance: two shards with their global token offsets and the
    # deltas summed between the sample and the apply of every sweep
    cut = c.num_docs // 2
    off = c.doc_off
    shards = [GibbsSampler(K, V, off[a:b + 1], c.words[off[a]:off[b]], alpha, 0.01, seed=5,
                           token_base=int(off[a]), sampler=kind)
              for a, b in ((0, cut), (cut, c.num_docs))]

    def allreduce():
        for s in shards:
            s.synchronize()
        ts = [s.delta_tensor() for s in shards]
        tot = ts[0] + ts[1]
        for t in ts:
            t.copy_(tot)
        torch.cuda.synchronize()

    allreduce()
    for s in shards:
        s.apply()
    for _ in range(sweeps):
        for s in shards:
            s.sample()
        allreduce()
        for s in shards:
            s.apply()
    np.testing.assert_array_equal(np.concatenate([s.z() for s in shards]), z)
    for s in shards:
        s.close()


def test_c4_shard_dense_full_size():
    _sweeps("dense", 1_250_000, 100_000, 512, sweeps=3)


def test_c5_shard_large_k_sparse_full_size():
    _sweeps("sparse", 1_250_000, 262_144, 4096, sweeps=2)
