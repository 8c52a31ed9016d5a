"""Multi-rank AD-LDA on CPU (gloo, world_size 2 and 3): the product driver
(ldagibbssampling_amd.distributed) with the cpu_exact oracle injected as the
engine must reproduce the single-process run bit for bit."""
import os
import sys
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

K, SEED, SWEEPS = 32, 17, 3


class OracleEngine:
    """cpu_exact behind the engine interface ADLDATrainer drives (tests only)."""

    def __init__(self, sampler):
        self.s = sampler

    def sample(self):
        self.s.sample()

    def apply(self):
        self.s.apply()

    def synchronize(self):
        pass

    def delta_tensor(self):
        return torch.from_numpy(self.s.delta())

    def log_likelihood_parts(self):
        return self.s.log_likelihood_parts()

    # the compact exchange (lda_exchange_pack / _unpack) restated in numpy;
    # cells: lda_set_exchange_cells (2 or 4 cells per packed word)
    cells = 2

    @property
    def N(self):
        return self.s.N

    def _buf(self, part):
        return self.s.delta()

    def exchange_sizes(self, world, max_tokens):
        from oracle import oracle as O
        return (self.s.V * self.s.Kp // self.cells + self.s.Kp,
                1 + 3 * O.exchange_cap(world, max_tokens, self.cells))

    def exchange_pack(self, part, world, max_tokens):
        from oracle import oracle as O
        pk, es = O.exchange_pack(self._buf(part), world, self.s.Kp, max_tokens, cells=self.cells)
        self._packed = getattr(self, "_packed", {})
        self._packed[part] = torch.from_numpy(pk)
        return self._packed[part], torch.from_numpy(es)

    def exchange_unpack(self, part, world, max_tokens, escapes_all, list_cap=None):
        from oracle import oracle as O
        self.unpacked_lists = getattr(self, "unpacked_lists", []) + [list_cap]
        self._buf(part)[:] = O.exchange_unpack(self._packed[part].numpy(),
                                               None if escapes_all is None else escapes_all.numpy(), world,
                                               self.s.Kp, max_tokens, list_cap=list_cap, cells=self.cells)

    def counts_checksum(self):
        from oracle import oracle as O
        nw, nwsum, _, _ = self.s.counts()
        return O.counts_checksum(nw, nwsum)


class SplitOracleEngine(OracleEngine):
    """cpu_exact behind the split-sweep engine interface (lda_sample_part /
    lda_delta_buffer_part): part i's changes land in buffer i, which the
    trainer all-reduces asynchronously while part i+1 samples."""

    def __init__(self, sampler, parts):
        super().__init__(sampler)
        self.exchange_parts = parts
        off = sampler.doc_off
        n = int(off[-1] - off[0])
        self.cuts = [0] + [int(np.searchsorted(off, off[0] + n * (i + 1) // parts, side="left"))
                           for i in range(parts - 1)] + [sampler.D]
        scratch = sampler.delta()
        self.bufs = [np.zeros_like(scratch) for _ in range(parts)]
        self.bufs[0][:] = scratch      # the shard's initial counts (pending at create)
        scratch[:] = 0
        self.next = 0

    def sample(self):
        for i in range(self.exchange_parts):
            self.sample_part(i)

    def sample_part(self, i):
        assert i == self.next
        scratch = self.s.delta()
        self.s.sample_docs(self.cuts[i], self.cuts[i + 1])
        self.bufs[i][:] = scratch
        scratch[:] = 0
        self.next = (i + 1) % self.exchange_parts
        if self.next == 0:
            self.s.end_sweep()

    def apply(self):
        scratch = self.s.delta()
        for b in self.bufs:
            scratch += b
            b[:] = 0
        self.s.apply()

    def delta_tensor(self, part=0):
        return torch.from_numpy(self.bufs[part])

    def _buf(self, part):
        return self.bufs[part]


class WarmOracleEngine(OracleEngine):
    """cpu_exact with the warm start (lda_set_warm_start): the sampler ABI's
    sweep_parts / sample_part protocol of a sequential sweep."""

    def sweep_parts(self):
        runs = self.s._sweep_runs()
        return (len(runs), True) if runs is not None else (1, False)

    def sample_part(self, i):
        runs = self.s._sweep_runs()
        for d0, d1 in runs[i]:
            self.s.sample_docs(d0, d1)
        if i + 1 == len(runs):
            self.s.end_sweep()


def _corpus():
    from ldagibbssampling_amd.corpus import synthetic_lda
    return synthetic_lda(num_docs=70, num_types=300, num_topics=K, doc_len=None, mean_len=40,
                         min_len=0, max_len=150, seed=13)


WARM = (3, 2)          # sweeps 0 and 1 in 3 sequential parts


def _hot_corpus():
    """Half the tokens are one word whose tokens start in topics 0 and 1: the
    first exchange (the initial counts) has cells beyond both biases, so
    escape lists travel (test_gloo_escape_lists)."""
    rng = np.random.default_rng(5)
    D, L = 480, 150
    words = rng.integers(1, 200, size=D * L).astype(np.int32)
    hot = rng.random(D * L) < 0.5
    words[hot] = 0
    z0 = rng.integers(0, K, size=D * L).astype(np.int32)
    z0[hot] = rng.integers(0, 2, size=int(hot.sum()))
    return np.arange(D + 1, dtype=np.int64) * L, words, z0, 200


def _worker(rank, world, port, outdir, parts=1, compact=True, escape_lists="used", corpus="plain", cells=2):
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import oracle as O
    from ldagibbssampling_amd.distributed import ADLDATrainer, shard_corpus
    if corpus == "hot":
        doc_off, words, z0, V = _hot_corpus()
    else:
        c = _corpus()
        doc_off, words, z0, V = c.doc_off, c.words, None, c.num_types
    sh = shard_corpus(doc_off, words, world, rank)
    o = O.ExactSampler(K, V, sh.doc_off, sh.words, 0.1, 0.01, SEED, token_base=sh.token_base,
                       z_init=None if z0 is None else z0[sh.token_base:sh.token_base + len(sh.words)])
    if parts in ("warm", "steady"):
        o.set_warm_start(*WARM, 0, len(words))          # parts cut in the whole corpus
        if parts == "steady":                           # + Mallet-staleness sweeps after it
            o.set_sequential_sweeps(*O.staleness_schedule(4), 0, len(words))
        eng = WarmOracleEngine(o)
    else:
        eng = OracleEngine(o) if parts == 1 else SplitOracleEngine(o, parts)
    eng.cells = cells
    if corpus == "corrupt" and rank == world - 1:
        eng.counts_checksum = lambda: 12345             # a replica that differs
    tr = ADLDATrainer(eng, compact=compact, escape_lists=escape_lists)
    if parts not in ("warm", "steady"):
        assert tr.parts == parts
    assert tr.compact == compact
    tr.sweep(SWEEPS)
    ll = tr.log_likelihood()
    chk = tr.replica_check(seconds=0.5 + rank)
    nw, nwsum, _, _ = o.counts()
    np.savez(os.path.join(outdir, f"r{rank}.npz"), z=o.z(), nw=nw, nwsum=nwsum, ll=ll,
             docs=np.array([sh.doc_begin, sh.doc_end]), agree=chk["replicas_agree"],
             ranks=chk["ranks_counted"], world=chk["world_size"], secs=np.array(chk["rank_seconds"]),
             checksum=chk["counts_checksum"], lists=np.array([-1 if x is None else x for x in
                                                               getattr(eng, "unpacked_lists", [])]),
             xb=str(tr.exchange_bytes()))
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world,parts,compact", [(2, 1, True), (3, 1, True), (2, 3, True), (3, 2, True),
                                                 (2, "warm", True), (3, "warm", True), (3, "steady", True),
                                                 (2, "steady", False), (2, 1, False),
                                                 (3, 2, False)])
def test_gloo_adlda_matches_single(oracle, world, parts, compact):
    """parts > 1: split sweeps, every part's all-reduce overlapping the next
    part's sampling (async gloo collectives) -- the same result bit for bit.
    "warm": the warm start (sequential parts cut in the whole corpus, each
    part summed and applied before the next) against one context's.
    compact: the packed exchange (two cells per int32 word + escape lists);
    False: the int32 buffers."""
    res = _run(world, parts, compact)
    c = _corpus()
    single = oracle.ExactSampler(K, c.num_types, c.doc_off, c.words, 0.1, 0.01, SEED)
    if parts in ("warm", "steady"):
        single.set_warm_start(*WARM)
    if parts == "steady":
        single.set_sequential_sweeps(*oracle.staleness_schedule(4))
    single.sweep(SWEEPS)
    np.testing.assert_array_equal(np.concatenate([r["z"] for r in res]), single.z())
    nw, nwsum, _, _ = single.counts()
    for r in res:
        np.testing.assert_array_equal(r["nw"], nw)       # every replica identical
        np.testing.assert_array_equal(r["nwsum"], nwsum)
        assert abs(float(r["ll"]) - single.log_likelihood()) < 1e-9 * abs(single.log_likelihood())
    spans = [tuple(r["docs"]) for r in res]
    assert spans[0][0] == 0 and spans[-1][1] == c.num_docs
    assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
    # the replica check bench.py prints: every rank agrees, on the hash of the
    # counts the oracle restates, over all `world` ranks
    for r in res:
        assert bool(r["agree"]) and int(r["ranks"]) == world and int(r["world"]) == world
        assert str(r["checksum"]) == f"{oracle.counts_checksum(nw, nwsum):016x}"
        np.testing.assert_array_equal(r["secs"], 0.5 + np.arange(world))


def _run(world, parts=1, compact=True, escape_lists="used", corpus="plain", cells=2):
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_worker, args=(world, _free_port(), d, parts, compact, escape_lists, corpus, cells),
                           nprocs=world, start_method="spawn")
        return [dict(np.load(os.path.join(d, f"r{r}.npz"))) for r in range(world)]


@pytest.mark.parametrize("world,parts,escape_lists,cells", [(2, 1, "used", 2), (3, 1, "used", 2),
                                                            (3, 2, "used", 2), (2, 1, "capacity", 2),
                                                            (2, 1, "used", 4), (3, 2, "used", 4),
                                                            (3, "steady", "used", 4)])
def test_gloo_escape_lists(oracle, world, parts, escape_lists, cells):
    """A corpus whose first exchange has escapes (cells beyond 2^14/world):
    "used" all-gathers the lists at the MAX-reduced count (lda_exchange_
    unpack_lists; list_cap 0 without escapes, when nothing is gathered),
    "capacity" the whole lists; both give the single-process run.  cells 4:
    four 8-bit cells per packed word (lda_set_exchange_cells), whose narrow
    fields send escapes in later sweeps too."""
    res = _run(world, parts, True, escape_lists, "hot", cells)
    doc_off, words, z0, V = _hot_corpus()
    single = oracle.ExactSampler(K, V, doc_off, words, 0.1, 0.01, SEED, z_init=z0)
    if parts == "steady":
        single.set_warm_start(*WARM)
        single.set_sequential_sweeps(*oracle.staleness_schedule(4))
    single.sweep(SWEEPS)
    np.testing.assert_array_equal(np.concatenate([r["z"] for r in res]), single.z())
    nw, nwsum, _, _ = single.counts()
    for r in res:
        np.testing.assert_array_equal(r["nw"], nw)
        np.testing.assert_array_equal(r["nwsum"], nwsum)
        assert bool(r["agree"])
        lists = r["lists"]
        if escape_lists == "used" and cells == 2:
            assert lists[0] >= 1                     # the initial counts' escapes, at their count
            assert (lists[1:] == 0).all()            # later deltas: none, nothing gathered
            assert "'escape_lists': 'used'" in str(r["xb"])
        elif escape_lists == "used":
            assert lists[0] >= 1 and (lists[1:] >= 0).all()
            assert "'escape_lists': 'used'" in str(r["xb"])
        else:
            assert (lists == -1).all()


def test_replica_check_flags_a_differing_replica():
    res = _run(2, corpus="corrupt")
    assert not any(bool(r["agree"]) for r in res)


def test_escape_count_above_capacity_raises():
    """A count beyond the list capacity (the bound's premise broken) stops
    the exchange instead of unpacking a truncated list."""
    from ldagibbssampling_amd.distributed import ADLDATrainer

    class Fake:
        def exchange_sizes(self, world, max_tokens):
            return 8, 1 + 3 * 4

    tr = ADLDATrainer.__new__(ADLDATrainer)
    tr.escape_lists, tr.compact, tr.world, tr.max_tokens, tr._sent = "used", True, 2, 100, []
    tr.engine = Fake()
    tr._counts = torch.tensor([5], dtype=torch.int32)
    with pytest.raises(RuntimeError, match="escape list overflow"):
        tr._read_counts(1)
    tr._counts = torch.tensor([4], dtype=torch.int32)
    assert tr._read_counts(1) == [4]


def test_shard_balanced_by_tokens():
    from ldagibbssampling_amd.distributed import shard_corpus
    c = _corpus()
    world = 4
    shards = [shard_corpus(c.doc_off, c.words, world, r) for r in range(world)]
    assert shards[0].doc_begin == 0 and shards[-1].doc_end == c.num_docs
    toks = [len(s.words) for s in shards]
    assert sum(toks) == c.num_tokens
    assert max(toks) - min(toks) <= 200                    # within ~one doc
    assert [s.token_base for s in shards] == list(np.cumsum([0] + toks[:-1]))


@pytest.mark.parametrize("world", [2, 3, 8, 16])
def test_compact_exchange_roundtrip_with_escapes(world):
    """The packed exchange restated in numpy (oracle.exchange_pack / _unpack,
    the checker of lda_exchange_pack): summing `world` ranks' packed words
    plus their escape lists gives the int32 sum, bit for bit, with cells at
    and beyond the biases (escapes), at both halves of a word, negative and
    positive, and the nwsum tail; each rank's escapes stay within the bound
    2 N / b1 when its |cells| sum to at most 2 N."""
    from oracle import oracle as O
    rng = np.random.default_rng(world)
    Kp, V = 64, 40
    cells = V * Kp
    b0, b1 = O.exchange_biases(world)
    bufs = []
    for r in range(world):
        b = np.zeros(cells + Kp, dtype=np.int64)
        idx = rng.choice(cells, size=300, replace=False)
        b[idx] = rng.integers(-3, 4, size=300)
        # boundary and escape values in both halves
        for v in (b0 - 1, -b0, b0, -b0 - 1, b1 - 1, -b1, b1, -b1 - 1, 3 * b0):
            b[rng.integers(cells)] = v
        b[cells:] = rng.integers(-50, 50, size=Kp)
        bufs.append(b.astype(np.int32))
    # the escape bound's premise: a rank's |cells| sum to at most 2 N (N: the
    # largest shard's tokens)
    N = max(int(np.abs(b[:cells].astype(np.int64)).sum()) for b in bufs) // 2 + 1
    packed, escs = zip(*(O.exchange_pack(b, world, Kp, N) for b in bufs))
    psum = np.sum(np.stack([p.astype(np.int64) for p in packed]), axis=0)
    assert psum.max() < 2 ** 31                 # no int32 overflow in the collective
    out = O.exchange_unpack(psum.astype(np.int32), np.concatenate(escs), world, Kp, N)
    np.testing.assert_array_equal(out, np.sum(np.stack(bufs).astype(np.int64), axis=0).astype(np.int32))
    assert all(int(e[0]) <= O.exchange_cap(world, N) for e in escs)
    assert sum(int(e[0]) for e in escs) >= 1
