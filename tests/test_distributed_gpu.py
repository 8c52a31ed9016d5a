"""Two ranks on one MI355X (gloo over device tensors): the product engine
(GibbsSampler) + ADLDATrainer must equal the single-process GPU run and the
oracle bit for bit.  (RCCL needs one GPU per rank; the 8-GPU RCCL path is
exercised by bench.py under torch.distributed.run.)"""
import os
import sys
import tempfile

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
K, SEED, SWEEPS = 128, 23, 4


def _corpus():
    from ldagibbssampling_amd.corpus import synthetic_lda
    return synthetic_lda(num_docs=160, num_types=900, num_topics=K, doc_len=None, mean_len=70,
                         min_len=0, max_len=300, seed=31)


def _worker(rank, world, port, outdir, stream_ordered=False, parts=1):
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from ldagibbssampling_amd.distributed import ADLDATrainer, shard_corpus
    from ldagibbssampling_amd.sampler import GibbsSampler
    c = _corpus()
    sh = shard_corpus(c.doc_off, c.words, world, rank)
    g = GibbsSampler(K, c.num_types, sh.doc_off, sh.words, 0.1, 0.01, seed=SEED,
                     token_base=sh.token_base)
    if parts > 1:
        g.set_exchange_parts(parts, reserve_cus=8)    # split sweeps, async collectives
    if stream_ordered:
        # bench.py's arrangement: sampler and collective on one torch stream, no host sync
        st = torch.cuda.Stream()
        torch.cuda.set_stream(st)
        g.set_stream(st.cuda_stream)
        tr = ADLDATrainer(g, sync_before_reduce=False)
        # the default stream is refused (handle 0 would not order the collective)
        torch.cuda.set_stream(torch.cuda.default_stream())
        try:
            ADLDATrainer(g, sync_before_reduce=False)
            raise AssertionError("default stream accepted")
        except ValueError:
            pass
        torch.cuda.set_stream(st)
    else:
        tr = ADLDATrainer(g)
    tr.sweep(SWEEPS)
    ll = tr.log_likelihood()
    chk = tr.replica_check(seconds=1.0 + rank)
    nw, nwsum, _, _ = g.counts()
    np.savez(os.path.join(outdir, f"r{rank}.npz"), z=g.z(), nw=nw, nwsum=nwsum, ll=ll,
             agree=chk["replicas_agree"], ranks=chk["ranks_counted"], checksum=chk["counts_checksum"],
             secs=np.array(chk["rank_seconds"]))
    g.close()
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("stream_ordered,parts", [(False, 1), (True, 1), (False, 3), (True, 2)])
def test_two_ranks_one_gpu(oracle, stream_ordered, parts):
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    world = 2
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_worker, args=(world, port, d, stream_ordered, parts), nprocs=world,
                           start_method="spawn")
        res = [np.load(os.path.join(d, f"r{r}.npz")) for r in range(world)]
    c = _corpus()
    o = oracle.ExactSampler(K, c.num_types, c.doc_off, c.words, 0.1, 0.01, SEED)
    o.sweep(SWEEPS)
    np.testing.assert_array_equal(np.concatenate([r["z"] for r in res]), o.z())
    nw, nwsum, _, _ = o.counts()
    for r in res:
        np.testing.assert_array_equal(r["nw"], nw)
        np.testing.assert_array_equal(r["nwsum"], nwsum)
        assert abs(float(r["ll"]) - o.log_likelihood()) < 1e-9 * abs(o.log_likelihood())
        # the replica check of bench.py's multi-GPU line (lda_counts_checksum)
        assert bool(r["agree"]) and int(r["ranks"]) == world
        assert str(r["checksum"]) == f"{oracle.counts_checksum(nw, nwsum):016x}"
        np.testing.assert_array_equal(r["secs"], [1.0, 2.0])


class _SlowCollective:
    """Stands in for torch.distributed with the nccl backend's stream
    semantics: the "all-reduce" runs on a side stream (RCCL's own) after a
    delay and adds a marker; torch's current stream waits for it, the host
    does not."""

    def __init__(self, marker_cells, twice=False):
        self.marker_cells = marker_cells
        self.twice = twice

    class ReduceOp:
        SUM = "sum"
        MIN = "min"
        MAX = "max"

    def get_backend(self, group=None):
        return "nccl"

    def all_reduce(self, t, op=None, group=None, async_op=False):
        import torch
        if op in (self.ReduceOp.MIN, self.ReduceOp.MAX):
            return                                   # one real rank: the extreme is its own value
        cur = torch.cuda.current_stream(t.device)
        side = torch.cuda.Stream(device=t.device)
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            torch.cuda._sleep(200_000_000)            # ~0.1 s of spinning
            if self.twice:
                t.mul_(2)                             # two identical ranks
            for i in self.marker_cells:
                t[i] += 7
        cur.wait_stream(side)

    def all_gather_into_tensor(self, out, t, group=None, async_op=False):
        import torch
        cur = torch.cuda.current_stream(t.device)
        side = torch.cuda.Stream(device=t.device)
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            torch.cuda._sleep(100_000_000)
            out.view(2, -1).copy_(t.view(1, -1).expand(2, -1))
        cur.wait_stream(side)


@pytest.mark.parametrize("compact", [False, True])
def test_default_mode_waits_for_async_collective(compact):
    """ADLDATrainer's default mode (engine on its own stream): the apply after
    an all-reduce that returns before the collective has landed must still
    see the reduced delta (the RCCL/apply race).  compact: the
    packed exchange, whose unpack runs on the engine's stream after the
    collectives (two identical "ranks": the sum is twice the counts)."""
    from ldagibbssampling_amd.corpus import synthetic_lda
    from ldagibbssampling_amd.distributed import ADLDATrainer
    from ldagibbssampling_amd.sampler import GibbsSampler
    c = synthetic_lda(num_docs=50, num_types=300, num_topics=16, doc_len=None, mean_len=40,
                      min_len=1, max_len=100, seed=2)
    g = GibbsSampler(16, c.num_types, c.doc_off, c.words, 0.1, 0.01, seed=4)
    ref = GibbsSampler(16, c.num_types, c.doc_off, c.words, 0.1, 0.01, seed=4)
    ref.sweep(0)
    tr = ADLDATrainer(g)                       # default: sync_before_reduce=True
    tr.world, tr.exchange = 2, True            # as if sharded: reduce, then apply
    tr._delta = g.delta_tensor()
    Kp = g.Kp
    if compact:
        tr.compact, tr.max_tokens = True, g.N
        # packed word 0 (nw[0][0] in its low half) and the packed nwsum tail
        tr.dist = _SlowCollective([0, c.num_types * Kp // 2], twice=True)
    else:
        tr.dist = _SlowCollective([0, c.num_types * Kp])   # nw[0][0] and nwsum[0]
    tr.init_counts()
    nw, nwsum, _, _ = g.counts()
    rnw, rnwsum, _, _ = ref.counts()
    if compact:
        rnw, rnwsum = 2 * rnw, 2 * rnwsum
    assert nw[0, 0] == rnw[0, 0] + 7 and nwsum[0] == rnwsum[0] + 7
    nw[0, 0] -= 7
    nwsum[0] -= 7
    np.testing.assert_array_equal(nw, rnw)
    np.testing.assert_array_equal(nwsum, rnwsum)
    g.synchronize()
    assert int(g.delta_tensor().abs().sum()) == 0      # nothing landed after the apply


def _rccl_worker(rank, port, outdir, stream_ordered, parts, compact, k=None, kind="dense"):
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    from ldagibbssampling_amd.distributed import ADLDATrainer
    from ldagibbssampling_amd.sampler import GibbsSampler
    c = _corpus()
    g = GibbsSampler(k or K, c.num_types, c.doc_off, c.words, 0.1, 0.01, seed=SEED, sampler=kind)
    if parts > 1:
        g.set_exchange_parts(parts, reserve_cus=8)
    if stream_ordered:
        st = torch.cuda.Stream()
        torch.cuda.set_stream(st)
        g.set_stream(st.cuda_stream)
    tr = ADLDATrainer(g, sync_before_reduce=not stream_ordered, compact=compact, exchange=True,
                      time_reduce=True)
    assert tr.exchange and tr.compact == compact
    tr.sweep(SWEEPS)
    ll = tr.log_likelihood()
    torch.cuda.synchronize()
    assert tr.reduce_ms(SWEEPS) is not None          # the collectives ran
    chk = tr.replica_check(seconds=0.25)
    assert chk["replicas_agree"] and chk["ranks_counted"] == 1 and chk["rank_seconds"] == [0.25]
    nw, nwsum, _, _ = g.counts()
    np.savez(os.path.join(outdir, "r0.npz"), z=g.z(), nw=nw, nwsum=nwsum, ll=ll,
             bytes=tr.exchange_bytes()["allreduce_bytes"], cells=g.exchange_cells, kp=g.Kp)
    g.close()
    dist.destroy_process_group()


@pytest.mark.parametrize("stream_ordered,parts,compact,k,kind", [
    (True, 1, True, None, "dense"), (False, 1, True, None, "dense"), (True, 2, True, None, "dense"),
    (True, 1, False, None, "dense"), (True, 1, True, 2048, "sparse"), (True, 2, True, 2048, "sparse")])
def test_rccl_exchange_one_rank(oracle, stream_ordered, parts, compact, k, kind):
    """The RCCL path bench.py takes at N > 1 (torch.distributed "nccl"),
    exercised on the one-GPU box with one rank and the exchange forced on:
    process-group init on the device, the in-place SUM all-reduce of the
    library's packed (or int32) buffer, the all-gather of the escape lists,
    the pack / unpack kernels, stream-ordered and host-synchronised, split
    sweeps.  One rank's sum is the identity, so the chain must equal the
    oracle bit for bit -- a wrong stream order, size or dtype at the RCCL
    boundary shows up as a difference.  k = 2048 (the large-K sampler): the
    trainer's default exchange packs four cells per word."""
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_rccl_worker, args=(port, d, stream_ordered, parts, compact, k, kind), nprocs=1,
                           start_method="spawn")
        r = np.load(os.path.join(d, "r0.npz"))
    c = _corpus()
    o = oracle.ExactSampler(k or K, c.num_types, c.doc_off, c.words, 0.1, 0.01, SEED,
                            kind="sparse" if kind == "sparse" else "dense")
    o.sweep(SWEEPS)
    np.testing.assert_array_equal(r["z"], o.z())
    nw, nwsum, _, _ = o.counts()
    np.testing.assert_array_equal(r["nw"], nw)
    np.testing.assert_array_equal(r["nwsum"], nwsum)
    assert abs(float(r["ll"]) - o.log_likelihood()) < 1e-9 * abs(o.log_likelihood())
    kp = int(r["kp"])
    vk = c.num_types * kp
    cells = int(r["cells"])
    assert cells == (4 if kp >= 2048 else 2)
    # compact: two (four) nw cells per int32 word, the nwsum part as raw
    # int32, and the escape count's 4-byte MAX all-reduce
    assert int(r["bytes"]) == (4 * (vk // cells + kp) + 4 if compact else 4 * (vk + kp))
