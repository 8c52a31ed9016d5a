"""AD-LDA across GPUs: one process per GPU, documents sharded, nw replicated.

The reference's only parallelism is Mallet's document-parallel worker
threads (setNumThreads(4) at src/cmu_ron/TrainAndPredict.java:164 and
src/cmu/TrainAndPredict.java:262): contiguous doc blocks per thread, and after
every sweep the per-thread counts are summed into the global typeTopicCounts
/ tokensPerTopic and copied back (ParallelTopicModel.sumTypeTopicCounts).
Here that exchange is an in-place SUM all-reduce of the int32 delta buffer
[V*Kp nw delta | Kp nwsum delta] over the process group (RCCL over xGMI for
the "nccl" backend; gloo for CPU tests).  Integer sums commute and every draw
is keyed by the GLOBAL token index, so the result is bit-identical for any
number of ranks (tests/test_distributed.py).

Compact exchange (default, compact=True): instead of the int32
buffer the ranks sum packed words, two cells per int32 (lda_exchange_pack:
cell 2i biased by 2^15/world in the low half, cell 2i+1 by 2^14/world in the
high half, so the sum cannot carry between them), and all-gather short
escape lists for the cells whose change is out of that range; the unpack
gives the int32 sum bit for bit at half the bytes (C4: 102 MB instead of
205 MB per sweep, C5: 2.15 GB instead of 4.3 GB).

Split sweeps (engine.exchange_parts > 1, lda_set_exchange_parts): the shard's
documents are sampled in P parts with one delta buffer each; part i's
all-reduce is issued asynchronously as soon as part i has been sampled, so it
runs while part i+1 samples, and only the last part's exchange is exposed.
The snapshot does not change inside a sweep, so this is the same sweep, bit
for bit, as the unsplit one (tests/test_distributed.py::*split*).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np


@dataclass
class Shard:
    rank: int
    world: int
    doc_begin: int
    doc_end: int
    doc_off: np.ndarray   # int64 [docs+1], absolute offsets into the corpus stream
    words: np.ndarray     # int32 [tokens]
    token_base: int       # global index of the shard's first token


def shard_corpus(doc_off, words, world: int, rank: int) -> Shard:
    """Contiguous document ranges balanced by token count (the GPU analogue of
    Mallet's docsPerThread blocks, balanced on tokens instead of documents)."""
    doc_off = np.asarray(doc_off, dtype=np.int64)
    D = len(doc_off) - 1
    total = int(doc_off[-1] - doc_off[0])
    targets = [doc_off[0] + (total * r) // world for r in range(world + 1)]
    cuts = [0] + [int(np.searchsorted(doc_off, t, side="left")) for t in targets[1:-1]] + [D]
    cuts = [min(max(c, 0), D) for c in cuts]
    for i in range(1, len(cuts)):
        cuts[i] = max(cuts[i], cuts[i - 1])
    a, b = cuts[rank], cuts[rank + 1]
    off = doc_off[a:b + 1]
    return Shard(rank, world, a, b, off, np.asarray(words[off[0]:off[-1]], dtype=np.int32),
                 int(off[0] - doc_off[0]))


class ADLDATrainer:
    """Drives one rank's sampler engine through AD-LDA sweeps.

    engine: sample(), apply(), delta_tensor() -> torch int32 tensor aliasing
    the engine's pending delta, synchronize(), log_likelihood_parts().
    GibbsSampler (GPU) is the product engine; tests inject a CPU one.
    """

    def __init__(self, engine, group=None, sync_before_reduce: bool = True,
                 time_reduce: bool = False, compact: bool = True, exchange=None):
        """sync_before_reduce=False when the engine already launches on the
        stream the collective runs behind (GibbsSampler.set_stream(torch's
        current stream)): then no host synchronisation per sweep is needed.
        time_reduce: record CUDA events around every all-reduce on torch's
        current stream (reduce_ms reads them after a synchronize).
        exchange: run the collectives (default: with more than one rank);
        True on one rank puts the real backend's calls -- RCCL's in-place
        all-reduce on the library's buffers, the all-gather, the pack and
        unpack -- on the path of a one-GPU run, whose sums are then the
        identity (tests/test_distributed_gpu.py)."""
        import torch.distributed as dist

        self.engine = engine
        self.time_reduce = time_reduce
        self._events = []
        self.sync_before_reduce = sync_before_reduce
        self.group = group
        self.dist = dist
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.exchange = self.world > 1 if exchange is None else bool(exchange and dist.is_initialized())
        self._delta = engine.delta_tensor() if self.exchange else None
        self._part_deltas = {}
        self._initialised = False
        # the compact exchange needs engine.exchange_pack / exchange_unpack and
        # the largest shard's tokens (every rank sizes its escape list alike)
        self.compact = bool(compact and self.exchange and hasattr(engine, "exchange_pack"))
        self._esc_all = {}
        self.max_tokens = self._max_tokens() if self.compact else 0
        if self.exchange and not sync_before_reduce:
            self._check_stream_order()

    def _check_stream_order(self):
        """Without a host sync the collective is ordered behind the sampler
        only if both run on torch's current stream, and that stream is a real
        one (handle 0 would make lda_set_stream pick the context's own)."""
        import torch
        if not hasattr(self.engine, "stream_handle") or self._delta is None or \
                self._delta.device.type != "cuda":
            return
        cur = torch.cuda.current_stream(self._delta.device).cuda_stream
        if cur == 0 or self.engine.stream_handle() != cur:
            raise ValueError("sync_before_reduce=False needs the engine on torch's current, "
                             "non-default stream: torch.cuda.set_stream(s); "
                             "engine.set_stream(s.cuda_stream)")

    def _collective_device(self):
        backend = getattr(self.dist, "get_backend", None)
        if backend is not None and backend(self.group) != "nccl":
            return "cpu"
        return self._delta.device

    def _max_tokens(self) -> int:
        import torch
        t = torch.tensor([int(self.engine.N)], dtype=torch.int64, device=self._collective_device())
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX, group=self.group)
        return int(t.item())

    def exchange_bytes(self) -> dict:
        """Bytes one rank hands to the collectives per exchanged buffer: the
        all-reduced message and the all-gathered escape lists (world copies)."""
        cells = int(self._delta.numel())
        if not self.compact:
            return {"allreduce_bytes": 4 * cells, "allgather_bytes": 0}
        n_pk, n_es = self.engine.exchange_sizes(self.world, self.max_tokens)
        return {"allreduce_bytes": 4 * n_pk, "allgather_bytes": 4 * n_es * self.world}

    def _escapes_all(self, part: int, esc):
        """The all-gather target of part `part`: world x len(esc) int32."""
        import torch
        buf = self._esc_all.get(part)
        if buf is None or buf.numel() != self.world * esc.numel() or buf.device != esc.device:
            buf = torch.empty(self.world * esc.numel(), dtype=esc.dtype, device=esc.device)
            self._esc_all[part] = buf
        return buf

    def _exchange_start(self, part: int, async_op: bool):
        """Issue part `part`'s sum across the ranks; returns (works, finish):
        wait on the works (and, with sync_before_reduce, synchronize torch's
        current stream), then finish() leaves the sum in the part's buffer.
        Compact: the pack is enqueued on the engine's stream, the collectives
        on torch's current one (the same stream when sync_before_reduce is
        off), and finish() enqueues the unpack on the engine's stream."""
        dist = self.dist
        if not self.compact:
            if self.sync_before_reduce:
                self.engine.synchronize()
            w = dist.all_reduce(self._part_delta(part), op=dist.ReduceOp.SUM, group=self.group,
                                async_op=async_op)
            return ([w] if async_op else []), (lambda: None)
        packed, esc = self.engine.exchange_pack(part, self.world, self.max_tokens)
        esc_all = self._escapes_all(part, esc)
        if self.sync_before_reduce:
            self.engine.synchronize()
        works = [dist.all_reduce(packed, op=dist.ReduceOp.SUM, group=self.group, async_op=async_op)]
        if esc.device.type == "cuda" and dist.get_backend(self.group) == "nccl":
            works.append(dist.all_gather_into_tensor(esc_all, esc, group=self.group, async_op=async_op))
        else:
            # gloo: a list of views of the one target array
            chunks = list(esc_all.view(self.world, -1).unbind(0))
            works.append(dist.all_gather(chunks, esc, group=self.group, async_op=async_op))

        def finish():
            self.engine.exchange_unpack(part, self.world, self.max_tokens, esc_all)
        return ([w for w in works if w is not None] if async_op else []), finish

    def _landed(self):
        """With sync_before_reduce the engine's stream is not ordered behind
        the collective (RCCL returns once it is enqueued; torch's current
        stream waits for it): wait on the host before the engine reads the
        sum."""
        if self.sync_before_reduce and self._delta.device.type == "cuda":
            import torch
            torch.cuda.current_stream(self._delta.device).synchronize()

    def _reduce(self):
        if self.exchange:
            ev = None
            if self.time_reduce and self._delta.device.type == "cuda":
                import torch
                ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                ev[0].record()
            _, finish = self._exchange_start(0, async_op=False)
            self._landed()
            finish()
            if ev is not None:
                ev[1].record()
                self._events = (self._events + [ev])[-256:]

    def reduce_ms(self, last: int):
        """Mean duration (ms, CUDA events on torch's stream) of the last `last`
        all-reduces (time_reduce=True; None when none were recorded).  In a
        split sweep this is the exposed part: from the last part's collective
        being issued to every part's sum having landed."""
        evs = self._events[-last:] if last > 0 else []
        if not evs:
            return None
        evs[-1][1].synchronize()
        return sum(a.elapsed_time(b) for a, b in evs) / len(evs)

    def _agree_count_update(self):
        """Every rank must recount or keep a delta in the same sweeps (the
        buffers they sum hold counts or changes accordingly): the same mode,
        and for AUTO the smallest recount_sweeps of any rank."""
        if not self.exchange or not hasattr(self.engine, "count_update"):
            return
        import torch
        from . import capi
        mode, r = self.engine.count_update()
        backend = getattr(self.dist, "get_backend", None)
        dev = "cpu" if backend is not None and backend(self.group) != "nccl" else self._delta.device
        t = torch.tensor([capi.COUNT_UPDATE[mode], -capi.COUNT_UPDATE[mode], r], dtype=torch.int64,
                         device=dev)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MIN, group=self.group)
        lo, hi, rmin = int(t[0]), -int(t[1]), int(t[2])
        if lo != hi:
            raise ValueError("ranks disagree on the count-update mode (lda_set_count_update)")
        if mode == "auto" and rmin != r:
            self.engine.set_count_update("auto", rmin)

    def init_counts(self):
        """Global nw/nwsum from every rank's local counts (addInstances)."""
        self._agree_count_update()
        self._reduce()
        self.engine.apply()
        self._initialised = True

    @property
    def parts(self) -> int:
        return int(getattr(self.engine, "exchange_parts", 1) or 1)

    def _split_sweep(self, parts: int):
        """One sweep in `parts` parts, part i's exchange overlapping part
        i+1's sampling (async collectives; the engine's stream or, in the
        default mode, a host sync orders each collective behind its part)."""
        on_cuda = self._delta.device.type == "cuda"
        works, finishers = [], []
        ev = None
        for i in range(parts):
            self.engine.sample_part(i)
            if i == parts - 1 and self.time_reduce and on_cuda:
                import torch
                ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                ev[0].record()
            w, fin = self._exchange_start(i, async_op=True)
            works += w
            finishers.append(fin)
        for w in works:
            w.wait()           # the current stream waits for every part's sum
        self._landed()
        for fin in finishers:
            fin()
        if ev is not None:
            ev[1].record()      # exposed exchange: the last part's collective (+ unpacks)
            self._events = (self._events + [ev])[-256:]

    def _part_delta(self, i: int):
        """Tensor view of part i's buffer, re-made whenever the engine's buffer
        moved (lda_set_exchange_parts frees and reallocates part buffers when
        the part count changes: a stale view would reduce freed memory)."""
        if i == 0:
            return self._delta
        key = self.engine.delta_buffer(i)[0] if hasattr(self.engine, "delta_buffer") else None
        cached = self._part_deltas.get(i)
        if cached is None or key is None or cached[0] != key:
            cached = (key, self.engine.delta_tensor(i))
            self._part_deltas[i] = cached
        return cached[1]

    def _sequential_sweep(self, parts: int):
        """A warm-start sweep (lda_set_warm_start): each part sampled, its
        changes (always buffer 0) summed across ranks and applied before the
        next part samples."""
        for i in range(parts):
            self.engine.sample_part(i)
            self._reduce()
            self.engine.apply()

    def sweep(self, n: int = 1):
        if not self._initialised:
            self.init_counts()
        for _ in range(n):
            parts, seq = (self.engine.sweep_parts() if hasattr(self.engine, "sweep_parts")
                          else (self.parts, False))
            if seq:
                self._sequential_sweep(parts)
                continue
            if not self.exchange:
                self.engine.sample()
            elif parts > 1:
                self._split_sweep(parts)
            else:
                self.engine.sample()
                self._reduce()
            self.engine.apply()

    def log_likelihood(self) -> float:
        """modelLogLikelihood of the whole corpus: doc parts summed over ranks,
        the word part (global counts) taken once."""
        import torch

        doc, word = self.engine.log_likelihood_parts()
        if self.exchange:
            dev = self._delta.device if self.dist.get_backend(self.group) == "nccl" else "cpu"
            t = torch.tensor([doc], dtype=torch.float64, device=dev)
            self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM, group=self.group)
            doc = float(t.item())
        return doc + word
