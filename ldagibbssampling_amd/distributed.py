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
                 time_reduce: bool = False):
        """sync_before_reduce=False when the engine already launches on the
        stream the collective runs behind (GibbsSampler.set_stream(torch's
        current stream)): then no host synchronisation per sweep is needed.
        time_reduce: record CUDA events around every all-reduce on torch's
        current stream (reduce_ms reads them after a synchronize)."""
        import torch.distributed as dist

        self.engine = engine
        self.time_reduce = time_reduce
        self._events = []
        self.sync_before_reduce = sync_before_reduce
        self.group = group
        self.dist = dist
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self._delta = engine.delta_tensor() if self.world > 1 else None
        self._part_deltas = {}
        self._initialised = False
        if self.world > 1 and not sync_before_reduce:
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

    def _reduce(self):
        if self.world > 1:
            if self.sync_before_reduce:
                self.engine.synchronize()
            ev = None
            if self.time_reduce and self._delta.device.type == "cuda":
                import torch
                ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                ev[0].record()
            self.dist.all_reduce(self._delta, op=self.dist.ReduceOp.SUM, group=self.group)
            if ev is not None:
                ev[1].record()
                self._events = (self._events + [ev])[-256:]
            if self.sync_before_reduce and self._delta.device.type == "cuda":
                # RCCL returns once the collective is enqueued (torch's current
                # stream waits for it, the engine's own stream does not): the
                # apply that follows must not read the delta before the sum
                # has landed
                import torch
                torch.cuda.current_stream(self._delta.device).synchronize()

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
        if self.world < 2 or not hasattr(self.engine, "count_update"):
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
        """One sweep in `parts` parts, part i's all-reduce overlapping part
        i+1's sampling (async collectives; the engine's stream or, in the
        default mode, a host sync orders each collective behind its part)."""
        dist = self.dist
        on_cuda = self._delta.device.type == "cuda"
        works = []
        ev = None
        for i in range(parts):
            self.engine.sample_part(i)
            if self.sync_before_reduce:
                self.engine.synchronize()
            if i == parts - 1 and self.time_reduce and on_cuda:
                import torch
                ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                ev[0].record()
            works.append(dist.all_reduce(self._part_delta(i), op=dist.ReduceOp.SUM,
                                         group=self.group, async_op=True))
        for w in works:
            w.wait()           # the current stream waits for every part's sum
        if ev is not None:
            ev[1].record()      # exposed exchange: the last part's collective
            self._events = (self._events + [ev])[-256:]
        if self.sync_before_reduce and on_cuda:
            import torch
            torch.cuda.current_stream(self._delta.device).synchronize()

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
            if self.world < 2:
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
        if self.world > 1:
            dev = self._delta.device if self.dist.get_backend(self.group) == "nccl" else "cpu"
            t = torch.tensor([doc], dtype=torch.float64, device=dev)
            self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM, group=self.group)
            doc = float(t.item())
        return doc + word
