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

Escape lists at their used length (escape_lists="used", the default): each
rank's escape count is MAX-all-reduced first (4 bytes), every rank then
all-gathers only that many triples (none when no rank has one), and
lda_exchange_unpack_lists unpacks them; a count above the list capacity
(impossible while every shard holds at most max_tokens tokens) raises.
escape_lists="capacity" all-gathers the whole fixed-capacity lists (C4 at
N = 8: 2.9 MB per rank) without the count read.

Replica check (replica_check, bench.py's multi-GPU line): after the timed
region the ranks MIN- and MAX-all-reduce a hash of their nw / nwsum
(lda_counts_checksum) and the bits of the LL's word part; the replicas agree
when MIN == MAX.

Split sweeps (engine.exchange_parts > 1, lda_set_exchange_parts): the shard's
documents are sampled in P parts with one delta buffer each; part i's
all-reduce is issued asynchronously as soon as part i has been sampled, so it
runs while part i+1 samples, and only the last part's exchange is exposed.
The snapshot does not change inside a sweep, so this is the same sweep, bit
for bit, as the unsplit one (tests/test_distributed.py::*split*).
"""
from __future__ import annotations

import struct
from dataclasses import dataclass

import numpy as np


# the compact exchange's four-cells-per-word default starts at this padded K
# (the large-K sampler's C >= 32 tables)
LARGE_K_CELLS4 = 2048


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
                 time_reduce: bool = False, compact: bool = True, exchange=None,
                 escape_lists: str = "used", cells_per_word=None):
        """sync_before_reduce=False when the engine already launches on the
        stream the collective runs behind (GibbsSampler.set_stream(torch's
        current stream)): then no host synchronisation per sweep is needed.
        time_reduce: record CUDA events around every all-reduce on torch's
        current stream (reduce_ms reads them after a synchronize).
        exchange: run the collectives (default: with more than one rank);
        True on one rank puts the real backend's calls -- RCCL's in-place
        all-reduce on the library's buffers, the all-gather, the pack and
        unpack -- on the path of a one-GPU run, whose sums are then the
        identity (tests/test_distributed_gpu.py).
        escape_lists: "used" (all-gather the escape lists at their used
        length, after a MAX all-reduce of the counts) or "capacity" (the
        whole fixed-capacity lists).
        cells_per_word: cells per packed word of the compact exchange
        (lda_set_exchange_cells): 2 or 4; None picks 4 for the large-K
        sampler's tables (Kp >= LARGE_K_CELLS4, C5: 1.07 GB instead of 2.15 GB
        per exchange, ~1e5 escapes per rank per sweep at 8 ranks,
        profiles/r06/exchange/) when the lists travel at their used length,
        else 2 (C4: the narrower fields escape about as many bytes as they
        save)."""
        import torch.distributed as dist

        if escape_lists not in ("used", "capacity"):
            raise ValueError('escape_lists must be "used" or "capacity"')
        self.escape_lists = escape_lists
        self._sent = []            # list_cap all-gathered per exchanged buffer ("used")
        self._counts = None        # per-part escape counts, MAX-all-reduced ("used")
        self._host_counts = None   # their pinned host copies (GPU)
        self._count_events = {}    # part -> event recorded after its host copy

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
        if self.compact and hasattr(engine, "set_exchange_cells"):
            if cells_per_word is None:
                cells_per_word = 4 if (escape_lists == "used" and self.world <= 64 and
                                       int(getattr(engine, "Kp", 0)) >= LARGE_K_CELLS4) else 2
            engine.set_exchange_cells(int(cells_per_word))
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
        cap_bytes = 4 * n_es * self.world
        if self.escape_lists == "capacity":
            return {"allreduce_bytes": 4 * n_pk, "allgather_bytes": cap_bytes,
                    "allgather_capacity_bytes": cap_bytes, "escape_lists": "capacity"}
        # what the last exchanges (up to 256) gathered: 1 + 3 m int32 per rank
        # when m > 0 (m = the largest count of any rank), nothing when m = 0
        sent = self._sent or [0]
        gathered = [4 * self.world * (1 + 3 * m) if m > 0 else 0 for m in sent]
        return {"allreduce_bytes": 4 * n_pk + 4, "allgather_bytes": float(np.mean(gathered)),
                "allgather_capacity_bytes": cap_bytes, "escape_lists": "used",
                "escape_count_max": int(max(sent)), "exchanges_recorded": len(self._sent)}

    def _escapes_all(self, part: int, esc, n: int | None = None):
        """The all-gather target of part `part`: world x n int32 (n: the
        per-rank length sent, default len(esc)), a prefix of one buffer of
        the full capacity."""
        import torch
        n = esc.numel() if n is None else n
        buf = self._esc_all.get(part)
        # sized by what is gathered, not by the lists' capacity (with four
        # cells per word a C5 rank's capacity is 750 MB: world copies of it
        # would be 6 GB for lists that are normally short)
        if buf is None or buf.numel() < self.world * n or buf.device != esc.device:
            buf = torch.empty(self.world * n, dtype=esc.dtype, device=esc.device)
            self._esc_all[part] = buf
        return buf[:self.world * n]

    def _gather(self, part: int, esc, n: int, async_op: bool):
        """All-gather the first n int32 of every rank's escape list."""
        dist = self.dist
        send = esc[:n]
        esc_all = self._escapes_all(part, esc, n)
        if esc.device.type == "cuda" and dist.get_backend(self.group) == "nccl":
            w = dist.all_gather_into_tensor(esc_all, send, group=self.group, async_op=async_op)
        else:
            # gloo: a list of views of the one target array
            chunks = list(esc_all.view(self.world, -1).unbind(0))
            w = dist.all_gather(chunks, send, group=self.group, async_op=async_op)
        return esc_all, w

    def _count_slots(self, esc):
        import torch
        n = max(self.parts, 1)
        if self._counts is None or self._counts.numel() < n or self._counts.device != esc.device:
            self._counts = torch.zeros(n, dtype=torch.int32, device=esc.device)
        return self._counts

    def _exchange_start(self, part: int, async_op: bool):
        """Issue part `part`'s sum across the ranks; returns (works, pending):
        escape_lists "used": wait on pending.count_work (async), read the
        MAX-all-reduced escape counts on the host (_read_counts), and
        pending.gather(count) issues the lists' all-gather (more works).
        Then wait on the works and (with
        sync_before_reduce, after synchronizing torch's current stream)
        pending.finish() leaves the sum in the part's buffer.
        Compact: the pack is enqueued on the engine's stream, the collectives
        on torch's current one (the same stream when sync_before_reduce is
        off), and finish() enqueues the unpack on the engine's stream."""
        dist = self.dist
        if not self.compact:
            if self.sync_before_reduce:
                self.engine.synchronize()
            w = dist.all_reduce(self._part_delta(part), op=dist.ReduceOp.SUM, group=self.group,
                                async_op=async_op)
            return ([w] if async_op else []), _Pending()
        packed, esc = self.engine.exchange_pack(part, self.world, self.max_tokens)
        if self.sync_before_reduce:
            self.engine.synchronize()
        count_work = None
        if self.escape_lists == "used":
            # the count first: its all-reduce is done before the packed words'
            cnt = self._count_slots(esc)[part:part + 1]
            cnt.copy_(esc[:1])
            count_work = dist.all_reduce(cnt, op=dist.ReduceOp.MAX, group=self.group, async_op=True)
            if cnt.device.type == "cuda":
                # the count travels to pinned host memory behind its own
                # all-reduce only, before the packed words' all-reduce is
                # issued: the host's read (_read_counts) waits for this copy,
                # not for the packed sum, so it overlaps that collective and
                # leaves the GPU no gap (round 6)
                if count_work is not None:
                    count_work.wait()
                self._stage_count(part, cnt)
                count_work = None
        works = [dist.all_reduce(packed, op=dist.ReduceOp.SUM, group=self.group, async_op=async_op)]
        if self.escape_lists == "capacity":
            esc_all, w = self._gather(part, esc, esc.numel(), async_op)
            works.append(w)
            pend = _Pending(finish=lambda: self.engine.exchange_unpack(part, self.world, self.max_tokens,
                                                                       esc_all))
        else:
            pend = _Pending(self, part, esc)
            pend.count_work = count_work
        return ([w for w in works if w is not None] if async_op else []), pend

    def _stage_count(self, part: int, cnt):
        """Copy part `part`'s MAX-reduced count to pinned host memory on
        torch's current stream (ordered behind the count's all-reduce) and
        record the event _read_counts waits for."""
        import torch
        if self._host_counts is None or self._host_counts.numel() < max(self.parts, part + 1):
            self._host_counts = torch.zeros(max(self.parts, part + 1), dtype=torch.int32,
                                            pin_memory=True)
        self._host_counts[part:part + 1].copy_(cnt, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self._count_events[part] = ev

    def _read_counts(self, parts: int):
        """The MAX-all-reduced escape counts of the first `parts` parts.  On
        the GPU each count was staged to pinned memory right behind its own
        all-reduce (_stage_count): this waits for those copies only, while
        the packed all-reduces issued after them keep running, so the read
        costs the host a wait but the GPU no idle gap.  On the CPU (gloo) the
        caller has waited on the count all-reduces."""
        if self.escape_lists != "used" or not self.compact:
            return [0] * parts
        if getattr(self, "_count_events", None):
            for i in range(parts):
                self._count_events.pop(i).synchronize()
            cnt = [int(x) for x in self._host_counts[:parts].tolist()]
        else:
            cnt = [int(x) for x in self._counts[:parts].cpu().tolist()]
        _, n_es = self.engine.exchange_sizes(self.world, self.max_tokens)
        cap = (n_es - 1) // 3
        for m in cnt:
            if m > cap:
                raise RuntimeError(f"escape list overflow: {m} escapes, capacity {cap} "
                                   f"(a shard holds more than max_tokens = {self.max_tokens} tokens?)")
        self._sent = (self._sent + cnt)[-256:]
        return cnt

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
            _, pend = self._exchange_start(0, async_op=False)
            if pend.count_work is not None:
                pend.count_work.wait()
            for w in pend.gather(self._read_counts(1)[0], async_op=False):
                w.wait()
            self._landed()
            pend.finish()
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
            w, pend = self._exchange_start(i, async_op=True)
            works += w
            finishers.append(pend)
        if self.compact and self.escape_lists == "used":
            # every part's escape lists at their used length: one host read of
            # the parts' MAX-reduced counts (the count all-reduces were issued
            # ahead of each part's packed all-reduce)
            for pend in finishers:
                if pend.count_work is not None:
                    pend.count_work.wait()
            for pend, m in zip(finishers, self._read_counts(parts)):
                works += pend.gather(m, async_op=True)
        for w in works:
            w.wait()           # the current stream waits for every part's sum
        self._landed()
        for pend in finishers:
            pend.finish()
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

    def replica_check(self, seconds: float | None = None) -> dict:
        """After the timed region: every rank's replica of nw / nwsum and the
        LL's word part (computed from them) must be identical.  MIN and MAX
        all-reduces of (counts hash, word-part bits, total-LL bits); a SUM of
        ones counts the ranks the collective reached; `seconds` (this rank's
        timed-region time) is all-gathered into rank_seconds."""
        import torch

        h = int(self.engine.counts_checksum()) if hasattr(self.engine, "counts_checksum") else 0
        doc, word = self.engine.log_likelihood_parts()
        total = self.log_likelihood()

        def bits(x):
            return struct.unpack("<q", struct.pack("<d", float(x)))[0]

        signed = h - (1 << 64) if h >= 1 << 63 else h
        vals = [signed, bits(word), bits(total)]
        out = {"world_size": self.world, "counts_checksum": f"{h:016x}", "ll_word_part": word,
               "ll": total}
        if not self.exchange:
            out.update(replicas_agree=True, ranks_counted=1,
                       rank_seconds=[seconds] if seconds is not None else None)
            return out
        dist = self.dist
        dev = self._collective_device()
        lo = torch.tensor(vals, dtype=torch.int64, device=dev)
        hi = lo.clone()
        dist.all_reduce(lo, op=dist.ReduceOp.MIN, group=self.group)
        dist.all_reduce(hi, op=dist.ReduceOp.MAX, group=self.group)
        one = torch.ones(1, dtype=torch.int64, device=dev)
        dist.all_reduce(one, op=dist.ReduceOp.SUM, group=self.group)
        lo, hi = lo.cpu().tolist(), hi.cpu().tolist()
        out.update(replicas_agree=bool(lo == hi), ranks_counted=int(one.item()),
                   checksum_min=f"{lo[0] & ((1 << 64) - 1):016x}",
                   checksum_max=f"{hi[0] & ((1 << 64) - 1):016x}")
        if seconds is not None:
            t = torch.tensor([float(seconds)], dtype=torch.float64, device=dev)
            ts = [torch.zeros_like(t) for _ in range(self.world)]
            dist.all_gather(ts, t, group=self.group)
            out["rank_seconds"] = [float(x.item()) for x in ts]
        return out

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


class _Pending:
    """One exchanged buffer between its collectives and its unpack (see
    ADLDATrainer._exchange_start)."""

    def __init__(self, trainer=None, part=0, esc=None, finish=None):
        self.trainer, self.part, self.esc = trainer, part, esc
        self._finish = finish
        self._esc_all, self._m = None, 0
        self.count_work = None

    def gather(self, m: int, async_op: bool = False):
        """escape_lists "used": all-gather 1 + 3 m int32 of every rank's list
        (nothing when m = 0); returns the works to wait on."""
        if self.trainer is None or self._finish is not None:
            return []
        self._m = int(m)
        if self._m == 0:
            return []
        self._esc_all, w = self.trainer._gather(self.part, self.esc, 1 + 3 * self._m, async_op)
        return [w] if (async_op and w is not None) else []

    def finish(self):
        if self._finish is not None:
            self._finish()
        elif self.trainer is not None:
            t = self.trainer
            t.engine.exchange_unpack(self.part, t.world, t.max_tokens, self._esc_all, list_cap=self._m)
