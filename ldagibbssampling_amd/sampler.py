"""GibbsSampler: one document shard on one MI355X, driven through the C ABI.

This is the thin host object over ``lda_ctx`` (include/lda_mi355x.h).  It is
what ParallelTopicModel.estimate() (topic_model.py) and the AD-LDA driver
(distributed.py) run; it has no CPU path — every call goes to
liblda_mi355x.so and raises LdaError on failure.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import capi


def staleness_schedule(threads: int):
    """lda_staleness_schedule: (parts, fractions) of the sequential sweeps that
    give every token the mean live fraction of Mallet's `threads` worker
    threads (the native ParallelTopicModel's default schedule
    past the warm start, what the Java drop-in runs)."""
    L = capi.load()
    parts = C.c_int32()
    fr = np.zeros(capi.MAX_EXCHANGE_PARTS, dtype=np.float64)
    capi.check(L.lda_staleness_schedule(int(threads), C.byref(parts), fr.ctypes.data),
               "lda_staleness_schedule")
    return int(parts.value), fr[:parts.value].copy()


class _DeviceArray:
    """Exposes a device pointer through __cuda_array_interface__ (zero-copy
    torch.as_tensor view of the delta buffer for torch.distributed)."""

    def __init__(self, ptr: int, count: int, typestr: str = "<i4"):
        self.__cuda_array_interface__ = {
            "shape": (count,),
            "typestr": typestr,
            "data": (ptr, False),
            "version": 3,
            "strides": None,
        }


class GibbsSampler:
    def __init__(self, num_topics: int, num_types: int, doc_off, words, alpha, beta: float,
                 seed: int = 0, z_init=None, device: int = 0, token_base: int = 0,
                 tokens_per_range: int = 0, sampler: str = "dense"):
        L = capi.load()
        self.K = int(num_topics)
        self.V = int(num_types)
        doc_off = np.ascontiguousarray(doc_off, dtype=np.int64)
        words = np.ascontiguousarray(words, dtype=np.int32)
        if len(doc_off) < 1:
            raise ValueError("doc_off needs at least one entry")
        self.D = len(doc_off) - 1
        self.N = int(doc_off[-1] - doc_off[0])
        if len(words) < self.N:
            raise ValueError(f"words holds {len(words)} ids, doc_off spans {self.N}")
        if z_init is not None and len(z_init) != self.N:
            raise ValueError(f"z_init must hold {self.N} topics")
        alpha = np.ascontiguousarray(np.broadcast_to(np.asarray(alpha, dtype=np.float64), (self.K,)))
        self._alpha = alpha
        cfg = capi.lda_config()
        cfg.num_topics = self.K
        cfg.num_types = self.V
        cfg.num_docs = self.D
        cfg.alpha = alpha.ctypes.data_as(C.POINTER(C.c_double))
        cfg.beta = float(beta)
        cfg.seed = int(seed) & (2**64 - 1)
        cfg.device = int(device)
        cfg.sampler = capi.SAMPLERS[sampler]
        self.sampler_kind = sampler
        cfg.token_base = int(token_base)
        cfg.tokens_per_range = int(tokens_per_range)
        zp = None
        if z_init is not None:
            self._z_init = np.ascontiguousarray(z_init, dtype=np.int32)
            zp = self._z_init.ctypes.data
        h = C.c_void_p()
        capi.check(L.lda_create(C.byref(h), C.byref(cfg), doc_off,
                                words.ctypes.data if self.N else None, zp), "lda_create")
        self._h = h
        self._L = L
        self.device = int(device)
        kp = C.c_int32()
        capi.check(L.lda_get_shape(h, None, C.byref(kp), None, None, None), "lda_get_shape")
        self.Kp = kp.value
        self.beta = float(beta)

    # ---------------------------------------------------------------- life
    def close(self):
        h = getattr(self, "_h", None)
        if h:
            self._L.lda_destroy(h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    # --------------------------------------------------------------- sweeps
    def sweep(self, n: int = 1):
        capi.check(self._L.lda_sweep(self._h, int(n)), "lda_sweep")

    def sample(self):
        capi.check(self._L.lda_sample(self._h), "lda_sample")

    def apply(self):
        capi.check(self._L.lda_apply(self._h), "lda_apply")

    def delta_buffer(self, part: int = 0):
        ptr, cnt = C.c_void_p(), C.c_size_t()
        capi.check(self._L.lda_delta_buffer_part(self._h, int(part), C.byref(ptr), C.byref(cnt)),
                   "lda_delta_buffer_part")
        return int(ptr.value), int(cnt.value)

    def delta_tensor(self, part: int = 0):
        """Zero-copy torch int32 view of the pending delta of split-sweep part
        `part` (device memory; part 0 is lda_delta_buffer)."""
        import torch

        ptr, cnt = self.delta_buffer(part)
        t = torch.as_tensor(_DeviceArray(ptr, cnt), device=f"cuda:{self.device}")
        assert t.data_ptr() == ptr and t.dtype == torch.int32
        return t

    # ------------------------------------------------ compact exchange (§5)
    def exchange_sizes(self, world: int, max_tokens: int):
        """(packed int32 words, escape-list int32 words) of lda_exchange_pack."""
        a, b = C.c_size_t(), C.c_size_t()
        capi.check(self._L.lda_exchange_sizes(self._h, int(world), int(max_tokens), C.byref(a),
                                              C.byref(b)), "lda_exchange_sizes")
        return int(a.value), int(b.value)

    def set_exchange_cells(self, cells_per_word: int):
        """lda_set_exchange_cells: 2 (default) or 4 cells per packed exchange
        word (half the bytes, narrower fields, more escapes)."""
        capi.check(self._L.lda_set_exchange_cells(self._h, int(cells_per_word)), "lda_set_exchange_cells")

    @property
    def exchange_cells(self) -> int:
        n = C.c_int32()
        capi.check(self._L.lda_get_exchange_cells(self._h, C.byref(n)), "lda_get_exchange_cells")
        return int(n.value)

    def exchange_pack(self, part: int, world: int, max_tokens: int):
        """Pack part `part`'s exchange buffer (lda_exchange_pack, on this
        context's stream): zero-copy torch int32 views (packed words to
        SUM-all-reduce, this rank's escape list to all-gather)."""
        import torch
        pk, es = C.c_void_p(), C.c_void_p()
        capi.check(self._L.lda_exchange_pack(self._h, int(part), int(world), int(max_tokens),
                                             C.byref(pk), C.byref(es)), "lda_exchange_pack")
        n_pk, n_es = self.exchange_sizes(world, max_tokens)
        dev = f"cuda:{self.device}"
        return (torch.as_tensor(_DeviceArray(int(pk.value), n_pk), device=dev),
                torch.as_tensor(_DeviceArray(int(es.value), n_es), device=dev))

    def exchange_unpack(self, part: int, world: int, max_tokens: int, escapes_all, list_cap=None):
        """lda_exchange_unpack: the part's buffer = the summed packed words +
        every rank's escapes (escapes_all: device int32 [world x escape len]).
        list_cap: the lists were all-gathered at 1 + 3 list_cap int32 each
        (lda_exchange_unpack_lists; 0 with escapes_all None: no rank had one)."""
        if list_cap is None:
            assert escapes_all.dtype.itemsize == 4 and escapes_all.is_contiguous()
            capi.check(self._L.lda_exchange_unpack(self._h, int(part), int(world), int(max_tokens),
                                                   C.c_void_p(escapes_all.data_ptr())),
                       "lda_exchange_unpack")
            return
        ptr = None
        if escapes_all is not None:
            assert escapes_all.dtype.itemsize == 4 and escapes_all.is_contiguous()
            assert escapes_all.numel() == world * (1 + 3 * int(list_cap))
            ptr = C.c_void_p(escapes_all.data_ptr())
        capi.check(self._L.lda_exchange_unpack_lists(self._h, int(part), int(world), int(max_tokens), ptr,
                                                     int(list_cap)), "lda_exchange_unpack_lists")

    # ------------------------------------------------- split sweep (§5)
    def set_exchange_parts(self, parts: int, reserve_cus: int = 0):
        """Cut each sweep into `parts` token-balanced parts with their own delta
        buffers, so one part's all-reduce can overlap the next part's sampling
        (lda_set_exchange_parts)."""
        capi.check(self._L.lda_set_exchange_parts(self._h, int(parts), int(reserve_cus)),
                   "lda_set_exchange_parts")

    @property
    def exchange_parts(self) -> int:
        n = C.c_int32()
        capi.check(self._L.lda_get_exchange_parts(self._h, C.byref(n)), "lda_get_exchange_parts")
        return n.value

    def sample_part(self, part: int):
        capi.check(self._L.lda_sample_part(self._h, int(part)), "lda_sample_part")

    def set_stream(self, stream_handle: int | None):
        capi.check(self._L.lda_set_stream(self._h, stream_handle), "lda_set_stream")

    def stream_handle(self) -> int:
        """The hipStream_t every call of this context is ordered on."""
        h = C.c_void_p()
        capi.check(self._L.lda_get_stream(self._h, C.byref(h)), "lda_get_stream")
        return int(h.value or 0)

    def synchronize(self):
        capi.check(self._L.lda_synchronize(self._h), "lda_synchronize")

    @property
    def sweep_index(self) -> int:
        s = C.c_uint32()
        capi.check(self._L.lda_get_sweep(self._h, C.byref(s)), "lda_get_sweep")
        return s.value

    @sweep_index.setter
    def sweep_index(self, v: int):
        capi.check(self._L.lda_set_sweep(self._h, int(v)), "lda_set_sweep")

    def last_sample_ms(self) -> float:
        ms = C.c_float()
        capi.check(self._L.lda_last_sample_ms(self._h, C.byref(ms)), "lda_last_sample_ms")
        return float(ms.value)

    def sample_times(self, last: int) -> np.ndarray:
        """Kernel durations (ms) of the last `last` lda_sample launches."""
        ms = np.zeros(max(int(last), 0), dtype=np.float32)
        n = C.c_int32()
        capi.check(self._L.lda_sample_times(self._h, len(ms), ms.ctypes.data if len(ms) else None,
                                            C.byref(n)), "lda_sample_times")
        return ms[:n.value]

    def recount_times(self, last: int) -> np.ndarray:
        """Kernel durations (ms) of the recount after each of the last `last`
        lda_sample launches (zeros in the delta mode)."""
        ms = np.zeros(max(int(last), 0), dtype=np.float32)
        n = C.c_int32()
        capi.check(self._L.lda_recount_times(self._h, len(ms), ms.ctypes.data if len(ms) else None,
                                             C.byref(n)), "lda_recount_times")
        return ms[:n.value]

    def set_warm_start(self, parts: int = 4, sweeps: int = 50, corpus_first_token: int = 0,
                       corpus_tokens: int = 0):
        """lda_set_warm_start: sweeps whose sweep counter is below `sweeps` run in
        `parts` sequential parts (parts = 1: off), cut in the whole corpus of
        global tokens [corpus_first_token, + corpus_tokens) (0: this shard)."""
        capi.check(self._L.lda_set_warm_start(self._h, int(parts), int(sweeps), int(corpus_first_token),
                                              int(corpus_tokens)), "lda_set_warm_start")

    def set_sequential_sweeps(self, parts: int = 1, fractions=None, corpus_first_token: int = 0,
                              corpus_tokens: int = 0):
        """lda_set_sequential_sweeps: every sweep past the warm start in `parts`
        sequential parts, part i the fraction fractions[i] of every block
        (None: equal parts; parts = 1: plain snapshot sweeps)."""
        fr = None
        if parts > 1 and fractions is not None:
            self._seq_fr = np.ascontiguousarray(fractions, dtype=np.float64)
            assert self._seq_fr.shape == (parts,)
            fr = self._seq_fr.ctypes.data
        capi.check(self._L.lda_set_sequential_sweeps(self._h, int(parts), fr, int(corpus_first_token),
                                                     int(corpus_tokens)), "lda_set_sequential_sweeps")

    def sequential_sweeps(self):
        """(parts, cumulative cuts in units of 1/LDA_SEQ_FRACTION_UNIT)."""
        n = C.c_int32()
        cum = np.zeros(capi.MAX_EXCHANGE_PARTS + 1, dtype=np.int64)
        capi.check(self._L.lda_get_sequential_sweeps(self._h, C.byref(n), cum.ctypes.data),
                   "lda_get_sequential_sweeps")
        return int(n.value), cum[:n.value + 1].tolist()

    def sweep_parts(self):
        """(parts, sequential) of the sweep in progress or the next one."""
        p, q = C.c_int32(), C.c_int32()
        capi.check(self._L.lda_sweep_parts(self._h, C.byref(p), C.byref(q)), "lda_sweep_parts")
        return p.value, bool(q.value)

    def set_count_update(self, mode: str = "auto", recount_sweeps: int = -1):
        """Which sweeps recount (lda_set_count_update): "auto" (the first
        `recount_sweeps` sweeps after the counts are seeded; -1 keeps the
        library's choice), "recount" (all) or "delta" (none)."""
        capi.check(self._L.lda_set_count_update(self._h, capi.COUNT_UPDATE[mode], int(recount_sweeps)),
                   "lda_set_count_update")

    def count_update(self):
        """(mode name, recount_sweeps)."""
        m, r = C.c_int32(), C.c_int32()
        capi.check(self._L.lda_get_count_update(self._h, C.byref(m), C.byref(r)), "lda_get_count_update")
        return {v: k for k, v in capi.COUNT_UPDATE.items()}[m.value], r.value

    @property
    def recount(self) -> bool:
        """True when the exchange buffer holds recounted counts (dense samplers),
        False when it holds a delta (lda_count_update_mode)."""
        r = C.c_int32()
        capi.check(self._L.lda_count_update_mode(self._h, C.byref(r)), "lda_count_update_mode")
        return bool(r.value)

    # ---------------------------------------------------------------- state
    def z(self) -> np.ndarray:
        out = np.empty(self.N, dtype=np.int32)
        capi.check(self._L.lda_get_z(self._h, out), "lda_get_z")
        return out

    def set_z(self, z):
        z = np.ascontiguousarray(z, dtype=np.int32)
        if z.shape != (self.N,):
            raise ValueError(f"z must hold {self.N} topics, got shape {z.shape}")
        capi.check(self._L.lda_set_z(self._h, z), "lda_set_z")

    def counts(self, with_nd: bool = False):
        nw = np.empty((self.V, self.K), dtype=np.int32)
        nwsum = np.empty(self.K, dtype=np.int32)
        nd = np.empty((self.D, self.K), dtype=np.int32) if with_nd else None
        ndsum = np.empty(self.D, dtype=np.int32)
        capi.check(self._L.lda_get_counts(self._h, nw.ctypes.data, nwsum.ctypes.data,
                                          nd.ctypes.data if with_nd else None,
                                          ndsum.ctypes.data), "lda_get_counts")
        return nw, nwsum, nd, ndsum

    def counts_checksum(self) -> int:
        """lda_counts_checksum: a hash of the applied nw / nwsum (equal on every
        replica; oracle.counts_checksum of counts()'s nw, nwsum)."""
        h = C.c_uint64()
        capi.check(self._L.lda_counts_checksum(self._h, C.byref(h)), "lda_counts_checksum")
        return int(h.value)

    def set_alpha_beta(self, alpha, beta: float):
        a = np.ascontiguousarray(np.broadcast_to(np.asarray(alpha, dtype=np.float64), (self.K,)))
        capi.check(self._L.lda_set_alpha_beta(self._h, a, float(beta)), "lda_set_alpha_beta")
        self._alpha = a
        self.beta = float(beta)

    @property
    def alpha(self) -> np.ndarray:
        return self._alpha.copy()

    def log_likelihood_parts(self):
        a, b = C.c_double(), C.c_double()
        capi.check(self._L.lda_log_likelihood_parts(self._h, C.byref(a), C.byref(b)),
                   "lda_log_likelihood_parts")
        return a.value, b.value

    def log_likelihood(self) -> float:
        out = C.c_double()
        capi.check(self._L.lda_log_likelihood(self._h, C.byref(out)), "lda_log_likelihood")
        return out.value

    def infer(self, doc_off, words, n_iter: int = 100, thin: int = 10, burn_in: int = 10,
              seed: int = 0) -> np.ndarray:
        """TopicInferencer.getSampledDistribution(inst, numIterations, thinning,
        burnIn) over a batch of documents (positional order as Mallet's)."""
        doc_off = np.ascontiguousarray(doc_off, dtype=np.int64)
        words = np.ascontiguousarray(words, dtype=np.int32)
        if len(doc_off) < 1:
            raise ValueError("doc_off needs at least one entry")
        if len(words) < int(doc_off[-1] - doc_off[0]):
            raise ValueError("words is shorter than doc_off says")
        Dh = len(doc_off) - 1
        theta = np.zeros((Dh, self.K), dtype=np.float64)
        capi.check(self._L.lda_infer(self._h, Dh, doc_off, words, int(n_iter), int(thin),
                                     int(burn_in), int(seed) & (2**64 - 1), theta), "lda_infer")
        return theta

    # ------------------------------------------- hyperparameter statistics
    def max_doc_length(self) -> int:
        m = C.c_int32()
        capi.check(self._L.lda_max_doc_length(self._h, C.byref(m)), "lda_max_doc_length")
        return m.value

    def doc_topic_histograms(self, doc_len_counts=None, topic_doc_counts=None, max_len=None):
        """Add this shard's (docLengthCounts, topicDocCounts) from the current z
        into the given int32 arrays (allocated when None) and return them."""
        if max_len is None:
            max_len = self.max_doc_length() if doc_len_counts is None else len(doc_len_counts) - 1
        if doc_len_counts is None:
            doc_len_counts = np.zeros(max_len + 1, dtype=np.int32)
        if topic_doc_counts is None:
            topic_doc_counts = np.zeros((self.K, max_len + 1), dtype=np.int32)
        assert doc_len_counts.dtype == np.int32 and topic_doc_counts.dtype == np.int32
        assert doc_len_counts.shape == (max_len + 1,) and topic_doc_counts.shape == (self.K, max_len + 1)
        capi.check(self._L.lda_doc_topic_histograms(self._h, int(max_len), doc_len_counts,
                                                    topic_doc_counts), "lda_doc_topic_histograms")
        return doc_len_counts, topic_doc_counts

    def count_histogram(self, max_count: int, out=None):
        """optimizeBeta's countHistogram of the global nw (added into `out`)."""
        if out is None:
            out = np.zeros(int(max_count) + 1, dtype=np.int32)
        assert out.dtype == np.int32 and len(out) == int(max_count) + 1
        capi.check(self._L.lda_count_histogram(self._h, int(max_count), out), "lda_count_histogram")
        return out

    def row_stats(self) -> float:
        """Token-weighted mean nonzeros per word row of the snapshot."""
        v = C.c_double()
        capi.check(self._L.lda_row_stats(self._h, C.byref(v)), "lda_row_stats")
        return v.value

    def mallet_packed(self):
        """typeTopicCounts in Mallet's packed layout: (rows, row_off, topic_bits)."""
        row_off = np.zeros(self.V + 1, dtype=np.int64)
        bits = C.c_int32()
        capi.check(self._L.lda_to_mallet_packed(self._h, None, row_off, C.byref(bits)),
                   "lda_to_mallet_packed")
        rows = np.zeros(int(row_off[-1]), dtype=np.int32)
        capi.check(self._L.lda_to_mallet_packed(self._h, rows.ctypes.data if len(rows) else None,
                                                row_off, C.byref(bits)), "lda_to_mallet_packed")
        return rows, row_off, bits.value
