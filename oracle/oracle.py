"""ctypes binding of the CPU oracle (oracle/lda_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py — never by the product package.  See
oracle/lda_oracle.h for what each restatement follows and for its parity
status (cpu_exact: bit-exact definition of the GPU sampler, pinned by
tests/golden/; cpu_mallet: Mallet 2.0.7 restatement, parity unpinned against
Mallet itself because Mallet cannot be built or run in this image).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "lib", "liblda_oracle.so")
_lib = None

_i32p = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")
_i64p = np.ctypeslib.ndpointer(dtype=np.int64, flags="C_CONTIGUOUS")
_f64p = np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS")


def build() -> str:
    """Compile the oracle with its Makefile (gcc)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(_LIB_PATH):
        build()
    L = C.CDLL(_LIB_PATH)
    L.orc_philox4x32_10.argtypes = [C.POINTER(C.c_uint32), C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]
    L.orc_draw.restype = C.c_uint32
    L.orc_draw.argtypes = [C.c_uint64, C.c_uint64, C.c_uint32, C.c_uint32]
    L.orc_u01.restype = C.c_float
    L.orc_u01.argtypes = [C.c_uint32]
    L.orc_jrandom_seed.argtypes = [C.c_void_p, C.c_int64]
    L.orc_jrandom_next_int.restype = C.c_int32
    L.orc_jrandom_next_int.argtypes = [C.c_void_p]
    L.orc_jrandom_next_int_n.restype = C.c_int32
    L.orc_jrandom_next_int_n.argtypes = [C.c_void_p, C.c_int32]
    L.orc_jrandom_next_double.restype = C.c_double
    L.orc_jrandom_next_double.argtypes = [C.c_void_p]
    L.orc_log_gamma_stirling.restype = C.c_double
    L.orc_log_gamma_stirling.argtypes = [C.c_double]
    L.orc_digamma.restype = C.c_double
    L.orc_digamma.argtypes = [C.c_double]
    L.orc_learn_parameters.restype = C.c_double
    L.orc_learn_parameters.argtypes = [_f64p, C.c_int32, _i32p, _i32p, C.c_int32, C.c_double,
                                       C.c_double, C.c_int32]
    L.orc_learn_symmetric_concentration.restype = C.c_double
    L.orc_learn_symmetric_concentration.argtypes = [_i32p, C.c_int64, _i32p, C.c_int64, C.c_int32,
                                                    C.c_double]

    L.orc_exact_create.restype = C.c_void_p
    L.orc_exact_create.argtypes = [C.c_int32, C.c_int32, C.c_int64, _i64p, _i32p, C.c_void_p,
                                   _f64p, C.c_double, C.c_uint64, C.c_int64]
    L.orc_exact_destroy.argtypes = [C.c_void_p]
    L.orc_exact_kpad.restype = C.c_int32
    L.orc_exact_kpad.argtypes = [C.c_void_p]
    L.orc_exact_sample.argtypes = [C.c_void_p, C.c_int]
    L.orc_exact_sample_docs.argtypes = [C.c_void_p, C.c_int64, C.c_int64]
    L.orc_exact_end_sweep.argtypes = [C.c_void_p]
    L.orc_exact_delta.restype = C.POINTER(C.c_int32)
    L.orc_exact_delta.argtypes = [C.c_void_p]
    L.orc_exact_apply.argtypes = [C.c_void_p]
    L.orc_exact_set_alpha_beta.argtypes = [C.c_void_p, _f64p, C.c_double]
    L.orc_exact_set_sweep.argtypes = [C.c_void_p, C.c_uint32]
    L.orc_exact_load_snapshot.argtypes = [C.c_void_p, _i32p, _i32p]
    L.orc_exact_set_kind.argtypes = [C.c_void_p, C.c_int]
    L.orc_exact_set_half.argtypes = [C.c_void_p, C.c_int]
    L.orc_exact_get_sweep.restype = C.c_uint32
    L.orc_exact_get_sweep.argtypes = [C.c_void_p]
    L.orc_exact_get_z.argtypes = [C.c_void_p, _i32p]
    L.orc_exact_get_counts.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
    L.orc_exact_log_likelihood.restype = C.c_double
    L.orc_exact_log_likelihood.argtypes = [C.c_void_p]
    L.orc_exact_log_likelihood_parts.argtypes = [C.c_void_p, C.POINTER(C.c_double),
                                                 C.POINTER(C.c_double)]
    L.orc_exact_big_draw.restype = C.c_int
    L.orc_exact_big_draw.argtypes = [C.c_void_p, C.c_int32, _i32p, C.c_int32,
                                     np.ctypeslib.ndpointer(dtype=np.uint32, flags="C_CONTIGUOUS")]
    L.orc_exact_infer.argtypes = [C.c_void_p, C.c_int64, _i64p, _i32p, C.c_int32, C.c_int32,
                                  C.c_int32, C.c_uint64, _f64p]

    L.orc_mallet_create.restype = C.c_void_p
    L.orc_mallet_create.argtypes = [C.c_int32, C.c_double, C.c_double, C.c_int32, C.c_int64,
                                    _i64p, _i32p, C.c_int64, C.c_int32]
    L.orc_mallet_destroy.argtypes = [C.c_void_p]
    L.orc_mallet_estimate.argtypes = [C.c_void_p, C.c_int32]
    L.orc_mallet_set_pin_threads.argtypes = [C.c_void_p, C.c_int32]
    L.orc_mallet_timing.argtypes = [C.c_void_p, C.POINTER(C.c_double), C.POINTER(C.c_double), C.c_int32]
    L.orc_mallet_timing_build.argtypes = [C.c_void_p, C.POINTER(C.c_double)]
    L.orc_mallet_set_optimize.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_int32]
    L.orc_mallet_get_hyper.argtypes = [C.c_void_p, _f64p, C.POINTER(C.c_double)]
    L.orc_mallet_log_likelihood.restype = C.c_double
    L.orc_mallet_log_likelihood.argtypes = [C.c_void_p]
    L.orc_mallet_get_z.argtypes = [C.c_void_p, _i32p]
    L.orc_mallet_get_counts.argtypes = [C.c_void_p, _i32p, _i32p]
    L.orc_mallet_infer.argtypes = [C.c_void_p, C.c_int64, _i64p, _i32p, C.c_int32, C.c_int32,
                                   C.c_int32, C.c_int64, _f64p]
    L.orc_doc_completion_loglik.restype = C.c_double
    L.orc_doc_completion_loglik.argtypes = [C.c_int32, C.c_int32, _i32p, _i32p, C.c_double,
                                            C.c_int64, _f64p, _i64p, _i32p]
    _lib = L
    return L


# ---------------------------------------------------------------- primitives
def philox4x32_10(ctr, key):
    L = lib()
    c = (C.c_uint32 * 4)(*ctr)
    k = (C.c_uint32 * 2)(*key)
    o = (C.c_uint32 * 4)()
    L.orc_philox4x32_10(c, k, o)
    return [int(x) for x in o]


def draw(seed: int, gtok: int, c2: int, c3: int) -> int:
    return int(lib().orc_draw(seed, gtok, c2, c3))


def u01(x: int) -> float:
    return float(lib().orc_u01(x))


def log_gamma_stirling(z: float) -> float:
    return float(lib().orc_log_gamma_stirling(z))


def digamma(x: float) -> float:
    return float(lib().orc_digamma(x))


def learn_parameters(alpha, topic_doc_counts, doc_len_counts, shape=1.001, scale=1.0, iters=1):
    """Dirichlet.learnParameters: returns (new alpha, new alpha sum)."""
    a = np.ascontiguousarray(alpha, dtype=np.float64).copy()
    h = np.ascontiguousarray(topic_doc_counts, dtype=np.int32)
    lens = np.ascontiguousarray(doc_len_counts, dtype=np.int32)
    K, W = h.shape
    assert len(lens) == W and len(a) == K
    s = lib().orc_learn_parameters(a, K, h, lens, W - 1, shape, scale, iters)
    return a, float(s)


def learn_symmetric_concentration(count_hist, length_hist, dims, value) -> float:
    """Dirichlet.learnSymmetricConcentration with DENSE histograms."""
    c = np.ascontiguousarray(count_hist, dtype=np.int32)
    lens = np.ascontiguousarray(length_hist, dtype=np.int32)
    return float(lib().orc_learn_symmetric_concentration(c, len(c) - 1, lens, len(lens) - 1,
                                                         dims, value))


class JavaRandom:
    """java.util.Random (the base of cc.mallet.util.Randoms)."""

    def __init__(self, seed: int):
        self._state = (C.c_uint64 * 1)()
        lib().orc_jrandom_seed(self._state, seed)

    def nextInt(self, n: int | None = None) -> int:
        if n is None:
            return int(lib().orc_jrandom_next_int(self._state))
        return int(lib().orc_jrandom_next_int_n(self._state, n))

    def nextDouble(self) -> float:
        return float(lib().orc_jrandom_next_double(self._state))


# ---------------------------------------------------------------- cpu_exact
SEQ_FRACTION_UNIT = 720720      # include/lda_mi355x.h LDA_SEQ_FRACTION_UNIT


def equal_cum(parts: int):
    """lda_capi.cpp equal_cum: cumulative cuts of equal parts (exact)."""
    return [SEQ_FRACTION_UNIT * i // parts for i in range(parts + 1)]


def quantise_fractions(fractions):
    """lda_capi.cpp quantise_fractions: cumulative fractions in units of
    1 / SEQ_FRACTION_UNIT (llround of the running double sum; the last = 1)."""
    import math
    cum, acc = [0], 0.0
    for i, f in enumerate(fractions):
        acc += float(f)
        cum.append(SEQ_FRACTION_UNIT if i + 1 == len(fractions)
                   else int(math.floor(acc * SEQ_FRACTION_UNIT + 0.5)))
    return cum


def staleness_schedule(threads: int):
    """lda_staleness_schedule: (parts, fractions) with Mallet's mean live
    fraction 1/(2T) for T worker threads."""
    import math
    if threads == 1:
        return 4, [0.25] * 4
    f = 0.5 * (1.0 - math.sqrt(1.0 - 2.0 / threads))
    return 2, [f, 1.0 - f]
class ExactSampler:
    """cpu_exact: the bit-exact definition of the GPU sampler (one shard)."""

    def __init__(self, K, V, doc_off, words, alpha, beta, seed, z_init=None, token_base=0,
                 kind="dense", half=None):
        """half: which dense kernel's draw to follow for K <= 128 (the GPU's
        LDA_DENSE_HALF): 0 = full-wave k_sample<C>, 1 = half-wave, 2 =
        quarter-wave (the library's default); None = as the library would
        choose under the current environment."""
        self.K, self.V = int(K), int(V)
        self.doc_off = np.ascontiguousarray(doc_off, dtype=np.int64)
        self.words = np.ascontiguousarray(words, dtype=np.int32)
        self.D = len(self.doc_off) - 1
        self.N = int(self.doc_off[-1] - self.doc_off[0])
        alpha = np.ascontiguousarray(np.broadcast_to(np.asarray(alpha, dtype=np.float64), (self.K,)))
        zi = None
        if z_init is not None:
            self._zi = np.ascontiguousarray(z_init, dtype=np.int32)
            zi = self._zi.ctypes.data
        self._h = lib().orc_exact_create(self.K, self.V, self.D, self.doc_off, self.words, zi,
                                         alpha, float(beta), int(seed) & (2**64 - 1), int(token_base))
        self.Kp = int(lib().orc_exact_kpad(self._h))
        self._pending = True      # create leaves the shard's counts as the pending delta
        self.token_base = int(token_base)
        lib().orc_exact_set_kind(self._h, {"dense": 0, "dense32": 0, "sparse": 1}[kind])
        if half is None:
            half = os.environ.get("LDA_DENSE_HALF", "2")[:1]
            half = int(half) if half in ("0", "1", "2") else 2
        lib().orc_exact_set_half(self._h, int(half))

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            lib().orc_exact_destroy(h)
            self._h = None

    def delta(self) -> np.ndarray:
        """View of the pending delta buffer (nw delta [V*Kp] then nwsum delta [Kp])."""
        p = lib().orc_exact_delta(self._h)
        n = self.V * self.Kp + self.Kp
        return np.ctypeslib.as_array(p, shape=(n,))

    def set_warm_start(self, parts: int, sweeps: int, corpus_first_token: int = 0, corpus_tokens: int = 0):
        """lda_set_warm_start: sweeps whose sweep counter is below `sweeps` run in
        `parts` sequential parts (equal pieces of each block of the corpus,
        _seq_runs), each applied before the next."""
        self._warm = (int(parts), int(sweeps) if parts > 1 else 0)
        self._warm_cum = equal_cum(int(parts))
        self._warm_corpus = self._corpus(corpus_first_token, corpus_tokens)

    def set_sequential_sweeps(self, parts: int, fractions=None, corpus_first_token: int = 0,
                              corpus_tokens: int = 0):
        """lda_set_sequential_sweeps: every sweep that is not a warm-start sweep
        in `parts` sequential parts, part i the fraction fractions[i] of every
        block (quantised as lda_capi.cpp quantise_fractions)."""
        parts = int(parts)
        self._steady_cum = equal_cum(parts) if (parts == 1 or fractions is None) else \
            quantise_fractions(fractions)
        self._steady_corpus = self._corpus(corpus_first_token, corpus_tokens)

    def _corpus(self, g0, gn):
        if gn <= 0:                                  # this shard is the whole corpus
            return (self.token_base, self.N)
        return (int(g0), int(gn))

    WARM_BLOCKS = 64      # include/lda_mi355x.h LDA_WARM_BLOCKS

    def _seq_runs(self, cum, corpus):
        """lda_capi.cpp seq_part_runs: the corpus [g0, g0 + gn) cut into
        WARM_BLOCKS blocks, block b into pieces at the cumulative fractions
        cum[i] / Q; the cut at (b, i) is the first document starting at or
        after g0 + gn (b Q + cum[i]) // (B Q); piece i of every block is part
        i.  Returns part i's local document runs [(d0, d1), ...]."""
        P, B, Q = len(cum) - 1, self.WARM_BLOCKS, SEQ_FRACTION_UNIT
        g0, gn = corpus
        off = self.doc_off - self.doc_off[0]
        runs = [[] for _ in range(P)]
        prev = 0
        for b in range(B):
            for i in range(P):
                nxt = self.D
                if b + 1 < B or i + 1 < P:
                    d = int(np.searchsorted(off, g0 + gn * (b * Q + cum[i + 1]) // (B * Q) - self.token_base,
                                            side="left"))
                    nxt = min(max(d, prev), self.D)
                if nxt > prev:
                    runs[i].append((prev, nxt))
                prev = nxt
        return runs

    def _warm_runs(self):
        return self._seq_runs(self._warm_cum, self._warm_corpus)

    def _sweep_runs(self):
        """The runs of the next sweep's sequential parts, or None (a plain sweep)."""
        warm = getattr(self, "_warm", (1, 0))
        if warm[0] > 1 and self.sweep_index < warm[1]:
            return self._warm_runs()
        cum = getattr(self, "_steady_cum", None)
        if cum is not None and len(cum) > 2:
            return self._seq_runs(cum, self._steady_corpus)
        return None

    def sample(self, frozen=False):
        if self._pending:
            raise RuntimeError("sample with a pending delta: apply first (as lda_sample)")
        runs = None if frozen else self._sweep_runs()
        if runs is not None:
            for i, part in enumerate(runs):
                for d0, d1 in part:
                    self.sample_docs(d0, d1)
                if i + 1 < len(runs):
                    self.apply()
            self.end_sweep()
            return
        lib().orc_exact_sample(self._h, 1 if frozen else 0)
        self._pending = not frozen

    def sample_docs(self, d0: int, d1: int):
        """Documents [d0, d1) of the current sweep into the delta, the sweep
        counter unchanged (one part of a split sweep; end_sweep() advances)."""
        lib().orc_exact_sample_docs(self._h, int(d0), int(d1))

    def end_sweep(self):
        lib().orc_exact_end_sweep(self._h)
        self._pending = True

    def apply(self):
        lib().orc_exact_apply(self._h)
        self._pending = False

    def sweep(self, n=1):
        """Same contract as lda_sweep: apply a pending delta, then n x (sample + apply)."""
        if self._pending:
            self.apply()
        for _ in range(n):
            self.sample()
            self.apply()

    @property
    def sweep_index(self) -> int:
        return int(lib().orc_exact_get_sweep(self._h))

    @sweep_index.setter
    def sweep_index(self, v: int):
        lib().orc_exact_set_sweep(self._h, int(v))

    def load_snapshot(self, nw, nwsum):
        """Replace the snapshot by a global one (nw [V, K], nwsum [K]); drops
        the pending delta (a slice of a larger corpus, checked against the
        GPU's state of that corpus)."""
        nw = np.ascontiguousarray(nw, dtype=np.int32)
        nwsum = np.ascontiguousarray(nwsum, dtype=np.int32)
        assert nw.shape == (self.V, self.K) and nwsum.shape == (self.K,)
        lib().orc_exact_load_snapshot(self._h, nw, nwsum)
        self._pending = False

    def set_alpha_beta(self, alpha, beta):
        a = np.ascontiguousarray(np.broadcast_to(np.asarray(alpha, dtype=np.float64), (self.K,)))
        lib().orc_exact_set_alpha_beta(self._h, a, float(beta))

    def z(self) -> np.ndarray:
        out = np.empty(self.N, dtype=np.int32)
        lib().orc_exact_get_z(self._h, out)
        return out

    def counts(self, with_nd=False):
        nw = np.empty((self.V, self.K), dtype=np.int32)
        nwsum = np.empty(self.K, dtype=np.int32)
        nd = np.empty((self.D, self.K), dtype=np.int32) if with_nd else None
        ndsum = np.empty(self.D, dtype=np.int32)
        lib().orc_exact_get_counts(self._h, nw.ctypes.data, nwsum.ctypes.data,
                                   nd.ctypes.data if with_nd else None, ndsum.ctypes.data)
        return nw, nwsum, nd, ndsum

    def log_likelihood(self) -> float:
        return float(lib().orc_exact_log_likelihood(self._h))

    def log_likelihood_parts(self):
        a, b = C.c_double(), C.c_double()
        lib().orc_exact_log_likelihood_parts(self._h, C.byref(a), C.byref(b))
        return a.value, b.value

    def big_draw(self, w: int, nd, zo: int, x) -> int:
        """One large-K draw (exact_draw_big) for word w, document counts nd
        [Kp] without the token, old topic zo (-1: frozen), Philox words x[0..2]."""
        nd = np.ascontiguousarray(nd, dtype=np.int32)
        assert nd.shape == (self.Kp,)
        x = np.ascontiguousarray(x, dtype=np.uint32)
        return int(lib().orc_exact_big_draw(self._h, int(w), nd, int(zo), x))

    def infer(self, doc_off, words, n_iter=100, burn_in=10, thin=10, seed=0):
        doc_off = np.ascontiguousarray(doc_off, dtype=np.int64)
        words = np.ascontiguousarray(words, dtype=np.int32)
        Dh = len(doc_off) - 1
        theta = np.zeros((Dh, self.K), dtype=np.float64)
        lib().orc_exact_infer(self._h, Dh, doc_off, words, n_iter, burn_in, thin, int(seed), theta)
        return theta


# ---------------------------------------------------------------- cpu_mallet
class MalletModel:
    """cpu_mallet: Mallet 2.0.7 ParallelTopicModel restatement (parity unpinned)."""

    def __init__(self, K, alpha_sum, beta, V, doc_off, words, seed, num_threads=1):
        self.K, self.V = int(K), int(V)
        self.doc_off = np.ascontiguousarray(doc_off, dtype=np.int64)
        self.words = np.ascontiguousarray(words, dtype=np.int32)
        self.D = len(self.doc_off) - 1
        self.N = int(self.doc_off[-1] - self.doc_off[0])
        self.alpha_sum, self.beta = float(alpha_sum), float(beta)
        self._h = lib().orc_mallet_create(self.K, self.alpha_sum, self.beta, self.V, self.D,
                                          self.doc_off, self.words, int(seed), int(num_threads))

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            lib().orc_mallet_destroy(h)
            self._h = None

    def set_pin_threads(self, on: bool = True):
        """Pin worker t to the t-th CPU of this process's affinity mask."""
        lib().orc_mallet_set_pin_threads(self._h, 1 if on else 0)

    def timing(self, reset: bool = False):
        """(sampling s, sumTypeTopicCounts merge s) accumulated by estimate()."""
        a, b = C.c_double(), C.c_double()
        lib().orc_mallet_timing(self._h, C.byref(a), C.byref(b), 1 if reset else 0)
        return a.value, b.value

    def build_time(self) -> float:
        """Seconds of the timed sampling phase spent in the workers'
        buildLocalTypeTopicCounts (the slowest worker per sweep; 0 with one
        thread, which Mallet does not rebuild); reset with timing(reset=True)."""
        a = C.c_double()
        lib().orc_mallet_timing_build(self._h, C.byref(a))
        return a.value

    def estimate(self, n_iter):
        lib().orc_mallet_estimate(self._h, int(n_iter))

    def set_optimize(self, interval: int, burnin: int = 200, symmetric: bool = False):
        """setOptimizeInterval / setBurninPeriod / setSymmetricAlpha."""
        lib().orc_mallet_set_optimize(self._h, int(interval), int(burnin), int(bool(symmetric)))

    def hyper(self):
        """(alpha[K], beta) after any optimisation."""
        a = np.empty(self.K, dtype=np.float64)
        b = C.c_double()
        lib().orc_mallet_get_hyper(self._h, a, C.byref(b))
        return a, b.value

    def log_likelihood(self) -> float:
        return float(lib().orc_mallet_log_likelihood(self._h))

    def z(self):
        out = np.empty(self.N, dtype=np.int32)
        lib().orc_mallet_get_z(self._h, out)
        return out

    def counts(self):
        nw = np.empty((self.V, self.K), dtype=np.int32)
        nwsum = np.empty(self.K, dtype=np.int32)
        lib().orc_mallet_get_counts(self._h, nw, nwsum)
        return nw, nwsum

    def infer(self, doc_off, words, n_iter=100, burn_in=10, thin=10, seed=0):
        doc_off = np.ascontiguousarray(doc_off, dtype=np.int64)
        words = np.ascontiguousarray(words, dtype=np.int32)
        Dh = len(doc_off) - 1
        theta = np.zeros((Dh, self.K), dtype=np.float64)
        lib().orc_mallet_infer(self._h, Dh, doc_off, words, n_iter, burn_in, thin, int(seed), theta)
        return theta


def doc_completion_loglik(K, V, nw, nwsum, beta, theta, doc_off, words) -> float:
    nw = np.ascontiguousarray(nw, dtype=np.int32)
    nwsum = np.ascontiguousarray(nwsum, dtype=np.int32)
    theta = np.ascontiguousarray(theta, dtype=np.float64)
    doc_off = np.ascontiguousarray(doc_off, dtype=np.int64)
    words = np.ascontiguousarray(words, dtype=np.int32)
    return float(lib().orc_doc_completion_loglik(K, V, nw, nwsum, float(beta), len(doc_off) - 1,
                                                 theta, doc_off, words))


# ------------------------------------------------ compact exchange (checker)
def exchange_biases(world: int, cells: int = 2):
    """Per-field biases of the packed word: lda_kernels.h exch_bias0 /
    exch_bias1 (2 cells per word), or exch_bias4 x 3 + exch_bias4_top
    (4 cells per word, lda_set_exchange_cells)."""
    if cells == 4:
        return (128 // world,) * 3 + (64 // world,)
    return 32768 // world, 16384 // world


def _field_shifts(cells: int):
    return (0, 8, 16, 24) if cells == 4 else (0, 16)


def exchange_cap(world: int, max_tokens: int, cells: int = 2) -> int:
    """lda_capi.cpp exchange_dims: escapes per rank <= 2 N / (smallest bias) (+1)."""
    return 2 * int(max_tokens) // min(exchange_biases(world, cells)) + 1


def exchange_pack(buf, world: int, Kp: int, max_tokens: int, cells: int = 2):
    """Numpy restatement of lda_exchange_pack (k_exch_pack, k_exch_pack4):
    buf int32 [V Kp | Kp] -> (packed int32 [V Kp / cells | Kp], escapes
    int32 [1 + 3 cap]).  Escapes are listed in cell order here (the GPU's
    order is scheduling-dependent; the sum they produce is not)."""
    bs = exchange_biases(world, cells)
    cap = exchange_cap(world, max_tokens, cells)
    buf = np.asarray(buf, dtype=np.int64)
    n = buf.size - Kp
    d = buf[:n].reshape(-1, cells)
    packed = np.zeros(n // cells + Kp, dtype=np.int64)
    escs = []
    for j, (b, sh) in enumerate(zip(bs, _field_shifts(cells))):
        x = d[:, j]
        e = (x < -b) | (x >= b)
        packed[:n // cells] += np.where(e, b, x + b) << sh
        escs.append(e)
    packed[n // cells:] = buf[n:]
    idx = np.flatnonzero(np.stack(escs, axis=1).reshape(-1))
    assert len(idx) <= cap, "escape bound violated"
    esc = np.zeros(1 + 3 * cap, dtype=np.int64)
    esc[0] = len(idx)
    e = esc[1:1 + 3 * len(idx)].reshape(-1, 3)
    e[:, 0] = idx & 0xFFFFFFFF
    e[:, 1] = idx >> 32
    e[:, 2] = buf[idx]
    return packed.astype(np.int32), esc.astype(np.int32)


def exchange_unpack(packed_sum, escapes_all, world: int, Kp: int, max_tokens: int, list_cap=None,
                    cells: int = 2):
    """lda_exchange_unpack: the summed packed words (int32 [V Kp / cells |
    Kp]) and every rank's escape list (world x [1 + 3 cap], rank order) ->
    the int32 sum of the ranks' buffers [V Kp | Kp].  list_cap: the lists were
    sent at 1 + 3 list_cap int32 each (lda_exchange_unpack_lists; 0 and
    escapes_all None: no rank had an escape)."""
    bs = exchange_biases(world, cells)
    cap = exchange_cap(world, max_tokens, cells)
    if list_cap is not None:
        assert 0 <= list_cap <= cap
        cap = int(list_cap)
        if escapes_all is None:
            assert cap == 0
            escapes_all = np.zeros(world, dtype=np.int32)
    p = np.asarray(packed_sum, dtype=np.int64) & 0xFFFFFFFF
    words = p.size - Kp
    out = np.empty(cells * words + Kp, dtype=np.int64)
    width = 32 // cells
    for j, (b, sh) in enumerate(zip(bs, _field_shifts(cells))):
        out[j:cells * words:cells] = ((p[:words] >> sh) & ((1 << width) - 1)) - world * b
    out[cells * words:] = np.asarray(packed_sum[words:], dtype=np.int64)
    ea = np.asarray(escapes_all, dtype=np.int64).reshape(world, 1 + 3 * cap)
    for r in range(world):
        n = min(int(ea[r, 0]), cap)
        e = ea[r, 1:1 + 3 * n].reshape(-1, 3)
        cell = (e[:, 0] & 0xFFFFFFFF) | (e[:, 1] << 32)
        np.add.at(out, cell, e[:, 2])
    return out.astype(np.int32)


def _mix64(x):
    """splitmix64's finaliser on uint64 arrays (k_counts_checksum's mix64)."""
    x = x ^ (x >> np.uint64(30))
    x = x * np.uint64(0xBF58476D1CE4E5B9)
    x = x ^ (x >> np.uint64(27))
    x = x * np.uint64(0x94D049BB133111EB)
    return x ^ (x >> np.uint64(31))


def counts_checksum(nw, nwsum) -> int:
    """lda_counts_checksum restated: sum mod 2^64 over the nonzero cells of nw
    (V x K) and nwsum (K) of mix64(index << 32 | (uint32) value), index = w K +
    k in nw and V K + k in nwsum."""
    nw = np.asarray(nw, dtype=np.int64)
    V, K = nw.shape
    vals = np.concatenate([nw.reshape(-1), np.asarray(nwsum, dtype=np.int64).reshape(-1)[:K]])
    idx = np.flatnonzero(vals)
    x = (idx.astype(np.uint64) << np.uint64(32)) | (vals[idx] & 0xFFFFFFFF).astype(np.uint64)
    with np.errstate(over="ignore"):
        return int(_mix64(x).sum(dtype=np.uint64))
