"""ParallelTopicModel / TopicInferencer / InstanceList: Python face of the
native host mirror (liblda_topic_model.so, include/lda_topic_model.h).

Method names and meaning follow Mallet 2.0.7 as the reference calls it
(src/cmu_ron/TrainAndPredict.java:108-177, 230-234;
src/cmu/TrainAndPredict.java:93-114, 258-274, 436), so the reference's
driver reads the same:

    model = ParallelTopicModel(500, 100, 1)
    model.addInstances(training)
    model.setOptimizeInterval(20)
    model.setNumThreads(4)          # GPU shards (min with the visible GPUs)
    model.setNumIterations(10000)
    model.estimate()
    inferencer = model.getInferencer()
    theta = inferencer.getSampledDistribution(instance, 100, 10, 10)

Everything runs in the C++ library; there is no Python sampling path.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from . import capi
from .corpus import Corpus, parse_inverse_docs, read_inverse_docs

TM_LIB_PATH = os.path.join(os.path.dirname(capi.LIB_PATH), "liblda_topic_model.so")

_i32p = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")
_i64p = np.ctypeslib.ndpointer(dtype=np.int64, flags="C_CONTIGUOUS")
_f64p = np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS")
_vp = C.c_void_p
_i32 = C.c_int32

# every symbol include/lda_topic_model.h declares
TM_SIGNATURES = {
    "ldatm_create": (_i32, [C.POINTER(_vp), _i32, C.c_double, C.c_double]),
    "ldatm_destroy": (None, [_vp]),
    "ldatm_set_alphabet": (_i32, [_vp, _i32, C.POINTER(C.c_char_p)]),
    "ldatm_add_instances": (_i32, [_vp, C.c_int64, _i64p, _vp, C.POINTER(C.c_char_p)]),
    "ldatm_set_num_iterations": (_i32, [_vp, _i32]),
    "ldatm_set_optimize_interval": (_i32, [_vp, _i32]),
    "ldatm_set_burnin_period": (_i32, [_vp, _i32]),
    "ldatm_set_save_sample_interval": (_i32, [_vp, _i32]),
    "ldatm_set_symmetric_alpha": (_i32, [_vp, _i32]),
    "ldatm_set_topic_display": (_i32, [_vp, _i32, _i32]),
    "ldatm_set_random_seed": (_i32, [_vp, C.c_int64]),
    "ldatm_set_num_threads": (_i32, [_vp, _i32]),
    "ldatm_set_sampler": (_i32, [_vp, _i32]),
    "ldatm_set_exchange_parts": (_i32, [_vp, _i32]),
    "ldatm_set_devices": (_i32, [_vp, _i32, _vp]),
    "ldatm_set_warm_start": (_i32, [_vp, _i32, _i32]),
    "ldatm_set_staleness_threads": (_i32, [_vp, _i32]),
    "ldatm_num_shards": (_i32, [_vp, C.POINTER(_i32)]),
    "ldatm_exchange_info": (_i32, [_vp, C.POINTER(_i32), C.POINTER(_i32), C.POINTER(_i32), C.POINTER(C.c_int64)]),
    "ldatm_plan_shards": (_i32, [_i32, _i32, C.c_int64, _i32, _i32, C.c_int64]),
    "ldatm_set_topics": (_i32, [_vp, C.c_int64, _vp]),
    "ldatm_set_hyper": (_i32, [_vp, _vp, C.c_double, C.c_double]),
    "ldatm_get_sweep": (_i32, [_vp, C.POINTER(C.c_uint32)]),
    "ldatm_set_sweep": (_i32, [_vp, C.c_uint32]),
    "ldatm_set_verbosity": (_i32, [_vp, _i32]),
    "ldatm_set_print_log_likelihood": (_i32, [_vp, _i32]),
    "ldatm_estimate": (_i32, [_vp]),
    "ldatm_get_ll_trace": (_i32, [_vp, _vp, _vp, _i32, C.POINTER(_i32)]),
    "ldatm_model_log_likelihood": (_i32, [_vp, C.POINTER(C.c_double)]),
    "ldatm_get_shape": (_i32, [_vp, C.POINTER(_i32), C.POINTER(_i32), C.POINTER(C.c_int64),
                              C.POINTER(C.c_int64)]),
    "ldatm_get_hyper": (_i32, [_vp, _vp, C.POINTER(C.c_double), C.POINTER(C.c_double)]),
    "ldatm_get_z": (_i32, [_vp, _i32p]),
    "ldatm_get_counts": (_i32, [_vp, _vp, _vp]),
    "ldatm_get_topic_probabilities": (_i32, [_vp, C.c_int64, _f64p]),
    "ldatm_print_document_topics": (_i32, [_vp, C.c_char_p, C.c_double, _i32]),
    "ldatm_document_topics_text": (_i32, [_vp, C.c_double, _i32, _vp, C.c_size_t,
                                          C.POINTER(C.c_size_t)]),
    "ldatm_print_top_words": (_i32, [_vp, C.c_char_p, _i32, _i32]),
    "ldatm_top_words_text": (_i32, [_vp, _i32, _i32, _vp, C.c_size_t, C.POINTER(C.c_size_t)]),
    "ldatm_save": (_i32, [_vp, C.c_char_p]),
    "ldatm_load": (_i32, [C.POINTER(_vp), C.c_char_p]),
    "ldatm_infer": (_i32, [_vp, C.c_int64, _i64p, _vp, _i32, _i32, _i32, C.c_uint64, _f64p]),
    "ldatm_format_double": (_i32, [C.c_double, _i32, C.c_char_p, C.c_size_t]),
    "ldatm_last_error": (C.c_char_p, []),
}

_tm = None


def load_tm(path: str = TM_LIB_PATH):
    """Load liblda_topic_model.so (after the sampler library and torch)."""
    global _tm
    if _tm is not None:
        return _tm
    capi.load()                     # torch first, then liblda_mi355x.so (one HIP runtime)
    if not os.path.exists(path):
        raise ImportError(f"{path} not found: build the native libraries first "
                          "(python -c 'import __graft_entry__ as g; g.build()')")
    L = C.CDLL(path)
    for name, (res, args) in TM_SIGNATURES.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _tm = L
    return L


def _check(status: int, where: str):
    if status != capi.LDA_OK:
        msg = load_tm().ldatm_last_error()
        raise capi.LdaError(status, where, msg.decode() if msg else "")


def format_double(x: float, style: int = 0) -> str:
    """Java Double.toString (style 0) / Mallet's 5-digit NumberFormat (style 1)."""
    buf = C.create_string_buffer(128)
    _check(load_tm().ldatm_format_double(float(x), int(style), buf, 128), "ldatm_format_double")
    return buf.value.decode()


class Alphabet:
    """cc.mallet.types.Alphabet: word <-> id in insertion order."""

    def __init__(self, entries=()):
        self._ids: dict = {}
        self._words: list = []
        for e in entries:
            self.lookupIndex(e)

    def lookupIndex(self, entry, addIfNotPresent: bool = True) -> int:
        i = self._ids.get(entry)
        if i is None:
            if not addIfNotPresent:
                return -1
            i = len(self._words)
            self._ids[entry] = i
            self._words.append(entry)
        return i

    def lookupObject(self, index: int):
        return self._words[index]

    def size(self) -> int:
        return len(self._words)

    def toArray(self) -> list:
        return list(self._words)

    def __len__(self):
        return len(self._words)


class Instance:
    """Mallet Instance after the pipe: data = word ids (FeatureSequence)."""

    def __init__(self, data, target=None, name=None, source=None):
        self.data = np.ascontiguousarray(data, dtype=np.int32)
        self.target, self.name, self.source = target, name, source

    def getSource(self):
        return self.source


class InstanceList:
    """Tokenised documents over one data alphabet (InstanceList + its pipe).

    ``fromInverseDocs`` applies the reference's pipe: lines
    "<target>\\t<data>", tokens ``[^\\t]+`` lower-cased
    (src/cmu_ron/InstanceImporter.java:23-57, SFDCIterator.java:60-66).
    """

    def __init__(self, alphabet: Alphabet | None = None):
        self.alphabet = alphabet if alphabet is not None else Alphabet()
        self.instances: list = []

    def __len__(self):
        return len(self.instances)

    def __iter__(self):
        return iter(self.instances)

    def __getitem__(self, i):
        return self.instances[i]

    def getDataAlphabet(self) -> Alphabet:
        return self.alphabet

    def add(self, instance: Instance):
        self.instances.append(instance)

    def addTokens(self, tokens, target=None, name=None, source=None, grow: bool = True):
        ids = [self.alphabet.lookupIndex(t, grow) for t in tokens]
        self.add(Instance([i for i in ids if i >= 0], target, name, source))

    @classmethod
    def fromCorpus(cls, corpus: Corpus, alphabet: Alphabet | None = None) -> "InstanceList":
        if alphabet is None:
            alphabet = Alphabet(corpus.alphabet if corpus.alphabet else range(corpus.num_types))
        il = cls(alphabet)
        for d in range(corpus.num_docs):
            t = corpus.targets[d] if corpus.targets else None
            il.add(Instance(corpus.doc(d), t, f"example:{d}", None))
        return il

    @classmethod
    def fromInverseDocs(cls, path_or_text: str, alphabet: Alphabet | None = None,
                        grow: bool = True) -> "InstanceList":
        amap = None
        if alphabet is not None:
            amap = dict(alphabet._ids)
        is_path = "\n" not in path_or_text and os.path.exists(path_or_text)
        c = read_inverse_docs(path_or_text, amap, grow) if is_path else \
            parse_inverse_docs(path_or_text, amap, grow)
        if alphabet is not None:
            for w in c.alphabet[alphabet.size():]:
                alphabet.lookupIndex(w)
        return cls.fromCorpus(c, alphabet)


def _flatten(instances):
    lens = np.fromiter((len(i.data) for i in instances), dtype=np.int64, count=len(instances))
    off = np.zeros(len(instances) + 1, dtype=np.int64)
    np.cumsum(lens, out=off[1:])
    words = np.concatenate([i.data for i in instances]).astype(np.int32) if len(instances) \
        else np.zeros(0, np.int32)
    return off, np.ascontiguousarray(words)


class ParallelTopicModel:
    """Mallet 2.0.7 ParallelTopicModel over the GPU sampler (see module doc)."""

    def __init__(self, numberOfTopics: int, alphaSum: float | None = None, beta: float = 0.01):
        L = load_tm()
        self.numTopics = int(numberOfTopics)
        h = C.c_void_p()
        alpha_sum = float(numberOfTopics if alphaSum is None else alphaSum)
        _check(L.ldatm_create(C.byref(h), self.numTopics, alpha_sum, float(beta)), "ldatm_create")
        self._h, self._L = h, L
        self.alphabet: Alphabet | None = None
        self.data: list = []

    def close(self):
        if getattr(self, "_h", None):
            self._L.ldatm_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ------------------------------------------------------------ data
    def addInstances(self, training: InstanceList):
        """New documents get random topics; earlier documents keep theirs."""
        self.alphabet = training.getDataAlphabet()
        V = self.alphabet.size()
        words = (C.c_char_p * V)(*[str(w).encode() for w in self.alphabet.toArray()])
        _check(self._L.ldatm_set_alphabet(self._h, V, words), "ldatm_set_alphabet")
        new = [i for i in training]
        off, w = _flatten(new)
        src = (C.c_char_p * len(new))(*[None if i.source is None else str(i.source).encode()
                                        for i in new]) if new else None
        _check(self._L.ldatm_add_instances(self._h, len(new), off,
                                           w.ctypes.data if len(w) else None, src),
               "ldatm_add_instances")
        self.data.extend(new)

    def getAlphabet(self) -> Alphabet:
        return self.alphabet

    # ---------------------------------------------------------- options
    def setNumIterations(self, n): _check(self._L.ldatm_set_num_iterations(self._h, int(n)), "setNumIterations")
    def setOptimizeInterval(self, n): _check(self._L.ldatm_set_optimize_interval(self._h, int(n)), "setOptimizeInterval")
    def setBurninPeriod(self, n): _check(self._L.ldatm_set_burnin_period(self._h, int(n)), "setBurninPeriod")
    def setSaveSampleInterval(self, n): _check(self._L.ldatm_set_save_sample_interval(self._h, int(n)), "setSaveSampleInterval")
    def setSymmetricAlpha(self, on): _check(self._L.ldatm_set_symmetric_alpha(self._h, int(bool(on))), "setSymmetricAlpha")
    def setTopicDisplay(self, interval, n): _check(self._L.ldatm_set_topic_display(self._h, int(interval), int(n)), "setTopicDisplay")
    def setRandomSeed(self, seed): _check(self._L.ldatm_set_random_seed(self._h, int(seed)), "setRandomSeed")
    def setNumThreads(self, n): _check(self._L.ldatm_set_num_threads(self._h, int(n)), "setNumThreads")
    def setVerbosity(self, level): _check(self._L.ldatm_set_verbosity(self._h, int(level)), "setVerbosity")
    def setPrintLogLikelihood(self, on): _check(self._L.ldatm_set_print_log_likelihood(self._h, int(bool(on))), "setPrintLogLikelihood")

    def setSampler(self, kind: str):
        _check(self._L.ldatm_set_sampler(self._h, capi.SAMPLERS[kind]), "setSampler")

    def setExchangeParts(self, parts: int):
        """Split sweeps across GPU shards (exchange overlapped with sampling)."""
        _check(self._L.ldatm_set_exchange_parts(self._h, int(parts)), "setExchangeParts")

    def setDevices(self, devices):
        """Explicit shard placement: shard g on HIP device devices[g] (an empty
        list returns to setNumThreads' plan).  Shards that all share one device
        exchange through a device-side sum (the multi-shard path on one GPU)."""
        d = np.ascontiguousarray(list(devices), dtype=np.int32)
        _check(self._L.ldatm_set_devices(self._h, len(d), d.ctypes.data if len(d) else None),
               "setDevices")

    def setWarmStart(self, parts: int, sweeps: int):
        """Sweeps 0..sweeps-1 in `parts` sequential parts (default 4 x 50; (1, 0) = off)."""
        _check(self._L.ldatm_set_warm_start(self._h, int(parts), int(sweeps)), "setWarmStart")

    def setStalenessThreads(self, threads: int):
        """Sweeps past the warm start with the staleness of Mallet's T worker
        threads (0 = setNumThreads' T, the default; < 0 = snapshot sweeps)."""
        _check(self._L.ldatm_set_staleness_threads(self._h, int(threads)), "setStalenessThreads")

    def numShards(self) -> int:
        n = C.c_int32()
        _check(self._L.ldatm_num_shards(self._h, C.byref(n)), "numShards")
        return n.value

    def exchangeInfo(self) -> dict:
        """The shards' compact exchange (ldatm_exchange_info): cells per
        packed word (0: none), used-length escape lists, the largest escape
        count gathered, the count reads so far."""
        c, u, m, n = C.c_int32(), C.c_int32(), C.c_int32(), C.c_int64()
        _check(self._L.ldatm_exchange_info(self._h, C.byref(c), C.byref(u), C.byref(m), C.byref(n)),
               "exchangeInfo")
        return {"cells_per_word": c.value, "used_lists": bool(u.value), "escapes_max": m.value,
                "list_exchanges": n.value}

    # --------------------------------------------------------- training
    def estimate(self):
        _check(self._L.ldatm_estimate(self._h), "estimate")

    def llTrace(self):
        """[(iteration, LL/token)] of the last estimate() (every 10 sweeps)."""
        n = C.c_int32()
        _check(self._L.ldatm_get_ll_trace(self._h, None, None, 0, C.byref(n)), "ldatm_get_ll_trace")
        it = np.zeros(n.value, np.int32)
        ll = np.zeros(n.value, np.float64)
        if n.value:
            _check(self._L.ldatm_get_ll_trace(self._h, it.ctypes.data, ll.ctypes.data, n.value,
                                              C.byref(n)), "ldatm_get_ll_trace")
        return list(zip(it.tolist(), ll.tolist()))

    def modelLogLikelihood(self) -> float:
        out = C.c_double()
        _check(self._L.ldatm_model_log_likelihood(self._h, C.byref(out)), "modelLogLikelihood")
        return out.value

    # ------------------------------------------------------------ state
    def _shape(self):
        K, V, D, N = C.c_int32(), C.c_int32(), C.c_int64(), C.c_int64()
        _check(self._L.ldatm_get_shape(self._h, C.byref(K), C.byref(V), C.byref(D), C.byref(N)),
               "ldatm_get_shape")
        return K.value, V.value, D.value, N.value

    @property
    def alpha(self) -> np.ndarray:
        a = np.zeros(self.numTopics, np.float64)
        _check(self._L.ldatm_get_hyper(self._h, a.ctypes.data, None, None), "ldatm_get_hyper")
        return a

    @property
    def alphaSum(self) -> float:
        s = C.c_double()
        _check(self._L.ldatm_get_hyper(self._h, None, C.byref(s), None), "ldatm_get_hyper")
        return s.value

    @property
    def beta(self) -> float:
        b = C.c_double()
        _check(self._L.ldatm_get_hyper(self._h, None, None, C.byref(b)), "ldatm_get_hyper")
        return b.value

    def topicAssignments(self) -> np.ndarray:
        """z of every token (TopicAssignment.topicSequence, concatenated)."""
        z = np.zeros(self._shape()[3], np.int32)
        _check(self._L.ldatm_get_z(self._h, z), "ldatm_get_z")
        return z

    def typeTopicCounts(self):
        """(nw[V, K], tokensPerTopic[K]) dense."""
        K, V, _, _ = self._shape()
        nw = np.zeros((V, K), np.int32)
        nwsum = np.zeros(K, np.int32)
        _check(self._L.ldatm_get_counts(self._h, nw.ctypes.data, nwsum.ctypes.data), "ldatm_get_counts")
        return nw, nwsum

    def getTopicProbabilities(self, doc: int) -> np.ndarray:
        out = np.zeros(self.numTopics, np.float64)
        _check(self._L.ldatm_get_topic_probabilities(self._h, int(doc), out), "getTopicProbabilities")
        return out

    # ---------------------------------------------------------- outputs
    def _text(self, fn, *args) -> str:
        n = C.c_size_t()
        _check(fn(self._h, *args, None, 0, C.byref(n)), fn.__name__)
        buf = C.create_string_buffer(n.value + 1)
        _check(fn(self._h, *args, buf, n.value + 1, C.byref(n)), fn.__name__)
        return buf.value.decode()

    def documentTopics(self, threshold: float = 0.0, max: int = -1) -> str:
        return self._text(self._L.ldatm_document_topics_text, float(threshold), int(max))

    def printDocumentTopics(self, path, threshold: float = 0.0, max: int = -1):
        _check(self._L.ldatm_print_document_topics(self._h, os.fsencode(path), float(threshold),
                                                   int(max)), "printDocumentTopics")

    def displayTopWords(self, numWords: int, usingNewLines: bool = False) -> str:
        return self._text(self._L.ldatm_top_words_text, int(numWords), int(bool(usingNewLines)))

    def printTopWords(self, path, numWords: int, usingNewLines: bool = False):
        _check(self._L.ldatm_print_top_words(self._h, os.fsencode(path), int(numWords),
                                             int(bool(usingNewLines))), "printTopWords")

    # ------------------------------------------------ checkpoint / resume
    def save(self, path):
        """Everything needed to continue this run bit for bit."""
        _check(self._L.ldatm_save(self._h, os.fsencode(path)), "ldatm_save")

    @classmethod
    def load(cls, path) -> "ParallelTopicModel":
        L = load_tm()
        h = C.c_void_p()
        _check(L.ldatm_load(C.byref(h), os.fsencode(path)), "ldatm_load")
        m = cls.__new__(cls)
        m._h, m._L = h, L
        m.numTopics = m._shape()[0]
        m.alphabet = None
        m.data = []
        return m

    # -------------------------------------------------------- inference
    def getInferencer(self) -> "TopicInferencer":
        return TopicInferencer(self)


class TopicInferencer:
    """getSampledDistribution against the model's current (frozen) counts."""

    def __init__(self, model: ParallelTopicModel):
        self.model = model

    def getSampledDistributions(self, instances, numIterations: int = 100, thinning: int = 10,
                                burnIn: int = 10, seed: int = 0) -> np.ndarray:
        off, w = _flatten(list(instances))
        theta = np.zeros((len(off) - 1, self.model.numTopics), np.float64)
        _check(self.model._L.ldatm_infer(self.model._h, len(off) - 1, off,
                                         w.ctypes.data if len(w) else None, int(numIterations),
                                         int(thinning), int(burnIn), int(seed) & (2**64 - 1), theta),
               "getSampledDistribution")
        return theta

    def getSampledDistribution(self, instance, numIterations: int = 100, thinning: int = 10,
                               burnIn: int = 10, seed: int = 0) -> np.ndarray:
        if not isinstance(instance, Instance):
            instance = Instance(instance)
        return self.getSampledDistributions([instance], numIterations, thinning, burnIn, seed)[0]


def plan_shards(num_threads: int, num_devices: int, num_tokens: int, num_types: int,
                num_topics: int, num_docs: int) -> int:
    """GPU shards setNumThreads(num_threads) becomes for this corpus
    (ldatm_plan_shards; host-only)."""
    return int(load_tm().ldatm_plan_shards(int(num_threads), int(num_devices), int(num_tokens),
                                           int(num_types), int(num_topics), int(num_docs)))
