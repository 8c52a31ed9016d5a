import sys, ctypes as C
import numpy as np
sys.path.insert(0, "."); sys.path.insert(0, "tests")
from oracle import oracle as O
from ldagibbssampling_amd import capi
from ldagibbssampling_amd.sampler import GibbsSampler
from test_parity_gpu import _ragged_corpus
K = 20
c = _ragged_corpus(D=120, V=700, seed=K)
seed = 1234 + K
g = GibbsSampler(K, c.num_types, c.doc_off, c.words, 0.1, 0.01, seed=seed, tokens_per_range=300, sampler="sparse")
g.sweep(0)
L = capi.load()
L.lda_debug_sample_trace.argtypes = [C.c_void_p, C.c_void_p]
tr = np.zeros((c.num_tokens, 8), np.float32)
capi.check(L.lda_debug_sample_trace(g._h, tr.ctypes.data), "trace")
np.save("gpurun_out/trace_k20.npy", tr)
for i in (2412, 2413, 2414, 14275, 14280):
    print(i, tr[i].tolist())
