"""Debug helper: first token where the sparse GPU draw differs from the oracle,
with the branch/quantities recomputed in numpy float32 (test infrastructure)."""
import sys
import numpy as np
sys.path.insert(0, ".")
sys.path.insert(0, "tests")
from oracle import oracle as O
from ldagibbssampling_amd.sampler import GibbsSampler
from test_parity_gpu import _ragged_corpus

K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
c = _ragged_corpus(D=120, V=700, seed=K)
alpha = np.full(K, 0.1)
seed = 1234 + K
g = GibbsSampler(K, c.num_types, c.doc_off, c.words, alpha, 0.01, seed=seed, tokens_per_range=300, sampler="sparse")
o = O.ExactSampler(K, c.num_types, c.doc_off, c.words, alpha, 0.01, seed, kind="sparse")
g.sweep(0); o.apply()
z0 = o.z().copy()
nw, nwsum, _, _ = o.counts()
g.sweep(1); o.sweep(1)
zg, zo_ = g.z(), o.z()
bad = np.nonzero(zg != zo_)[0]
print("mismatches", len(bad), bad[:20])
docs = np.searchsorted(c.doc_off, bad, side="right") - 1
print("docs", docs[:20], "doc starts", c.doc_off[docs[:20]])
i = int(bad[0]); d = int(docs[0]); s0 = int(c.doc_off[d])
print("token", i, "doc", d, "pos", i - s0, "doc len", c.doc_off[d+1]-s0, "gpu", zg[i], "oracle", zo_[i], "old", z0[i], "word", c.words[i])
# reconstruct the state
Kp = (K + 63)//64*64; C = Kp//64
nd = np.zeros(Kp, np.int64)
for j in range(s0, i): nd[zo_[j]] += 1
for j in range(i, int(c.doc_off[d+1])): nd[z0[j]] += 1
zo = int(z0[i]); w = int(c.words[i])
nd[zo] -= 1
f32 = np.float32
vb = f32(700 * 0.01)
inv = np.zeros(Kp, f32); invm1 = np.zeros(Kp, f32); al = np.zeros(Kp, f32)
for k in range(K):
    inv[k] = f32(1.0)/(f32(nwsum[k]) + vb); invm1[k] = f32(1.0)/(f32(nwsum[k]-1) + vb); al[k] = f32(0.1)
coef = ((nd.astype(f32) + al) * inv).astype(f32)
coef[zo] = f32((f32(nd[zo]) + al[zo]) * invm1[zo])
u = O.u01(O.draw(seed, i, 0, 0))
row = nw[w]
ent = [(k, row[k] - (1 if k == zo else 0)) for k in range(K) if row[k] > 0]
print("u", u, "n entries", len(ent), "zo", zo, "nd", nd[:K])
TB = np.zeros(64, f32)
for l in range(64):
    acc = f32(0)
    for e in range(l, len(ent), 64): acc = f32(acc + f32(coef[ent[e][0]] * f32(ent[e][1])))
    TB[l] = acc
TA = np.zeros(64, f32)
for l in range(64):
    a = f32(0)
    for j in range(C): a = f32(np.float32(np.float64(coef[l*C+j])*np.float64(f32(0.01)) + np.float64(a)))
    TA[l] = a
print("TB lanes", TB[:len(ent)], "\nTA lanes", TA[:K])
print("cumB", np.cumsum(TB[:len(ent)], dtype=f32)[-1], "cumA", np.cumsum(TA, dtype=f32)[-1])
