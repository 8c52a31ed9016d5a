"""Corpora for the sampler: the reference's input format and synthetic data.

* ``read_inverse_docs`` / ``write_inverse_docs``: the training corpus format
  the reference builds in src/ron/GenerateInverseDocs.java:40-58
  (``test_id \\t file \\t file ...``, gzip) and reads through
  src/cmu_ron/InstanceImporter.java:23-75 + SFDCIterator.java:22-96: each line
  is split with limit 2 on the first tab (target = field 1, data = field 2,
  SFDCIterator.java:60-66), data is tokenised by the regex ``[^\\t]+``
  (InstanceImporter.java:24), lower-cased (:35) and mapped to an alphabet in
  first-seen order (:39, TokenSequence2FeatureSequence).
* ``synthetic_lda``: the LDA generative process of SURVEY.md §8d
  (phi_k ~ Dir(0.01) over V, theta_d ~ Dir(0.1) over K_true = min(K, 100)).
* ``synthetic_changelists``: the C1 plumbing corpus, changelist-shaped
  (Zipf(1.1) path-like tokens, L ~ Poisson(8)).
"""
from __future__ import annotations

import gzip
import io
import re
from dataclasses import dataclass, field

import numpy as np

_TOKEN = re.compile(r"[^\t]+")


@dataclass
class Corpus:
    """Flat token stream: documents are doc_off[d]:doc_off[d+1] of words."""

    doc_off: np.ndarray  # int64 [D+1]
    words: np.ndarray    # int32 [N]
    num_types: int
    alphabet: list = field(default_factory=list)  # id -> token string (may be empty)
    targets: list = field(default_factory=list)   # per-doc target (test id)

    @property
    def num_docs(self) -> int:
        return len(self.doc_off) - 1

    @property
    def num_tokens(self) -> int:
        return int(self.doc_off[-1] - self.doc_off[0])

    def doc(self, d: int) -> np.ndarray:
        return self.words[self.doc_off[d]:self.doc_off[d + 1]]

    def subset(self, docs) -> "Corpus":
        docs = np.asarray(docs, dtype=np.int64)
        lens = self.doc_off[docs + 1] - self.doc_off[docs]
        off = np.zeros(len(docs) + 1, dtype=np.int64)
        np.cumsum(lens, out=off[1:])
        words = np.concatenate([self.doc(int(d)) for d in docs]) if len(docs) else np.zeros(0, np.int32)
        return Corpus(off, words.astype(np.int32), self.num_types, self.alphabet,
                      [self.targets[int(d)] for d in docs] if self.targets else [])


def parse_inverse_docs(text: str, alphabet: dict | None = None, grow: bool = True) -> Corpus:
    """cmu_ron InstanceImporter pipeline over the lines of ``text``."""
    alphabet = {} if alphabet is None else alphabet
    off = [0]
    words = []
    targets = []
    for line in io.StringIO(text):
        line = line.rstrip("\n")
        if line.endswith("\r"):
            line = line[:-1]
        parts = line.split("\t", 1)          # String.split(sep, 2)
        targets.append(parts[0] if len(parts) >= 1 else None)
        data = parts[1] if len(parts) >= 2 else ""
        for tok in _TOKEN.findall(data):
            tok = tok.lower()
            idx = alphabet.get(tok)
            if idx is None:
                if not grow:
                    continue                  # out of vocabulary
                idx = len(alphabet)
                alphabet[tok] = idx
            words.append(idx)
        off.append(len(words))
    inv = [None] * len(alphabet)
    for t, i in alphabet.items():
        inv[i] = t
    return Corpus(np.asarray(off, dtype=np.int64), np.asarray(words, dtype=np.int32),
                  len(alphabet), inv, targets)


def read_inverse_docs(path: str, alphabet: dict | None = None, grow: bool = True) -> Corpus:
    opener = gzip.open if path.endswith(".gz") else open
    with opener(path, "rt", encoding="utf-8", newline="\n") as f:
        return parse_inverse_docs(f.read(), alphabet, grow)


def write_inverse_docs(path: str, corpus: Corpus):
    opener = gzip.open if path.endswith(".gz") else open
    with opener(path, "wt", encoding="utf-8", newline="\n") as f:
        for d in range(corpus.num_docs):
            target = corpus.targets[d] if corpus.targets else str(d)
            toks = [corpus.alphabet[w] for w in corpus.doc(d)]
            f.write(target + "".join("\t" + t for t in toks) + "\n")


def synthetic_lda(num_docs: int, num_types: int, num_topics: int, doc_len: int | None = 200,
                  mean_len: float = 200.0, min_len: int = 20, max_len: int = 1000,
                  seed: int = 20261015, phi_conc: float = 0.01, theta_conc: float = 0.1,
                  k_true: int | None = None) -> Corpus:
    """LDA generative process. doc_len=None -> Poisson lengths."""
    rng = np.random.default_rng(seed)
    kt = min(num_topics, 100) if k_true is None else k_true
    phi = rng.dirichlet(np.full(num_types, phi_conc), size=kt)
    theta = rng.dirichlet(np.full(kt, theta_conc), size=num_docs)
    if doc_len is None:
        lens = np.clip(rng.poisson(mean_len, size=num_docs), min_len, max_len)
    else:
        lens = np.full(num_docs, doc_len)
    off = np.zeros(num_docs + 1, dtype=np.int64)
    np.cumsum(lens, out=off[1:])
    topic_counts = rng.multinomial(lens, theta)                  # [D, kt]
    tok_topic = np.repeat(np.tile(np.arange(kt), num_docs), topic_counts.reshape(-1))
    words = np.empty(len(tok_topic), dtype=np.int32)
    order = np.argsort(tok_topic, kind="stable")
    bounds = np.searchsorted(tok_topic[order], np.arange(kt + 1))
    for k in range(kt):
        n = bounds[k + 1] - bounds[k]
        if n:
            cdf = np.cumsum(phi[k])
            cdf /= cdf[-1]
            words[order[bounds[k]:bounds[k + 1]]] = np.minimum(
                np.searchsorted(cdf, rng.random(n), side="right"), num_types - 1)
    # shuffle tokens inside each document (topic order is an artefact)
    key = rng.random(len(words)) + np.repeat(np.arange(num_docs), lens)
    words = words[np.argsort(key, kind="stable")]
    return Corpus(off, words, num_types)


def synthetic_changelists(num_docs: int = 2000, num_types: int = 5000, mean_len: float = 8.0,
                          zipf_a: float = 1.1, seed: int = 20261015) -> Corpus:
    """C1: changelist-shaped corpus, Zipf word frequencies, path-like tokens."""
    rng = np.random.default_rng(seed)
    ranks = np.arange(1, num_types + 1, dtype=np.float64)
    p = ranks ** -zipf_a
    p /= p.sum()
    lens = np.maximum(1, rng.poisson(mean_len, size=num_docs))
    off = np.zeros(num_docs + 1, dtype=np.int64)
    np.cumsum(lens, out=off[1:])
    draw = rng.choice(num_types, size=int(off[-1]), p=p)
    # Alphabet ids follow first-seen order, as Mallet's Alphabet does.
    first = {}
    words = np.empty(len(draw), dtype=np.int32)
    for i, w in enumerate(draw):
        idx = first.get(int(w))
        if idx is None:
            idx = len(first)
            first[int(w)] = idx
        words[i] = idx
    inv = [None] * len(first)
    for w, idx in first.items():
        inv[idx] = f"//depot/app/main/core/src/module{w % 97}/File{w}.java"
    targets = [str(100000 + d) for d in range(num_docs)]
    return Corpus(off, words, len(first), inv, targets)


def document_completion_split(corpus: Corpus):
    """Split each doc's tokens: first floor(L/2) observed, the rest scored."""
    D = corpus.num_docs
    obs_off = np.zeros(D + 1, dtype=np.int64)
    sc_off = np.zeros(D + 1, dtype=np.int64)
    obs, sc = [], []
    for d in range(D):
        w = corpus.doc(d)
        h = len(w) // 2
        obs.append(w[:h])
        sc.append(w[h:])
        obs_off[d + 1] = obs_off[d] + h
        sc_off[d + 1] = sc_off[d] + len(w) - h
    cat = lambda xs: np.concatenate(xs).astype(np.int32) if xs else np.zeros(0, np.int32)
    return (Corpus(obs_off, cat(obs), corpus.num_types), Corpus(sc_off, cat(sc), corpus.num_types))


def synthetic_lda_torch(num_docs: int, num_types: int, num_topics: int, doc_len: int = 200,
                        seed: int = 20261015, device: str = "cuda", phi_conc: float = 0.01,
                        theta_conc: float = 0.1, doc_seed: int | None = None) -> Corpus:
    """The same generative process as synthetic_lda, drawn on the GPU with
    torch (plumbing for benchmark-sized corpora: 1e8+ tokens in seconds).
    `seed` draws the topics (phi); `doc_seed` (default: seed) the documents,
    so that the shards of one corpus share its topics."""
    import torch

    kt = min(num_topics, 100)
    dev = torch.device(device)
    with torch.random.fork_rng(devices=[dev] if dev.type == "cuda" else []):
        torch.manual_seed(seed)
        phi = torch._standard_gamma(torch.full((kt, num_types), phi_conc, dtype=torch.float64,
                                               device=dev))
        phi = phi / phi.sum(1, keepdim=True)
        cdf = torch.cumsum(phi, 1)
        cdf = cdf / cdf[:, -1:]
        if doc_seed is not None and doc_seed != seed:
            torch.manual_seed(doc_seed)
        theta = torch._standard_gamma(torch.full((num_docs, kt), theta_conc, dtype=torch.float32,
                                                 device=dev))
        theta = theta / theta.sum(1, keepdim=True).clamp_min(1e-30)
        theta = torch.where(torch.isfinite(theta), theta, torch.full_like(theta, 1.0 / kt))
        words = torch.empty(num_docs * doc_len, dtype=torch.int32, device=dev)
        step = max(1, (1 << 26) // doc_len)   # bound the int64 topic matrix
        for d0 in range(0, num_docs, step):
            d1 = min(num_docs, d0 + step)
            topics = torch.multinomial(theta[d0:d1], doc_len, replacement=True).reshape(-1)
            out = torch.empty(topics.numel(), dtype=torch.int64, device=dev)
            for k in range(kt):
                idx = (topics == k).nonzero().squeeze(1)
                if idx.numel():
                    u = torch.rand(idx.numel(), dtype=torch.float64, device=dev)
                    out[idx] = torch.searchsorted(cdf[k], u).clamp_max(num_types - 1)
            words[d0 * doc_len:d1 * doc_len] = out.to(torch.int32)
        off = torch.arange(num_docs + 1, dtype=torch.int64) * doc_len
        return Corpus(off.numpy(), words.cpu().numpy(), num_types)
