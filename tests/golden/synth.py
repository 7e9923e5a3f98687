"""Deterministic synthetic chunks for parity tests (test infrastructure).

Everything here is regenerated from integer seeds with numpy's PCG64, so the
golden fixtures only need to store seeds and expected outputs.  The corpus
mimics what CLASSMATE-RAG ingests (SURVEY.md §8c "Golden-vector plan"):

* texts are letters-only words (ASCII + Latin-1 accents, >= 3 chars, never a
  stopword) drawn Zipf(s=1.1) from a fixed vocabulary, plus noise the
  reference tokenizer must strip (capitals, punctuation, digits, stopwords) —
  see ``rag/retrieval/bm25.py:34-70``;
* one very common word ("lezione") sits in ~70 % of the chunks so that its
  BM25 IDF is negative and the epsilon floor of rank_bm25 is exercised;
* embeddings are unit-norm Gaussian fp32 rows (the E5 encoder output is
  L2-normalised, ``rag/embeddings/__init__.py:85-105``);
* metadata follows the sanitised form ``rag/pipeline/rag.py:193-224`` writes
  (tags expanded to ``tag_<slug>: True``).
"""
from __future__ import annotations

import numpy as np

ALPHABET = list("abcdefghijklmnopqrstuvwxyz") + list("àèéìòù")
COMMON_WORD = "lezione"
NOISE_STOPWORDS = ["the", "and", "of", "is", "a", "to", "di", "con"]


def make_vocab(v: int, seed: int = 7) -> list[str]:
    from_stop = set(NOISE_STOPWORDS) | {"it", "in", "on", "at", "an", "be"}
    rng = np.random.default_rng(seed)
    out: list[str] = []
    seen = {COMMON_WORD}
    while len(out) < v:
        ln = int(rng.integers(3, 10))
        w = "".join(ALPHABET[int(i)] for i in rng.integers(0, len(ALPHABET), ln))
        if w in seen or w in from_stop:
            continue
        seen.add(w)
        out.append(w)
    return out


def zipf_probs(v: int, s: float = 1.1) -> np.ndarray:
    p = 1.0 / np.arange(1, v + 1, dtype=np.float64) ** s
    return p / p.sum()


def _decorate(words: list[str], rng) -> str:
    """Join words with separators the tokenizer must strip."""
    parts = []
    for w in words:
        r = rng.random()
        if r < 0.08:
            w = w.capitalize()
        elif r < 0.10:
            w = w.upper()
        parts.append(w)
        r = rng.random()
        if r < 0.05:
            parts.append(str(int(rng.integers(0, 999))))       # digits split tokens
        elif r < 0.10:
            parts.append(NOISE_STOPWORDS[int(rng.integers(0, len(NOISE_STOPWORDS)))])
        elif r < 0.13:
            parts.append("x")                                 # len<=1 dropped
    text = ""
    for i, p in enumerate(parts):
        sep = " " if i else ""
        if i and rng.random() < 0.06:
            sep = ", " if rng.random() < 0.5 else ". "
        text += sep + p
    return text


def make_corpus(n: int, dim: int = 768, seed: int = 1234, vocab_size: int = 2000,
                min_len: int = 40, max_len: int = 160, common_frac: float = 0.7):
    """Return (ids, texts, metadatas, embeddings[n, dim] fp32 unit rows)."""
    rng = np.random.default_rng(seed)
    vocab = make_vocab(vocab_size, seed=seed + 1)
    probs = zipf_probs(vocab_size)
    emb = rng.standard_normal((n, dim)).astype(np.float32)
    emb /= np.linalg.norm(emb, axis=1, keepdims=True)
    ids, texts, metas = [], [], []
    courses = ["cs101", "math201", None]
    units = ["u1", "u2", None]
    for i in range(n):
        ln = int(rng.integers(min_len, max_len + 1))
        words = [vocab[int(j)] for j in rng.choice(vocab_size, size=ln, p=probs)]
        if rng.random() < common_frac:
            words.insert(int(rng.integers(0, ln)), COMMON_WORD)
        texts.append(_decorate(words, rng))
        ids.append(f"cm_{i:08x}{int(rng.integers(0, 2**31)):08x}")
        meta = {"language": "en", "doc_type": "pdf" if i % 3 else "pptx",
                "page": int(i // 7), "chunk_id": int(i)}
        c = courses[i % 3]
        if c is not None:
            meta["course"] = c
        u = units[(i // 3) % 3]
        if u is not None:
            meta["unit"] = u
        if i % 5 == 0:
            meta["tag_exam"] = True
        if i % 4 == 1:
            meta["tag_oop"] = True
        metas.append(meta)
    return ids, texts, metas, emb


def make_queries(texts: list[str], emb: np.ndarray, nq: int = 16, seed: int = 99,
                 noise: float = 0.05, q_len: int = 8):
    """Half near-duplicates of corpus rows, half random; text = words of a target doc."""
    import re
    rng = np.random.default_rng(seed)
    n, dim = emb.shape
    targets = rng.integers(0, n, nq)
    qv = np.empty((nq, dim), dtype=np.float32)
    qt = []
    for i, t in enumerate(targets):
        if i < nq // 2:
            v = emb[t] + noise * rng.standard_normal(dim).astype(np.float32)
        else:
            v = rng.standard_normal(dim).astype(np.float32)
        qv[i] = v / np.linalg.norm(v)
        words = re.findall(r"[a-zàèéìòù]+", texts[t].lower())
        words = [w for w in words if len(w) > 2] or ["lezione"]
        pick = [words[int(j)] for j in rng.integers(0, len(words), q_len)]
        if i % 4 == 1:
            pick.append("the")            # stopword dropped by the tokenizer
        if i % 4 == 2:
            pick.append("qqqzzz")         # unknown term scores 0
        if i % 4 == 3:
            pick.append(pick[0])          # duplicate query token counts twice
        qt.append(" ".join(pick))
    return qt, qv, targets
