"""BM25 tokenizer — same rules as rag/retrieval/bm25.py:34-70 (host side).

Letters-only regex (ASCII + Latin-1 accents), lowercase, EN or IT stopwords
(IT when the language hint starts with "it"), tokens of length <= 1 dropped.
Tokenization stays on the CPU; the host maps tokens to int32 term ids that the
device postings use.
"""
from __future__ import annotations

import re
from typing import List, Optional

_TOKEN_RE = re.compile(r"[A-Za-zÀ-ÖØ-öø-ÿ]+")

_STOP_EN = frozenset("""
a an the and or but if then else for to of in on at by with from as is are was were be been being
it its this that these those i you he she we they them his her their my your our me us not no yes do
does did doing can could should would may might will shall about into over under again further there
here when where why how what which who whom""".split())

_STOP_IT = frozenset("""
un uno una le la il lo gli i l e o ma se allora altrimenti per di a da in su con come è era sono siamo
siete fui fu furono essere stato questo questa questi queste quello quella quelli quelle ciò cio io tu
lui lei noi voi loro mio mia tuo tua suo sua nostro vostro non no si sia fare fa fatto posso può puo
puoi possono dovrebbe potrebbe sarà sara sarebbe saremmo sarete siano che perché perche quando dove
cosa quale chi""".split())


def _choose_stopwords(lang_hint: Optional[str]) -> frozenset:
    return _STOP_IT if (lang_hint or "").lower().startswith("it") else _STOP_EN


_ASCII_RE = re.compile(r"[a-z]+")


def _tokenize(text: str, lang_hint: Optional[str] = None) -> List[str]:
    sw = _choose_stopwords(lang_hint)
    text = text or ""
    if text.isascii():
        # same tokens: on ASCII text case never decides membership in the letter class, so the
        # whole string can be lowered first (2.5x faster; non-ASCII text keeps the per-match path,
        # where lowering first would differ, e.g. U+212A KELVIN SIGN -> "k")
        return [t for t in _ASCII_RE.findall(text.lower()) if t not in sw and len(t) > 1]
    return [t for t in (m.group(0).lower() for m in _TOKEN_RE.finditer(text)) if t not in sw and len(t) > 1]


_LANGDETECT = None  # (DetectorFactory, detect) once imported; False when the package is absent


def _langdetect():
    global _LANGDETECT
    if _LANGDETECT is None:
        try:
            from langdetect import DetectorFactory, detect
            _LANGDETECT = (DetectorFactory, detect)
        except Exception:  # absent: every text is 'en' (the reference's except branch)
            _LANGDETECT = False
    return _LANGDETECT


def detect_lang_tag(text: str) -> str:
    """rag/utils/lang_detect.py:16-24: langdetect (seed 42) restricted to en/it, 'en' otherwise.
    The import is attempted once per process (a failed import per call cost ~60 us per query)."""
    ld = _langdetect()
    if not ld:
        return "en"
    try:
        ld[0].seed = 42
        lang = ld[1](text or "")
        return lang if lang in ("en", "it") else "en"
    except Exception:
        return "en"
