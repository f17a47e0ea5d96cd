"""Pure-Python text featurization rules (the specification the native featurizer matches).

Behaviour re-stated from the reference tokenizer ``utils/data_utils.py``:

* ``clean_str`` (data_utils.py:11-19): every character NOT in
  ``[\\wäöüß€#\\n.$]`` becomes one space (no collapsing), then ``strip()`` and
  ``lower()``.
* ``get_text_feature_splits`` (data_utils.py:21-55): ``word`` splits on a
  single ``" "`` (so runs of spaces yield empty tokens), ``char`` takes every
  code point, ``ngram`` takes overlapping 3-code-point windows crossing spaces.
  ``cutoff`` truncates.
* ``pad_sentences`` (data_utils.py:57-68): right-pad with ``<PAD/>``.
* ``build_vocab`` (data_utils.py:70-81): tokens by descending count.
* ``build_input_data`` (data_utils.py:83-92): dict lookup (OOV -> ``None`` in
  the reference; here OOV -> the ``<UNK/>`` id, a documented fix).

New: hashed ids (DSSM "word hashing") ``id = 1 + fnv1a32(utf8(token)) % (V-1)``
with id 0 reserved for padding, used by the 30k-trigram configs.

``normalize_html_line`` re-states ``utils/word2vec_normalizer.py:116-146``
(HTML unescape/strip, dot normalisation, non-alphanumeric removal, whitespace
collapse) for the optional ``html_normalize`` mode.
"""
from __future__ import annotations

import html
import itertools
import re
from collections import Counter
from html.parser import HTMLParser
from typing import Dict, Iterable, List, Optional, Sequence

PAD = "<PAD/>"
UNK = "<UNK/>"
SPACE = " "

MODES = {"word": 0, "ngram": 1, "char": 2}

_CLEAN_RGX = re.compile(r"[^\wäöüß€#\n.$]", re.UNICODE)
_W2V_RGX = re.compile(r"[^\wäöüß€\n.$]", re.UNICODE)
_DOTS = re.compile(r"(\.+)")
_SPACES = re.compile(r"(\s+)")


def clean_str(s: str) -> str:
    return _CLEAN_RGX.sub(" ", s).strip().lower()


def split_features(text: str, mode: str = "word", cutoff: Optional[int] = None, ngram: int = 3,
                   cleaned: bool = False) -> List[str]:
    """Tokens of one text (the single-string branch of get_text_feature_splits)."""
    t = text if cleaned else clean_str(text)
    if mode == "word":
        toks = t.split(" ")
    elif mode == "ngram":
        toks = [t[i:i + ngram] for i in range(len(t) - ngram + 1)]
    elif mode == "char":
        toks = list(t)
    else:
        raise ValueError(f"unknown feature mode {mode!r}")
    return toks[:cutoff]


def pad_tokens(tokens: List[str], length: int, padding_word: str = PAD) -> List[str]:
    return tokens + [padding_word] * (length - len(tokens))


def build_vocab_counts(sentences: Iterable[Sequence[str]]) -> List[str]:
    """Tokens by descending count; ties broken lexicographically (deterministic)."""
    c = Counter(itertools.chain(*sentences))
    return [w for w, _ in sorted(c.items(), key=lambda kv: (-kv[1], kv[0]))]


def fnv1a32(b: bytes) -> int:
    h = 0x811C9DC5
    for x in b:
        h ^= x
        h = (h * 0x01000193) & 0xFFFFFFFF
    return h


def hash_token(tok: str, size: int) -> int:
    if tok == PAD:
        return 0
    return 1 + fnv1a32(tok.encode("utf-8")) % (size - 1)


class Vocab:
    """Deterministic token -> id map. id 0 is always ``<PAD/>``, 1 ``<UNK/>``, 2 ``' '``.

    (The reference assigns ids in set-iteration order, data_helpers.py:109-118,
    which is non-deterministic under Python 3 hash seeding.)
    """

    def __init__(self, tokens: Sequence[str] = ()):  # tokens beyond the reserved ones
        self.itos: List[str] = [PAD, UNK, SPACE]
        self.stoi: Dict[str, int] = {t: i for i, t in enumerate(self.itos)}
        for t in tokens:
            self.add(t)

    def add(self, tok: str) -> int:
        i = self.stoi.get(tok)
        if i is None:
            i = len(self.itos)
            self.itos.append(tok)
            self.stoi[tok] = i
        return i

    def __len__(self) -> int:
        return len(self.itos)

    def lookup(self, tok: str) -> int:
        return self.stoi.get(tok, 1)

    @property
    def pad_id(self) -> int:
        return 0

    @property
    def unk_id(self) -> int:
        return 1

    def to_json(self) -> List[str]:
        return list(self.itos)

    @classmethod
    def from_json(cls, itos: Sequence[str]) -> "Vocab":
        v = cls()
        if list(itos[:3]) != v.itos:
            raise ValueError("vocab json must start with the reserved tokens")
        for t in itos[3:]:
            v.add(t)
        return v


def featurize_py(texts: Sequence[str], mode: str, length: int, vocab: Optional[Vocab] = None,
                 hash_size: int = 0, html: bool = False) -> List[List[int]]:
    """Reference (slow) featurizer: [normalise HTML ->] clean -> split -> cutoff -> pad -> ids."""
    out = []
    for t in texts:
        if html:
            t = normalize_html_line(t)
        toks = pad_tokens(split_features(t, mode, cutoff=length), length)
        if hash_size > 0:
            out.append([hash_token(x, hash_size) for x in toks])
        elif vocab is not None:
            out.append([vocab.lookup(x) for x in toks])
        else:
            raise ValueError("need a vocab or hash_size > 0")
    return out


# ---- HTML / word2vec normaliser (utils/word2vec_normalizer.py) ----------------
class _Stripper(HTMLParser):
    def __init__(self) -> None:
        super().__init__(convert_charrefs=True)
        self.fed: List[str] = []

    def handle_data(self, d: str) -> None:
        self.fed.append(d)


def normalize_html_line(line: str) -> str:
    if line.strip() == "":
        return line
    s = line.strip()
    for ent in (";lt;", ";gt;", ";amp;", ";apos;", ";quot;"):
        s = s.replace(ent, "")
    s = html.unescape(s)
    p = _Stripper()
    p.feed(s)
    p.close()
    s = "".join(p.fed)
    s = s.replace("\n", "").replace("\r", "").replace("\t", "")
    s = _DOTS.sub(".", s).replace(".", " . ")
    s = " ".join(_W2V_RGX.sub(" ", w.strip().lower()) for w in s.split(" "))
    return _SPACES.sub(" ", s)
