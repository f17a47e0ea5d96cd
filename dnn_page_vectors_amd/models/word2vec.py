"""Word2Vec trainer (CBOW / skip-gram with negative sampling) — reference C8.

The reference trains, saves and reloads a gensim ``Word2Vec`` and turns it into the
initial weights of the Embedding layer (``train_word2vec``, dssm_cnn_v2/w2v.py:8-53 and
its identical copy dssm_cnn/w2v.py):

* model name ``{num_features}features_{min_word_count}minwords_{context}context`` under
  ``word2vec_models/``; an existing model is loaded instead of retrained (:22-27);
* ``Word2Vec(sentences, workers=2, size=num_features, min_count=min_word_count,
  window=context, sample=1e-3)`` with gensim's defaults otherwise: CBOW (cbow_mean=1),
  5 negatives, alpha 0.025 decaying linearly to 0.0001, 5 passes (:29-39);
* ``init_sims(replace=True)``: rows L2-normalised in place (:43);
* embedding weights ``[array([model[w] if w in model else U(-0.25, 0.25)
  for w in vocabulary_inv])]`` (:50-53).

This module keeps that contract and the gensim-style object API (``model[word]``,
``word in model``, ``most_similar``, ``save``/``load``, ``save_word2vec_format``) with
no gensim dependency.  Training runs on the GPU through the asynchronous-SGD HIP kernel
(``ops/word2vec.py``, ``csrc/kernels/w2v.hip``); the corpus is subsampled and compacted on
the device every epoch (gensim's ``sample`` rule), negatives come from a unigram^0.75
table.  Files: ``<name>.safetensors`` (vectors) + ``<name>.json`` (vocabulary, counts,
hyper-parameters).
"""
from __future__ import annotations

import json
import math
import os
from typing import Dict, Iterable, List, Optional, Sequence, Tuple, Union

import numpy as np
import torch

from ..ops import word2vec as w2v_ops

TABLE_MIN = 1 << 20


class Word2Vec:
    def __init__(self, sentences=None, size: int = 100, window: int = 5, min_count: int = 5,
                 sample: float = 1e-3, negative: int = 5, sg: int = 0, alpha: float = 0.025,
                 min_alpha: float = 0.0001, iter: int = 5, seed: int = 1, workers: Optional[int] = None,
                 vocabulary: Optional[Sequence[str]] = None, device: Optional[Union[str, torch.device]] = None,
                 chunk: int = 1 << 16, ns_exponent: float = 0.75):
        """``sentences``: iterable of token lists, OR an int matrix / list of id lists
        together with ``vocabulary`` (id -> word).  ``workers`` is accepted for gensim
        compatibility (the GPU kernel is the parallelism)."""
        self.vector_size = int(size)
        self.window = int(window)
        self.min_count = int(min_count)
        self.sample = float(sample)
        self.negative = int(negative)
        self.sg = int(sg)
        self.alpha = float(alpha)
        self.min_alpha = float(min_alpha)
        self.iter = int(iter)
        self.seed = int(seed)
        self.chunk = int(chunk)
        self.min_chunk = 256  # floor of the vocabulary-sized centers per launch
        self.ns_exponent = float(ns_exponent)
        if device is None:
            device = "cuda" if torch.cuda.is_available() else "cpu"
        self.device = torch.device(device)
        self.index2word: List[str] = []
        self.counts: np.ndarray = np.zeros(0, dtype=np.int64)
        self.vocab: Dict[str, int] = {}
        self.syn0: Optional[torch.Tensor] = None
        self.syn1neg: Optional[torch.Tensor] = None
        self.normalized = False
        self.words_trained = 0
        if sentences is not None:
            ids, lens, words = _as_id_corpus(sentences, vocabulary)
            self.build_vocab(ids, lens, words)
            self.train(ids, lens)

    # ------------------------------------------------------------------ vocabulary
    def build_vocab(self, ids: np.ndarray, lens: np.ndarray, words: Sequence[str]) -> None:
        """Keep words with count >= min_count, most frequent first (gensim sorts the same
        way); ``self._remap`` maps corpus ids to model indices (-1 = dropped)."""
        counts = np.bincount(ids, minlength=len(words)).astype(np.int64)
        keep = np.nonzero(counts >= self.min_count)[0]
        order = keep[np.lexsort((keep, -counts[keep]))]
        self.index2word = [words[i] for i in order]
        self.counts = counts[order]
        self.vocab = {w: j for j, w in enumerate(self.index2word)}
        remap = np.full(len(words), -1, dtype=np.int64)
        remap[order] = np.arange(len(order))
        self._remap = remap
        V, D = len(order), self.vector_size
        g = torch.Generator().manual_seed(self.seed)
        # gensim: syn0 rows (rand - 0.5) / size, syn1neg zeros
        self.syn0 = ((torch.rand(V, D, generator=g) - 0.5) / D).to(self.device)
        self.syn1neg = torch.zeros(V, D, device=self.device)
        self.normalized = False

    def _table(self) -> torch.Tensor:
        V = len(self.counts)
        size = max(TABLE_MIN, 16 * V)
        p = self.counts.astype(np.float64) ** self.ns_exponent
        cum = np.cumsum(p / p.sum())
        idx = np.searchsorted(cum, (np.arange(size) + 0.5) / size, side="right")
        return torch.from_numpy(np.minimum(idx, V - 1).astype(np.int32)).to(self.device)

    # ------------------------------------------------------------------ training
    def train(self, ids: np.ndarray, lens: np.ndarray, epochs: Optional[int] = None) -> "Word2Vec":
        """Train on a flattened id corpus (vocabulary ids of the CORPUS, remapped here) with
        sentence lengths ``lens``."""
        if self.syn0 is None:
            raise RuntimeError("build_vocab first")
        dev = self.device
        mid = self._remap[ids]
        sid = np.repeat(np.arange(len(lens)), lens)
        kept = mid >= 0  # min_count-filtered words are removed before windowing (gensim)
        words = torch.from_numpy(mid[kept].astype(np.int32)).to(dev)
        sent = torch.from_numpy(sid[kept].astype(np.int64)).to(dev)
        total = int(self.counts.sum())
        if self.sample > 0:  # gensim: keep prob (sqrt(c / t) + 1) * t / c, t = sample * total
            thr = self.sample * total
            c = self.counts.astype(np.float64)
            pk = np.minimum(1.0, (np.sqrt(c / thr) + 1.0) * thr / c)
        else:
            pk = np.ones(len(self.counts))
        pkeep = torch.from_numpy(pk.astype(np.float32)).to(dev)
        table = self._table()
        epochs = self.iter if epochs is None else int(epochs)
        g = torch.Generator(device=dev).manual_seed(self.seed)
        n_all = words.numel()
        for ep in range(epochs):
            keep = torch.rand(n_all, generator=g, device=dev) < pkeep[words.long()]
            cw = words[keep].contiguous()
            cs = sent[keep].contiguous()
            T = cw.numel()
            if T == 0:
                continue
            sbeg = torch.searchsorted(cs, cs, right=False).to(torch.int32)
            send = torch.searchsorted(cs, cs, right=True).to(torch.int32)
            # centers per launch: every center of a launch reads the tables before the others'
            # updates land, so the summed step a row takes grows with chunk / V.  Mean
            # cross-topic cosine on the synthetic topic corpora (tools/w2v_probe.py; lower is
            # better, same-topic ~0.9995 throughout): 72 words 0.38 / 0.57 / 0.71 at 1 / 256 /
            # 1152 centers per launch, 800 words 0.42 / 0.45 / 0.48 at 1 / 1600 / 16000
            chunk = min(self.chunk, max(self.min_chunk, 2 * len(self.counts)))
            for b0 in range(0, T, chunk):
                progress = (ep + b0 / T) / epochs
                alpha = max(self.min_alpha, self.alpha - (self.alpha - self.min_alpha) * progress)
                seed = (self.seed * 1000003 + ep * 7919) & 0xFFFFFFFF
                w2v_ops.train_chunk(cw, sbeg, send, table, self.syn0, self.syn1neg, b0, min(T, b0 + chunk),
                                    self.window, self.negative, seed, alpha, bool(self.sg))
            self.words_trained += T
        self.normalized = False
        return self

    # ------------------------------------------------------------------ gensim-style API
    def init_sims(self, replace: bool = False) -> None:
        n = self.syn0.norm(dim=1, keepdim=True).clamp_min(1e-12)
        if replace:
            self.syn0 = self.syn0 / n
            self.normalized = True
        else:
            self.syn0norm = self.syn0 / n

    def __contains__(self, word: str) -> bool:
        return word in self.vocab

    def __getitem__(self, word: str) -> np.ndarray:
        return self.syn0[self.vocab[word]].float().cpu().numpy()

    @property
    def vectors(self) -> np.ndarray:
        return self.syn0.float().cpu().numpy()

    def similarity(self, a: str, b: str) -> float:
        x, y = self.syn0[self.vocab[a]], self.syn0[self.vocab[b]]
        return float((x @ y) / (x.norm() * y.norm()).clamp_min(1e-12))

    def most_similar(self, word: str, topn: int = 10) -> List[Tuple[str, float]]:
        from ..ops.topk import topk_cos

        n = self.syn0 / self.syn0.norm(dim=1, keepdim=True).clamp_min(1e-12)
        s, i = topk_cos(n[self.vocab[word]][None].contiguous(), n.contiguous(), k=min(topn + 1, n.shape[0]))
        out = [(self.index2word[int(j)], float(v)) for v, j in zip(s[0].tolist(), i[0].tolist())
               if int(j) != self.vocab[word]]
        return out[:topn]

    def save(self, path: str) -> None:
        from safetensors.torch import save_file

        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        save_file({"syn0": self.syn0.float().cpu().contiguous(), "syn1neg": self.syn1neg.float().cpu().contiguous()},
                  path + ".safetensors")
        meta = {k: getattr(self, k) for k in ("vector_size", "window", "min_count", "sample", "negative", "sg",
                                              "alpha", "min_alpha", "iter", "seed", "normalized", "words_trained")}
        meta["index2word"] = self.index2word
        meta["counts"] = self.counts.tolist()
        with open(path + ".json", "w", encoding="utf-8") as f:
            json.dump(meta, f)

    @classmethod
    def load(cls, path: str, device: Optional[Union[str, torch.device]] = None) -> "Word2Vec":
        from safetensors.torch import load_file

        with open(path + ".json", encoding="utf-8") as f:
            meta = json.load(f)
        m = cls(size=meta["vector_size"], window=meta["window"], min_count=meta["min_count"], sample=meta["sample"],
                negative=meta["negative"], sg=meta["sg"], alpha=meta["alpha"], min_alpha=meta["min_alpha"],
                iter=meta["iter"], seed=meta["seed"], device=device)
        t = load_file(path + ".safetensors")
        m.syn0, m.syn1neg = t["syn0"].to(m.device), t["syn1neg"].to(m.device)
        m.index2word = list(meta["index2word"])
        m.counts = np.asarray(meta["counts"], dtype=np.int64)
        m.vocab = {w: j for j, w in enumerate(m.index2word)}
        m.normalized = bool(meta["normalized"])
        m.words_trained = int(meta.get("words_trained", 0))
        return m

    @staticmethod
    def exists(path: str) -> bool:
        return os.path.exists(path + ".safetensors") and os.path.exists(path + ".json")

    def save_word2vec_format(self, path: str) -> None:
        """word2vec text format (``count dim`` header, ``word v1 .. vD`` lines): the format
        ``io/vectors.load_word_vectors`` reads (the reference's ``word_vectors_file``)."""
        W = self.vectors
        with open(path, "w", encoding="utf-8") as f:
            f.write(f"{W.shape[0]} {W.shape[1]}\n")
            for w, row in zip(self.index2word, W):
                if not w or any(ch.isspace() for ch in w):
                    continue  # not representable in the whitespace-separated format
                f.write(w + " " + " ".join(f"{x:.6g}" for x in row) + "\n")


def _as_id_corpus(sentences, vocabulary: Optional[Sequence[str]]) -> Tuple[np.ndarray, np.ndarray, List[str]]:
    """-> (flat int64 ids, per-sentence lengths, id -> word list)."""
    if isinstance(sentences, torch.Tensor):
        sentences = sentences.cpu().numpy()
    if isinstance(sentences, np.ndarray) and sentences.ndim == 2:
        if vocabulary is None:
            raise ValueError("an id matrix needs vocabulary (id -> word)")
        words = _itos(vocabulary)
        lens = np.full(sentences.shape[0], sentences.shape[1], dtype=np.int64)
        return sentences.reshape(-1).astype(np.int64), lens, words
    sents = list(sentences)
    if sents and len(sents[0]) and not isinstance(sents[0][0], str):
        if vocabulary is None:
            raise ValueError("id sentences need vocabulary (id -> word)")
        words = _itos(vocabulary)
        lens = np.array([len(s) for s in sents], dtype=np.int64)
        ids = np.concatenate([np.asarray(s, dtype=np.int64) for s in sents]) if sents else np.zeros(0, np.int64)
        return ids, lens, words
    stoi: Dict[str, int] = {}
    flat: List[int] = []
    lens = []
    for s in sents:
        for w in s:
            flat.append(stoi.setdefault(w, len(stoi)))
        lens.append(len(s))
    words = [None] * len(stoi)
    for w, i in stoi.items():
        words[i] = w
    return np.asarray(flat, dtype=np.int64), np.asarray(lens, dtype=np.int64), words


def _itos(vocabulary) -> List[str]:
    if isinstance(vocabulary, dict):  # id -> word (the reference calls it vocabulary_inv)
        n = max(vocabulary.keys()) + 1
        out = [""] * n
        for i, w in vocabulary.items():
            out[int(i)] = w
        return out
    return list(vocabulary)


def model_name(num_features: int, min_word_count: int, context: int) -> str:
    """dssm_cnn_v2/w2v.py:22."""
    return "{:d}features_{:d}minwords_{:d}context".format(num_features, min_word_count, context)


def train_word2vec(sentence_matrix, vocabulary_inv, num_features: int = 300, min_word_count: int = 1,
                   context: int = 10, model_dir: str = "word2vec_models", seed: int = 1337,
                   device: Optional[Union[str, torch.device]] = None, **kw) -> List[np.ndarray]:
    """The reference function: train (or load) the model, then the embedding weights for
    every vocabulary word (U(-0.25, 0.25) rows for words the model does not know).

    ``sentence_matrix``: int matrix (num_sentences x max_len) or list of id lists;
    ``vocabulary_inv``: id -> word (list or dict).  Extra keyword arguments go to
    ``Word2Vec`` (e.g. ``iter``, ``sg``, ``negative``)."""
    path = os.path.join(model_dir, model_name(num_features, min_word_count, context))
    if Word2Vec.exists(path):
        model = Word2Vec.load(path, device=device)
    else:
        model = Word2Vec(sentence_matrix, vocabulary=vocabulary_inv, size=num_features, min_count=min_word_count,
                         window=context, sample=1e-3, seed=seed, device=device, **kw)
        model.init_sims(replace=True)
        model.save(path)
    words = _itos(vocabulary_inv)
    rng = np.random.default_rng(seed)
    W = np.empty((len(words), model.vector_size), dtype=np.float32)
    vecs = model.vectors
    for i, w in enumerate(words):
        j = model.vocab.get(w)
        W[i] = vecs[j] if j is not None else rng.uniform(-0.25, 0.25, model.vector_size)
    return [W]


__all__ = ["Word2Vec", "train_word2vec", "model_name"]
