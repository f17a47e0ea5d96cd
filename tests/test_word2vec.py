"""Word2Vec trainer (reference C8, dssm_cnn_v2/w2v.py): CPU path (torch oracle) and the
HIP kernel (csrc/kernels/w2v.hip) against that oracle."""
import os

import numpy as np
import pytest
import torch

from dnn_page_vectors_amd.models.word2vec import Word2Vec, model_name, train_word2vec
from dnn_page_vectors_amd.ops import word2vec as wops


def topic_corpus(n_topics=6, words_per_topic=12, n_sent=600, sent_len=12, seed=0):
    """Each sentence draws its words from ONE topic: co-occurring words share a topic."""
    rng = np.random.default_rng(seed)
    vocab = [f"t{t}w{w}" for t in range(n_topics) for w in range(words_per_topic)]
    topic = rng.integers(0, n_topics, n_sent)
    ids = topic[:, None] * words_per_topic + rng.integers(0, words_per_topic, (n_sent, sent_len))
    return ids.astype(np.int64), vocab, n_topics, words_per_topic


def topic_separation(model, vocab, n_topics, wpt):
    V = np.stack([model[w] for w in vocab])
    V = V / np.linalg.norm(V, axis=1, keepdims=True)
    S = V @ V.T
    t = np.repeat(np.arange(n_topics), wpt)
    same = (t[:, None] == t[None, :]) & ~np.eye(len(vocab), dtype=bool)
    diff = t[:, None] != t[None, :]
    return float(S[same].mean()), float(S[diff].mean())


@pytest.mark.parametrize("sg", [0, 1])
def test_word2vec_learns_topics_cpu(sg):
    ids, vocab, nt, wpt = topic_corpus()
    m = Word2Vec(ids, vocabulary=vocab, size=32, window=4, min_count=1, sample=0.0, negative=5, sg=sg, iter=6,
                 seed=3, device="cpu", chunk=2048)
    same, diff = topic_separation(m, vocab, nt, wpt)
    assert same > diff + 0.3, (same, diff)
    nb = [w for w, _ in m.most_similar("t2w3", topn=5)]
    assert sum(w.startswith("t2w") for w in nb) >= 4, nb


def test_min_count_and_subsampling_rules():
    ids, vocab, _, _ = topic_corpus(n_sent=50)
    extra = vocab + ["rare"]
    ids2 = np.concatenate([ids, np.full((1, ids.shape[1]), len(vocab))])  # "rare" = one sentence only
    ids2[-1, 1:] = 0
    m = Word2Vec(ids2, vocabulary=extra, size=8, window=2, min_count=2, iter=1, device="cpu")
    assert "rare" not in m and "t0w0" in m
    # most frequent first, like gensim's sorted vocabulary
    assert list(m.counts) == sorted(m.counts, reverse=True)


def test_train_word2vec_reference_contract(tmp_path):
    ids, vocab, _, _ = topic_corpus(n_sent=120)
    vocab_inv = vocab + ["never_seen"]  # a vocabulary word absent from the corpus
    d = str(tmp_path / "word2vec_models")
    [W] = train_word2vec(ids, vocab_inv, num_features=16, min_word_count=1, context=3, model_dir=d, device="cpu",
                         iter=2)
    path = os.path.join(d, model_name(16, 1, 3))
    assert os.path.exists(path + ".safetensors") and os.path.exists(path + ".json")
    assert W.shape == (len(vocab_inv), 16)
    # init_sims(replace=True): trained rows are unit vectors; the unknown word is U(-0.25, 0.25)
    np.testing.assert_allclose(np.linalg.norm(W[:-1], axis=1), 1.0, rtol=1e-5)
    assert np.abs(W[-1]).max() <= 0.25 and np.linalg.norm(W[-1]) != pytest.approx(1.0)
    mtime = os.path.getmtime(path + ".safetensors")
    [W2] = train_word2vec(ids, vocab_inv, num_features=16, min_word_count=1, context=3, model_dir=d, device="cpu")
    assert os.path.getmtime(path + ".safetensors") == mtime  # loaded, not retrained
    np.testing.assert_array_equal(W[:-1], W2[:-1])


def test_word2vec_text_format_roundtrip(tmp_path):
    from dnn_page_vectors_amd.data.text import Vocab
    from dnn_page_vectors_amd.io.vectors import load_word_vectors

    ids, vocab, _, _ = topic_corpus(n_sent=60)
    m = Word2Vec(ids, vocabulary=vocab, size=8, window=2, min_count=1, iter=1, device="cpu")
    f = str(tmp_path / "vec.txt")
    m.save_word2vec_format(f)
    W, found = load_word_vectors(f, Vocab(vocab), 8)
    assert found == len(vocab)
    v = Vocab(vocab)
    np.testing.assert_allclose(W[v.lookup("t1w2")], m["t1w2"], rtol=1e-5, atol=1e-6)


def test_save_load_roundtrip(tmp_path):
    ids, vocab, _, _ = topic_corpus(n_sent=40)
    m = Word2Vec(ids, vocabulary=vocab, size=8, window=2, min_count=1, iter=1, device="cpu")
    p = str(tmp_path / "m")
    m.save(p)
    m2 = Word2Vec.load(p, device="cpu")
    assert m2.index2word == m.index2word
    np.testing.assert_array_equal(m2.vectors, m.vectors)


def _sequential_case(sg, D=40, T=64, V=50, window=3, negative=4, seed=11):
    g = torch.Generator().manual_seed(seed)
    words = torch.randint(0, V, (T,), generator=g).to(torch.int32)
    sid = torch.repeat_interleave(torch.arange(4), T // 4)
    sbeg = torch.searchsorted(sid, sid).to(torch.int32)
    send = torch.searchsorted(sid, sid, right=True).to(torch.int32)
    table = torch.randint(0, V, (257,), generator=g).to(torch.int32)
    win = (torch.rand(V, D, generator=g) - 0.5) / D
    wout = (torch.rand(V, D, generator=g) - 0.5) * 0.1
    return words, sbeg, send, table, win, wout, window, negative


@pytest.mark.gpu
@pytest.mark.parametrize("sg", [0, 1])
@pytest.mark.parametrize("D", [40, 300])
def test_w2v_kernel_matches_torch_oracle(sg, D):
    words, sbeg, send, table, win, wout, window, negative = _sequential_case(sg, D=D)
    cpu = [t.clone() for t in (win, wout)]
    gpu = [t.clone().cuda() for t in (win, wout)]
    dw = [t.cuda() for t in (words, sbeg, send, table)]
    # one center per launch: the kernel is then exactly sequential SGD
    for i in range(words.numel()):
        wops.train_chunk_torch(words, sbeg, send, table, cpu[0], cpu[1], i, i + 1, window, negative, 77, 0.05, sg)
        wops.train_chunk(*dw, gpu[0], gpu[1], i, i + 1, window, negative, 77, 0.05, sg)
    torch.testing.assert_close(gpu[0].cpu(), cpu[0], rtol=1e-4, atol=2e-6)
    torch.testing.assert_close(gpu[1].cpu(), cpu[1], rtol=1e-4, atol=2e-6)
    assert not torch.equal(cpu[0], win)  # something was trained


@pytest.mark.gpu
def test_word2vec_gpu_learns_topics():
    # 800 words: launches of 2 V centers train like sequential SGD (a 72-word vocabulary is
    # too small for concurrent updates: tools/w2v_probe.py)
    ids, vocab, nt, wpt = topic_corpus(n_topics=20, words_per_topic=40, n_sent=20000)
    m = Word2Vec(ids, vocabulary=vocab, size=100, window=4, min_count=1, sample=0.0, iter=5, seed=3, device="cuda")
    same, diff = topic_separation(m, vocab, nt, wpt)
    assert same > diff + 0.3, (same, diff)
