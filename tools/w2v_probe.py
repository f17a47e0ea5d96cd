"""Word2Vec GPU probe: topic separation vs centers per launch, and training throughput."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from test_word2vec import topic_corpus, topic_separation
from dnn_page_vectors_amd.models.word2vec import Word2Vec, _as_id_corpus

for nt_, wpt_, ns, chunks in ((6, 12, 3000, (1, 256, 1152)), (20, 40, 20000, (1, 1600, 16000, 65536))):
    for chunk in chunks:
        ids, vocab, nt, wpt = topic_corpus(n_topics=nt_, words_per_topic=wpt_, n_sent=ns)
        m = Word2Vec(vocabulary=vocab, size=100, window=4, min_count=1, sample=0.0, iter=5, seed=3, device="cuda",
                     chunk=chunk)
        i2, l2, w2 = _as_id_corpus(ids, vocab)
        m.build_vocab(i2, l2, w2)
        m.min_chunk = chunk
        t = time.time()
        m.train(i2, l2)
        torch.cuda.synchronize()
        print(len(vocab), chunk, topic_separation(m, vocab, nt, wpt), round(time.time() - t, 2), flush=True)

# throughput: 2M-token Zipf corpus, 50k words, D = 300, CBOW, window 10
rng = np.random.default_rng(0)
V = 50000
p = 1.0 / np.arange(1, V + 1)
p /= p.sum()
ids = rng.choice(V, size=(100000, 20), p=p)
vocab = [f"w{i}" for i in range(V)]
for sg in (0, 1):
    t = time.time()
    m = Word2Vec(ids, vocabulary=vocab, size=300, window=10, min_count=1, sample=1e-3, iter=1, seed=1, sg=sg,
                 device="cuda")
    torch.cuda.synchronize()
    dt = time.time() - t
    print({"sg": sg, "words_trained": m.words_trained, "s": round(dt, 3),
           "words_per_s": round(m.words_trained / dt)}, flush=True)
