import json

import numpy as np
import pytest
import torch

from dnn_page_vectors_amd.data import text as T
from dnn_page_vectors_amd.data.dataset import JsonlPairDataset, PairLoader
from dnn_page_vectors_amd.data.featurize import Featurizer


def _write(tmp_path, n=37, bad_every=5):
    rows = []
    for i in range(n):
        negs = [f"neg {i} a", f"neg {i} b ü", f"neg {i} c"] if (i % bad_every) != bad_every - 1 else [f"only {i}"]
        rows.append({"q": f"Query {i}!", "doc_corr": f"Page about {i}, \"quoted\" \\ backslash é",
                     "doc_incorr": negs, "extra": {"nested": [1, 2, {"x": "y"}]}})
    p = tmp_path / "data.jsonl"
    p.write_text("\n".join(json.dumps(r) for r in rows) + "\n\n")
    return str(p), rows


def test_native_dataset_reads_and_skips(tmp_path):
    path, rows = _write(tmp_path)
    fz = Featurizer("char", hash_size=997)
    ds = JsonlPairDataset(path, fz, 12, 30, 3)
    good = [r for r in rows if len(r["doc_incorr"]) == 3]
    assert len(ds) == len(good) and ds.skipped == len(rows) - len(good)
    q, d = ds.batch(np.arange(len(ds)))
    assert q.shape == (len(good), 12) and d.shape == (len(good), 4, 30)
    for i, r in enumerate(good):
        np.testing.assert_array_equal(q[i], T.featurize_py([r["q"]], "char", 12, hash_size=997)[0])
        texts = [r["doc_corr"]] + r["doc_incorr"]
        np.testing.assert_array_equal(d[i], np.array(T.featurize_py(texts, "char", 30, hash_size=997)))
    assert ds.texts(0)[1] == good[0]["doc_corr"]


def test_loader_sequential_shuffle_shard_resume(tmp_path):
    path, rows = _write(tmp_path, n=64, bad_every=1000)
    fz = Featurizer("word", hash_size=101)
    ds = JsonlPairDataset(path, fz, 5, 9, 3)
    seq = [q for q, _ in PairLoader(ds, 8).epoch_iter()]
    assert len(seq) == 8
    ref_q, _ = ds.batch(np.arange(8))
    assert torch.equal(seq[0], torch.from_numpy(ref_q))
    sh = PairLoader(ds, 8, shuffle=True, seed=3)
    a = [q for q, _ in sh.epoch_iter(0)]
    b = [q for q, _ in PairLoader(ds, 8, shuffle=True, seed=3).epoch_iter(0)]
    assert all(torch.equal(x, y) for x, y in zip(a, b))
    assert not all(torch.equal(x, y) for x, y in zip(a, seq))
    # rank shards are disjoint halves
    r0 = torch.cat([q for q, _ in PairLoader(ds, 8, rank=0, world_size=2).epoch_iter()])
    r1 = torch.cat([q for q, _ in PairLoader(ds, 8, rank=1, world_size=2).epoch_iter()])
    assert r0.shape[0] == r1.shape[0] == 32 and not torch.equal(r0, r1)
    # resume mid-epoch
    ld = PairLoader(ds, 8, shuffle=True, seed=3)
    it = ld.epoch_iter(0)
    first = [next(it) for _ in range(3)]
    st = ld.state()
    it.close()
    ld2 = PairLoader(ds, 8, shuffle=True, seed=3)
    ld2.load_state(st)
    rest = [q for q, _ in ld2.epoch_iter()]
    assert len(rest) == 5 and torch.equal(rest[0], a[3])


def test_dataset_missing_file(tmp_path):
    with pytest.raises(FileNotFoundError):
        JsonlPairDataset(str(tmp_path / "nope.jsonl"), Featurizer("char", hash_size=10), 4, 4, 3)


def test_in_memory_pairs_v1_semantics(tmp_path):
    """v1 data path (dssm_cnn/data_helpers.py + cnn_dssm.py:201): pad to the dataset's longest
    text (capped by the configured lengths), Keras validation_split = the LAST rows, a fresh
    shuffle of the training rows every epoch."""
    import json

    import numpy as np

    from dnn_page_vectors_amd.data.dataset import InMemoryPairs
    from dnn_page_vectors_amd.data.featurize import Featurizer

    rows = [{"q": "w " * (1 + i % 4), "doc_corr": "d " * (2 + i % 7), "doc_incorr": ["x", "y y", "z"]}
            for i in range(20)]
    rows.append({"q": "bad", "doc_corr": "row", "doc_incorr": ["only one"]})  # skipped (!= 3 negatives)
    p = tmp_path / "v1.jsonl"
    p.write_text("\n".join(json.dumps(r) for r in rows) + "\n")
    fz = Featurizer("word", hash_size=97)
    mem = InMemoryPairs(str(p), fz, 64, 64, 3, validation_split=0.25)
    assert len(mem) == 20 and mem.skipped == 1
    assert mem.n_val == 5 and mem.n_train == 15
    assert mem.query_length == 4 and mem.document_length == 8  # "w w w w" / 8 tokens ("d " * 8 -> 8 + '')
    tl = mem.train_loader(5, shuffle=True, seed=3)
    e0 = torch.cat([q for q, _ in tl.epoch_iter()])
    e1 = torch.cat([q for q, _ in tl.epoch_iter()])
    assert e0.shape == (15, 4) and not torch.equal(e0, e1)           # reshuffled per epoch
    assert sorted(map(tuple, e0.tolist())) == sorted(map(tuple, e1.tolist()))
    vq = torch.cat([q for q, _ in mem.val_loader(5).epoch_iter()])
    np.testing.assert_array_equal(vq.numpy(), mem.q[15:].numpy())    # the last 25% in file order


def test_in_memory_split_and_partial_batch_follow_keras(tmp_path):
    """Keras fit(validation_split=s): split_at = int(n * (1 - s)) (n = 7, s = 0.2 -> 5 train, 2
    validation rows), and the last partial batch is trained on."""
    import json

    from dnn_page_vectors_amd.data.dataset import InMemoryPairs
    from dnn_page_vectors_amd.data.featurize import Featurizer

    rows = [{"q": f"q{i}", "doc_corr": f"d{i}", "doc_incorr": ["x", "y", "z"]} for i in range(7)]
    p = tmp_path / "k.jsonl"
    p.write_text("\n".join(json.dumps(r) for r in rows) + "\n")
    mem = InMemoryPairs(str(p), Featurizer("word", hash_size=97), 8, 8, 3, validation_split=0.2)
    assert (mem.n_train, mem.n_val) == (5, 2)
    tl = mem.train_loader(2, shuffle=False)
    sizes = [q.shape[0] for q, _ in tl.epoch_iter()]
    assert sizes == [2, 2, 1] and tl.num_batches() == 3
    assert mem.train_loader(2, shuffle=False, drop_last=True).num_batches() == 2


def test_legacy_config_json_migrates_fp32_default(tmp_path, caplog):
    """A config saved before config_version existed with dtype='fp32' is ambiguous (the old
    no-op default before 066a651, or reference precision chosen on purpose after it; no field
    tells them apart): it keeps fp32 and warns, a current file keeps fp32 silently."""
    import json

    from dnn_page_vectors_amd.config import Configuration

    d = Configuration().to_dict()
    d.pop("config_version")
    d["dtype"] = "fp32"
    old = tmp_path / "old.json"
    old.write_text(json.dumps(d))
    c = Configuration.load_json(str(old))
    assert c.dtype == "fp32" and c.config_version == 2
    assert any("version-1" in r.message for r in caplog.records)
    new = tmp_path / "new.json"
    Configuration(dtype="fp32").save_json(str(new))
    assert Configuration.load_json(str(new)).dtype == "fp32"
