import json
import math
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, cwd):
    env = dict(os.environ, PYTHONPATH=ROOT, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    r = subprocess.run([sys.executable, "-m", "dnn_page_vectors_amd"] + args, cwd=cwd, env=env,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    return r.stdout


def test_cli_setup_train_encode(tmp_path):
    rows = [{"q": f"query {i % 7} about topic", "doc_corr": f"topic {i % 7} page text words {i}",
             "doc_incorr": [f"other {j} text" for j in range(3)]} for i in range(40)]
    src = tmp_path / "raw.jsonl"
    src.write_text("\n".join(json.dumps(r) for r in rows) + "\n")
    common = ["--set", f"experiment_root_directory={tmp_path}", "--set", "feature_level=word",
              "--set", "query_length=6", "--set", "document_length=12", "--set", "batch_size=8",
              "--set", "embedding_dim=16", "--set", "hidden_dims=8", "--set", "num_train_samples=24",
              "--set", "num_validation_samples=8", "--set", "nb_epoch=2"]
    _run(["setup", "--input", str(src)] + common, tmp_path)
    # word vectors trained on the split (reference w2v.py), then picked up by `train`
    w = json.loads(_run(["w2v", "--iter", "2", "--window", "3"] + common, tmp_path).strip().splitlines()[-1])
    assert os.path.exists(w["vectors"]) and w["dim"] == 16 and w["words"] > 10
    out = _run(["train"] + common, tmp_path)
    hist = json.loads(out.strip().splitlines()[-1])["history"]
    assert len(hist["loss"]) == 2 and len(hist["val_loss"]) == 2
    assert all(math.isfinite(v) for k in ("loss", "val_loss") for v in hist[k]), hist
    # v1 data path: one in-memory file, Keras validation_split, per-epoch shuffle
    out = _run(["train", "--data", str(src), "--validation-split", "0.25"] + common, tmp_path)
    hist = json.loads(out.strip().splitlines()[-1])["history"]
    assert len(hist["loss"]) == 2 and len(hist["val_loss"]) == 2
    assert all(math.isfinite(v) for k in ("loss", "val_loss") for v in hist[k]), hist
    texts = tmp_path / "pages.txt"
    texts.write_text("topic 3 page text\nother 1 text\n")
    out = _run(["encode", "--input", str(texts), "--output", str(tmp_path / "v.npy")] + common, tmp_path)
    assert json.loads(out.strip().splitlines()[-1])["shape"] == [2, 8]

    # Recall@k on the real validation file (reference: validation pass, cnn_dssm_th.py:189-194)
    r = json.loads(_run(["eval", "--data", "validation"] + common, tmp_path).strip().splitlines()[-1])
    assert set(r) >= {"recall@1", "recall@10", "recall@100", "queries", "pages"} and r["queries"] > 0
    assert 0.0 <= r["recall@1"] <= r["recall@10"] <= r["recall@100"] == 1.0  # fewer pages than 100
    # the same numbers from 2 ranks (rows / pages sharded, page vectors all-gathered over gloo)
    env = dict(os.environ, PYTHONPATH=ROOT, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    p = subprocess.run([sys.executable, "-m", "dnn_page_vectors_amd.launch", "--nproc", "2", "-m",
                        "dnn_page_vectors_amd", "eval", "--data", "validation"] + common, cwd=tmp_path, env=env,
                       capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stderr[-3000:]
    r2 = json.loads([l for l in p.stdout.splitlines() if l.startswith("{")][-1])
    for k in ("recall@1", "recall@10", "recall@100", "queries", "pages"):
        assert r2[k] == r[k], (k, r2, r)


def test_evaluate_pairs_dataset_dedup_and_oracle(tmp_path):
    """A model whose query vector is its page's vector finds every page at rank 1; pages that
    repeat across rows count once."""
    import numpy as np
    import torch

    from dnn_page_vectors_amd.data.dataset import JsonlPairDataset
    from dnn_page_vectors_amd.data.featurize import Featurizer
    from dnn_page_vectors_amd.eval.retrieval import evaluate_pairs_dataset

    rows = [{"q": f"p{i % 5}", "doc_corr": f"p{i % 5}", "doc_incorr": ["n1", "n2", f"p{(i + 1) % 5}"]}
            for i in range(12)]
    f = tmp_path / "v.jsonl"
    f.write_text("\n".join(json.dumps(r) for r in rows) + "\n")
    ds = JsonlPairDataset(str(f), Featurizer("word", hash_size=997), 1, 1, 3)

    class Oracle(torch.nn.Module):
        out_dim = 997

        def encode(self, ids, tower, batch_size=0):
            return torch.nn.functional.one_hot(ids[:, 0].long(), 997).float()

    r = evaluate_pairs_dataset(Oracle(), ds, torch.device("cpu"), ks=(1, 2))
    assert r["queries"] == 12 and r["pages"] == 7  # p0..p4 + n1 + n2
    assert r["recall@1"] == 1.0
    r = evaluate_pairs_dataset(Oracle(), ds, torch.device("cpu"), ks=(1,), include_negatives=False)
    assert r["pages"] == 5


def test_cli_synthetic_train_every_epoch_has_batches(tmp_path):
    """`train --synthetic` over several epochs: every epoch (and its validation pass) runs its
    batches.  The synthetic loader used to restart only when its generator was exhausted, which
    the trainer (it takes exactly steps_per_epoch batches) never does: every other epoch was
    empty and logged NaN."""
    out = _run(["train", "--preset", "reference_char", "--synthetic", "--set", f"experiment_root_directory={tmp_path}",
                "--set", "num_train_samples=64", "--set", "num_validation_samples=32", "--set", "batch_size=16",
                "--set", "nb_epoch=3", "--set", "document_length=24", "--set", "query_length=8"], tmp_path)
    hist = json.loads(out.strip().splitlines()[-1])["history"]
    assert len(hist["loss"]) == 3 and len(hist["val_loss"]) == 3
    assert all(math.isfinite(v) for k in ("loss", "val_loss") for v in hist[k]), hist
    state = json.loads(open(os.path.join(json.loads(out.strip().splitlines()[-1])["model_dir"],
                                         "trainer_state.json")).read())
    assert state["step"] == 3 * 4


def test_loaders_restart_after_a_consumer_stops_at_the_last_batch():
    """A consumer taking exactly the epoch's batches (the trainer) never triggers a generator's
    epilogue: the next epoch index (or fresh=True) must restart the cursor anyway."""
    import torch

    from dnn_page_vectors_amd.data.dataset import SyntheticLoader, _TensorLoader

    class Gen:
        def batch(self, B):
            return torch.zeros(B, 2), torch.zeros(B, 1, 3)

    for loader in (SyntheticLoader(Gen(), 4, 3),
                   _TensorLoader(torch.zeros(12, 2), torch.zeros(12, 1, 3), 4, True, 0, None, 0, 1)):
        for ep in range(3):
            it = loader.epoch_iter(ep)
            assert sum(1 for _ in zip(range(3), it)) == 3, (type(loader), ep)
        it = loader.epoch_iter(0, fresh=True)
        assert sum(1 for _ in zip(range(3), it)) == 3
        it = loader.epoch_iter(0, fresh=True)
        assert sum(1 for _ in zip(range(3), it)) == 3
