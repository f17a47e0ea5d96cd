import json
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
    texts = tmp_path / "pages.txt"
    texts.write_text("topic 3 page text\nother 1 text\n")
    out = _run(["encode", "--input", str(texts), "--output", str(tmp_path / "v.npy")] + common, tmp_path)
    assert json.loads(out.strip().splitlines()[-1])["shape"] == [2, 8]
