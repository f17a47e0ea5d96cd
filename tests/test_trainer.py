"""Trainer: Keras-style history, reference checkpoint layout, resume after an injected
fault (bitwise on CPU), NaN/inf step skipping."""
import json
import os

import pytest
import torch

from dnn_page_vectors_amd.config import Configuration
from dnn_page_vectors_amd.io import checkpoint as ck
from dnn_page_vectors_amd.models.cdssm import CDSSM
from dnn_page_vectors_amd.parallel import dist as pdist
from dnn_page_vectors_amd.train.trainer import InjectedFault, Trainer


def _cfg(tmp_path, **kw):
    base = dict(experiment_root_directory=str(tmp_path), feature_level="ngram", vocab_hash_size=200,
                query_length=10, document_length=24, batch_size=8, num_filters=150, embedding_dim=16,
                hidden_dims=32, num_train_samples=32, num_validation_samples=16, nb_epoch=2)
    base.update(kw)
    return Configuration(**base)


def _batches(seed_base):
    def make(epoch):
        g = torch.Generator().manual_seed(seed_base + 1000 * epoch)
        for _ in range(100):
            q = torch.randint(1, 200, (8, 10), generator=g, dtype=torch.int32)
            d = torch.randint(1, 200, (8, 4, 24), generator=g, dtype=torch.int32)
            d[:, 0, :10] = q
            yield q, d
    return make


@pytest.fixture(autouse=True)
def _single():
    pdist.init_distributed(device="cpu")


def test_fit_history_and_checkpoint_layout(tmp_path):
    cfg = _cfg(tmp_path)
    tr = Trainer(cfg, CDSSM(cfg, 200))
    hist = tr.fit(_batches(1), validation_batches=_batches(99), callbacks=[ck.ModelCheckpoint(cfg.trained_model_dir)])
    assert set(hist) == {"loss", "acc", "val_loss", "val_acc"} and len(hist["loss"]) == 2
    files = set(os.listdir(cfg.trained_model_dir))
    assert {"weights.01.safetensors", "weights.02.safetensors", "trainer_state.json"} <= files
    full, arch, wts = ck.save_final(tr, cfg.trained_model_dir)
    assert os.path.basename(full) == "cnn_model_dssm.safetensors"
    assert os.path.basename(arch) == "cnn_dssm_model_only.json"
    assert os.path.basename(wts) == "cnn_dssm_model_weights.safetensors"
    a = json.load(open(arch))
    assert a["class"] == "CDSSM" and "query_tower.embedding" in a["params"]
    # reload into a fresh model: identical encodings
    m2 = CDSSM(cfg, 200)
    ck.load_weights(m2, wts)
    ids = torch.randint(1, 200, (5, 24), dtype=torch.int32)
    torch.testing.assert_close(tr.model.encode(ids), m2.encode(ids), rtol=0, atol=0)


def test_resume_after_injected_fault_is_exact(tmp_path, monkeypatch):
    cfg_a = _cfg(tmp_path / "a", nb_epoch=3)
    ta = Trainer(cfg_a, CDSSM(cfg_a, 200))
    ta.fit(_batches(5), callbacks=[ck.ModelCheckpoint(cfg_a.trained_model_dir)])

    cfg_b = _cfg(tmp_path / "b", nb_epoch=3)
    monkeypatch.setenv("PAGEVEC_FAULT_STEP", "9")  # mid epoch 3 (4 steps per epoch)
    tb = Trainer(cfg_b, CDSSM(cfg_b, 200))
    with pytest.raises(InjectedFault):
        tb.fit(_batches(5), callbacks=[ck.ModelCheckpoint(cfg_b.trained_model_dir)])
    monkeypatch.delenv("PAGEVEC_FAULT_STEP")
    tc = Trainer(cfg_b, CDSSM(cfg_b, 200))
    assert ck.resume(tc, cfg_b.trained_model_dir)
    assert (tc.epoch, tc.step) == (2, 8)
    tc.fit(_batches(5), callbacks=[ck.ModelCheckpoint(cfg_b.trained_model_dir)])
    assert tc.step == ta.step == 12
    torch.testing.assert_close(tc.flat.data, ta.flat.data, rtol=0, atol=0)
    torch.testing.assert_close(tc.opt.m, ta.opt.m, rtol=0, atol=0)


def test_nonfinite_gradient_skips_step(tmp_path):
    cfg = _cfg(tmp_path)
    tr = Trainer(cfg, CDSSM(cfg, 200))
    q, d = next(_batches(3)(0))
    before = tr.flat.data.clone()
    h = tr.model.query_tower.dense_b.register_hook(lambda g: g * float("nan"))
    m = tr.train_step(q, d)
    h.remove()
    assert float(m["nonfinite"]) == 1.0
    torch.testing.assert_close(tr.flat.data, before, rtol=0, atol=0)
    m = tr.train_step(q, d)
    assert float(m["nonfinite"]) == 0.0 and not torch.equal(tr.flat.data, before)


def test_metrics_jsonl_has_step_breakdown(tmp_path):
    from dnn_page_vectors_amd.utils.metrics import MetricsLogger

    cfg = _cfg(tmp_path, log_every=2, nb_epoch=1)
    ml = MetricsLogger(str(tmp_path / "m.jsonl"))
    tr = Trainer(cfg, CDSSM(cfg, 200), metrics=ml)
    tr.fit(_batches(3))
    recs = [r for r in ml.read() if "step" in r]  # per-step records (epoch summaries have no "step")
    assert [r["step"] for r in recs] == [2, 4]
    for r in recs:
        for k in ("forward_ms", "backward_ms", "allreduce_ms", "optimizer_ms", "step_ms", "pairs_per_s", "hbm_gb"):
            assert k in r, r
        assert abs(r["step_ms"] - (r["forward_ms"] + r["backward_ms"] + r["allreduce_ms"] + r["optimizer_ms"])) < 0.01


def test_lazy_embedding_adam_keeps_untouched_rows(tmp_path):
    """cfg.lazy_embedding_adam: an embedding row whose tokens are absent from a step keeps its
    weights (dense Adam would keep moving it on its momentum); dense parameters still train."""
    moved = {}
    for lazy in (True, False):
        cfg = _cfg(tmp_path).replace(lazy_embedding_adam=lazy, dropout_prob=(0.0, 0.0))
        torch.manual_seed(0)
        tr = Trainer(cfg, CDSSM(cfg, 200))
        assert bool(tr.opt.lazy) == lazy
        emb = tr.model.doc_towers[0].embedding
        g = torch.Generator().manual_seed(0)
        q = torch.randint(1, 150, (cfg.batch_size, cfg.query_length), dtype=torch.int32, generator=g)
        d1 = torch.randint(1, 150, (cfg.batch_size, cfg.J + 1, cfg.document_length), dtype=torch.int32, generator=g)
        d2 = torch.randint(1, 100, (cfg.batch_size, cfg.J + 1, cfg.document_length), dtype=torch.int32, generator=g)
        tr.train_step(q, d1)
        after1 = emb.detach().clone()
        conv1 = tr.model.doc_towers[0].conv_w[0].detach().clone()
        tr.train_step(q, d2)
        moved[lazy] = float((emb.detach()[100:150] - after1[100:150]).abs().max())
        assert not torch.equal(emb.detach()[1:100], after1[1:100])
        assert not torch.equal(tr.model.doc_towers[0].conv_w[0].detach(), conv1)
    assert moved[True] == 0.0 and moved[False] > 0.0, moved


def test_inbatch_gamma_overrides_gamma_for_inbatch_losses_only():
    """cfg.inbatch_gamma is the softmax scale of the in-batch / cross-GPU losses (new modes);
    the reference's GAMMA keeps driving the explicit 1 + J head."""
    pdist.set_info(pdist.DistInfo(device=torch.device("cpu")))
    g = torch.Generator().manual_seed(2)
    q = torch.randint(1, 300, (8, 12), generator=g, dtype=torch.int32)
    d = torch.randint(1, 300, (8, 4, 30), generator=g, dtype=torch.int32)
    base = dict(feature_level="ngram", vocab_hash_size=300, query_length=12, document_length=30, batch_size=8,
                embedding_dim=24, hidden_dims=32, cos_clip=False)
    losses = {}
    for name, kw in {"ib_override": dict(loss_mode="in_batch", inbatch_gamma=40.0),
                     "ib_gamma": dict(loss_mode="in_batch", GAMMA=40.0),
                     "ib_default": dict(loss_mode="in_batch"),
                     "ex_override": dict(loss_mode="explicit", inbatch_gamma=40.0),
                     "ex_default": dict(loss_mode="explicit")}.items():
        torch.manual_seed(0)
        cfg = Configuration(**base, **kw)
        tr = Trainer(cfg, CDSSM(cfg, 300), torch.device("cpu"))
        with torch.no_grad():
            losses[name] = float(tr.compute_loss(q, d, seed=3)[0])
    assert losses["ib_override"] == losses["ib_gamma"]
    assert losses["ib_override"] != losses["ib_default"]
    assert losses["ex_override"] == losses["ex_default"]


def test_sparse_embedding_grad_single_process_matches_lazy():
    """One process: sparse-gradient tables (only touched rows zeroed / checked / updated)
    train exactly like LazyAdam over dense table gradients, and leave the untouched rows'
    gradient zero between steps."""
    import torch

    from dnn_page_vectors_amd.config import Configuration
    from dnn_page_vectors_amd.models.cdssm import CDSSM
    from dnn_page_vectors_amd.parallel import dist as pdist
    from dnn_page_vectors_amd.train.trainer import Trainer

    pdist.set_info(pdist.DistInfo())
    V = 5000
    res = []
    for sparse in (True, False):
        cfg = Configuration(feature_level="ngram", vocab_hash_size=V, query_length=8, document_length=16,
                            batch_size=8, embedding_dim=12, hidden_dims=16, dropout_prob=(0.25, 0.5),
                            loss_mode="in_batch", lazy_embedding_adam=True, sparse_embedding_grad=sparse)
        tr = Trainer(cfg, CDSSM(cfg, V))
        g = torch.Generator().manual_seed(1)
        for _ in range(3):
            m = tr.train_step(torch.randint(1, V, (8, 8), generator=g, dtype=torch.int32),
                              torch.randint(1, V, (8, 4, 16), generator=g, dtype=torch.int32))
        res.append((tr.flat.data.clone(), float(m["grad_sumsq"])))
        if sparse:
            t = tr.sparse.tables["query_tower.embedding"]
            g2 = tr.sparse.grad2d(t).clone()
            rows = t.rows[t.rows >= 0].long()  # fixed-size list, -1 padded
            mask = torch.ones(V, dtype=torch.bool)
            mask[rows] = False
            assert g2[mask].abs().sum() == 0 and g2[rows].abs().sum() > 0
    torch.testing.assert_close(res[0][0], res[1][0], rtol=0, atol=0)
    assert abs(res[0][1] - res[1][1]) <= 1e-5 * res[1][1]
