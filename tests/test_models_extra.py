"""MLP (configs 1/3), BERT (4), chunked fp8 (5) and legacy LSTM towers on CPU."""
import pytest
import torch

from dnn_page_vectors_amd.config import preset_config
from dnn_page_vectors_amd.data.synthetic import SyntheticPairs, spec_from_config
from dnn_page_vectors_amd.eval.retrieval import recall_at_k
from dnn_page_vectors_amd.models import build_model
from dnn_page_vectors_amd.parallel import dist as pdist
from dnn_page_vectors_amd.train.trainer import Trainer


@pytest.fixture(autouse=True)
def _single():
    pdist.init_distributed(device="cpu")


def test_tiny_dssm_config1_learns_recall():
    cfg = preset_config("tiny_dssm_cpu")
    m = build_model(cfg, cfg.vocab_hash_size)
    tr = Trainer(cfg, m)
    sp = SyntheticPairs(spec_from_config(cfg, cfg.vocab_hash_size, num_pages=2048), seed=3)
    qe, pe = sp.eval_set(256)
    r0 = recall_at_k(m.encode(qe, "query"), m.encode(pe, "doc"), torch.arange(256), 10)
    for _ in range(150):
        tr.train_step(*sp.batch(cfg.batch_size))
    r1 = recall_at_k(m.encode(qe, "query"), m.encode(pe, "doc"), torch.arange(256), 10)
    assert r1 > r0 + 0.1, (r0, r1)


@pytest.mark.parametrize("preset,kw", [
    ("bert_dp8", dict(bert_layers=2, bert_hidden=64, bert_heads=4, bert_intermediate=128, vocab_hash_size=300,
                      query_length=8, document_length=24, batch_size=8)),
    ("longpage_fp8", dict(vocab_hash_size=300, mlp_dims=(32, 32, 16), chunk_len=16, num_chunks=4,
                          document_length=64, query_length=12, batch_size=8)),
    ("longpage_cdssm", dict(vocab_hash_size=300, chunk_len=16, num_chunks=4, document_length=64, query_length=12,
                            batch_size=8)),
    ("lstm", dict(query_length=8, document_length=20, batch_size=8, loss_mode="explicit")),
    ("lstm", dict(query_length=8, document_length=20, batch_size=8, loss_mode="explicit", lstm_conv=True)),
])
def test_models_train_and_encode(preset, kw):
    cfg = preset_config(preset).replace(**kw)
    V = cfg.vocab_hash_size if cfg.vocab_hash_size > 1 else 300
    m = build_model(cfg, V)
    tr = Trainer(cfg, m)
    sp = SyntheticPairs(spec_from_config(cfg, V, num_pages=64))
    before = tr.flat.data.clone()
    out = tr.train_step(*sp.batch(cfg.batch_size))
    assert float(out["loss"]) == float(out["loss"]) and not torch.equal(before, tr.flat.data)
    q, p = sp.eval_set(5)
    v = m.encode(p, "doc")
    assert v.shape == (5, m.out_dim)


def test_chunked_mean_pool_masks_empty_chunks():
    cfg = preset_config("longpage_fp8").replace(vocab_hash_size=100, mlp_dims=(16, 8), chunk_len=4, num_chunks=3,
                                                document_length=12, use_fp8=False)
    m = build_model(cfg, 100).eval()
    ids = torch.zeros(1, 12, dtype=torch.int32)
    ids[0, :4] = torch.tensor([5, 6, 7, 8])
    full = m.tower_forward("doc", ids, False, 0)
    one = m.doc_towers[0](ids[:, :4])
    torch.testing.assert_close(full, one)


def test_chunked_cdssm_max_pool_is_max_of_chunk_features():
    """chunk_pool='max': the element-wise max of the non-empty chunks' pooled conv features
    through ONE Dense + ReLU (an all-padding chunk never wins)."""
    cfg = preset_config("longpage_cdssm").replace(vocab_hash_size=100, chunk_len=8, num_chunks=3,
                                                  document_length=24, chunk_pool="max")
    m = build_model(cfg, 100).eval()
    ids = torch.zeros(2, 24, dtype=torch.int32)
    ids[0, :16] = torch.randint(1, 100, (16,), dtype=torch.int32)
    ids[1, :] = torch.randint(1, 100, (24,), dtype=torch.int32)
    t = m.doc_towers[0]
    got = m.tower_forward("doc", ids, False, 0)
    f = t.features(ids.view(6, 8), False, 0).view(2, 3, -1)
    want = t.head(torch.stack([f[0, :2].amax(0), f[1].amax(0)]), False)
    torch.testing.assert_close(got, want)
    with pytest.raises(ValueError):
        build_model(preset_config("longpage_fp8").replace(chunk_pool="max", use_fp8=False), 100)


def test_bert_shared_tower_is_siamese():
    cfg = preset_config("bert_dp8").replace(bert_layers=1, bert_hidden=32, bert_heads=2, bert_intermediate=64,
                                            vocab_hash_size=100)
    m = build_model(cfg, 100)
    assert m.doc_towers[0] is m.query_tower
    n_params = sum(p.numel() for p in m.parameters())
    assert n_params == sum(p.numel() for p in m.query_tower.parameters())


def test_fp8_emulation_backward_is_straight_through():
    """CPU fp8 linear (e4m3 round trip of x and w): the gradient reaches x and w (straight-
    through, like the HIP path's bf16 backward GEMMs) — a float8 cast alone cuts autograd and
    trained only the last bias of the chunked fp8 encoder on the CPU path."""
    from dnn_page_vectors_amd.ops import fp8 as fops

    torch.manual_seed(0)
    x = torch.randn(16, 32, requires_grad=True)
    w = (torch.randn(8, 32) * 0.1).requires_grad_(True)
    b = torch.zeros(8, requires_grad=True)
    g = torch.randn(16, 8)
    (fops.fp8_linear(x, w, b, "tanh") * g).sum().backward()
    x2, w2, b2 = x.detach().clone().requires_grad_(True), w.detach().clone().requires_grad_(True), torch.zeros(8, requires_grad=True)
    (torch.tanh(torch.nn.functional.linear(x2, w2, b2)) * g).sum().backward()
    for got, want in ((x.grad, x2.grad), (w.grad, w2.grad), (b.grad, b2.grad)):
        assert float((got - want).norm() / want.norm()) < 0.1
