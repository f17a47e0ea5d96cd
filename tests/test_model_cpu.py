"""CDSSM semantics on CPU: shapes, weight sharing, init, loss closed form,
dropout-mask properties, conv/max-pool vs a brute-force loop."""
import math

import numpy as np
import pytest
import torch

from dnn_page_vectors_amd.config import Configuration
from dnn_page_vectors_amd.models.cdssm import CDSSM, cdssm_flops_per_sample
from dnn_page_vectors_amd.ops import loss as lops
from dnn_page_vectors_amd.ops import reference as ref


def test_reference_parameter_counts():
    cfg = Configuration(feature_level="ngram", vocab_hash_size=1000)
    m = CDSSM(cfg, 1000)
    tower = sum(p.numel() for n, p in m.query_tower.named_parameters() if n != "embedding")
    assert tower == 150450  # conv3 45,150 + conv4 60,150 + dense 45,150
    assert m.query_tower.embedding.shape == (1000, 100)
    assert len(m.doc_towers) == 1  # shared by positive + J negatives
    v1 = CDSSM(cfg.replace(share_doc_tower=False), 1000)
    assert len(v1.doc_towers) == 4


def test_init_ranges_and_determinism():
    cfg = Configuration(feature_level="ngram", vocab_hash_size=500)
    a, b = CDSSM(cfg, 500), CDSSM(cfg, 500)
    for (n, p), (_, q) in zip(a.named_parameters(), b.named_parameters()):
        assert torch.equal(p, q), n
    e = a.query_tower.embedding
    assert float(e.abs().max()) <= 0.05
    lim = math.sqrt(6.0 / (100 * 3 + 150 * 3))
    assert float(a.query_tower.conv_w[0].abs().max()) <= lim
    assert float(a.query_tower.conv_b[0].abs().max()) == 0.0


def test_forward_encode_shapes():
    cfg = Configuration(feature_level="ngram", vocab_hash_size=300, query_length=12, document_length=30)
    m = CDSSM(cfg, 300)
    q = torch.randint(0, 300, (4, 12), dtype=torch.int32)
    d = torch.randint(0, 300, (4, 4, 30), dtype=torch.int32)
    qv, dv = m(q, d)
    assert qv.shape == (4, 150) and dv.shape == (4, 4, 150) and float(qv.min()) >= 0.0  # final ReLU
    e = m.encode(d[:, 0])
    torch.testing.assert_close(e.norm(dim=1)[e.norm(dim=1) > 0], torch.ones_like(e.norm(dim=1)[e.norm(dim=1) > 0]))


def test_explicit_loss_closed_form():
    torch.manual_seed(0)
    q = torch.relu(torch.randn(6, 20))
    d = torch.relu(torch.randn(6, 4, 20))
    qn, dn = ref.l2_normalize(q), ref.l2_normalize(d)
    loss, P = lops.dssm_explicit_loss(qn, dn, 10.0)
    for i in range(6):
        R = [min(max(float(np.dot(q[i], d[i, j]) / (np.linalg.norm(q[i]) * np.linalg.norm(d[i, j]))), 0.0), 1.0)
             for j in range(4)]
        e = [math.exp(10 * r) for r in R]
        p = e[0] / sum(e)
        assert abs(float(P[i]) - p) < 1e-5
        assert abs(float(loss[i]) + math.log(min(max(p, 1e-7), 1 - 1e-7))) < 1e-4


def test_cosine_tiny_clamp_on_zero_vectors():
    z = torch.zeros(2, 5)
    assert torch.equal(ref.cosine_clip(z, z), torch.zeros(2))


def test_dropout_mask_properties():
    m = ref.dropout_keep_mask(7, 4000, 100, 0.25)
    assert abs(float(m.float().mean()) - 0.75) < 0.01
    assert torch.equal(m, ref.dropout_keep_mask(7, 4000, 100, 0.25))
    assert not torch.equal(m, ref.dropout_keep_mask(8, 4000, 100, 0.25))
    # row offset = a window of the same global mask
    assert torch.equal(m[1000:1010], ref.dropout_keep_mask(7, 10, 100, 0.25, row_offset=1000))
    t = ref.dropout_keep_mask(7, 100, 100, 0.25, mode="token")
    assert bool((t == t[:, :1]).all())


def test_conv_maxpool_bruteforce():
    torch.manual_seed(1)
    x = torch.randn(2, 9, 5)
    w = [torch.randn(3, 3, 5), torch.randn(3, 4, 5)]
    b = [torch.randn(3), torch.randn(3)]
    pooled, arg = ref.conv_relu_maxpool(x, w, b)
    for n in range(2):
        col = 0
        for wk, bk in zip(w, b):
            k = wk.shape[1]
            for f in range(3):
                vals = [float((x[n, t:t + k] * wk[f]).sum() + bk[f]) for t in range(9 - k + 1)]
                assert abs(float(pooled[n, col]) - max(0.0, max(vals))) < 1e-5
                assert int(arg[n, col]) == int(np.argmax(vals))
                col += 1


def test_flops_estimate_matches_survey():
    cfg = Configuration(feature_level="char")
    # char sample fwd ~4.25 GFLOP
    assert abs(cdssm_flops_per_sample(cfg) / 1e9 - 4.25) < 0.05


def test_query_stream_off_for_shared_towers():
    """tied query / page tower parameters must not take the side-stream path."""
    from dnn_page_vectors_amd.config import Configuration
    from dnn_page_vectors_amd.models import build_model

    cfg = Configuration(model="bert", bert_layers=1, bert_hidden=32, bert_intermediate=64, bert_heads=2,
                        bert_max_len=16, bert_out_dim=0, share_doc_tower=True)
    m = build_model(cfg, 50)
    assert m._towers_share_params()
    cfg2 = Configuration(model="bert", bert_layers=1, bert_hidden=32, bert_intermediate=64, bert_heads=2,
                         bert_max_len=16, bert_out_dim=0, share_doc_tower=False)
    assert not build_model(cfg2, 50)._towers_share_params()
