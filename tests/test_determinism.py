"""SURVEY §5.2 determinism.

* CPU (reference ops): two identical runs -> bit-identical parameters.
* GPU: the forward pass (fused conv, dense, L2 norm, in-batch loss with split sums
  reduced in a fixed order) is bit-reproducible; the backward uses fp32 atomics in the
  conv weight / embedding reductions, so repeated training steps agree to rounding.
"""
import pytest
import torch

from dnn_page_vectors_amd.config import Configuration
from dnn_page_vectors_amd.models.cdssm import CDSSM
from dnn_page_vectors_amd.parallel import dist as pdist
from dnn_page_vectors_amd.train.trainer import Trainer


def _cfg():
    return Configuration(feature_level="ngram", vocab_hash_size=300, query_length=12, document_length=40,
                         batch_size=16, embedding_dim=24, hidden_dims=32, loss_mode="in_batch", cos_clip=False)


def _batches(dev, n=3):
    g = torch.Generator().manual_seed(5)
    return [(torch.randint(1, 300, (16, 12), generator=g, dtype=torch.int32).to(dev),
             torch.randint(1, 300, (16, 4, 40), generator=g, dtype=torch.int32).to(dev)) for _ in range(n)]


def _run(dev):
    torch.manual_seed(0)
    pdist.set_info(pdist.DistInfo(device=torch.device(dev)))
    cfg = _cfg()
    tr = Trainer(cfg, CDSSM(cfg, 300), torch.device(dev))
    losses = [float(tr.train_step(q, d)["loss"]) for q, d in _batches(dev)]
    return tr, losses


def test_cpu_training_bit_identical():
    a, la = _run("cpu")
    b, lb = _run("cpu")
    assert la == lb
    assert torch.equal(a.flat.data, b.flat.data)


@pytest.mark.gpu
def test_gpu_forward_bit_identical_and_training_reproducible():
    a, la = _run("cuda")
    b, lb = _run("cuda")
    assert la[0] == lb[0]  # first step: identical weights, forward is deterministic
    torch.testing.assert_close(a.flat.data, b.flat.data, rtol=1e-5, atol=1e-6)
    q, d = _batches("cuda", 1)[0]
    with torch.no_grad():
        l1, _ = a.compute_loss(q, d, seed=11)
        l2, _ = a.compute_loss(q, d, seed=11)
    assert torch.equal(l1, l2)


def _run_det(dev, deterministic, steps=3, ld=40):
    torch.manual_seed(0)
    pdist.set_info(pdist.DistInfo(device=torch.device(dev)))
    cfg = _cfg().replace(deterministic=deterministic, document_length=ld, dropout_prob=(0.25, 0.5))
    tr = Trainer(cfg, CDSSM(cfg, 300), torch.device(dev))
    g = torch.Generator().manual_seed(5)
    losses = []
    for _ in range(steps):
        q = torch.randint(1, 300, (16, 12), generator=g, dtype=torch.int32).to(dev)
        d = torch.randint(1, 300, (16, 4, ld), generator=g, dtype=torch.int32).to(dev)
        losses.append(float(tr.train_step(q, d)["loss"]))
    torch.cuda.synchronize() if dev == "cuda" else None
    return tr, losses


def test_deterministic_flag_cpu_is_noop():
    """The config flag exists everywhere; on CPU the reference ops are order-free anyway."""
    a, la = _run_det("cpu", True, steps=2)
    b, lb = _run_det("cpu", False, steps=2)
    assert la == lb and torch.equal(a.flat.data, b.flat.data)
    from dnn_page_vectors_amd.ops import determinism
    determinism.set_deterministic(False)


@pytest.mark.gpu
@pytest.mark.parametrize("ld", [40, 200])
def test_gpu_deterministic_mode_bit_identical_training(ld):
    """with the deterministic reduction mode two GPU training runs give
    bit-identical losses AND parameters (fixed-point cross-workgroup sums, one stream);
    the mode changes the result only at rounding level.  ld = 40 takes the query-style
    dense-dX table backward, ld = 200 the page tower's emit / sort / reduce path."""
    from dnn_page_vectors_amd.ops import determinism
    try:
        a, la = _run_det("cuda", True, ld=ld)
        b, lb = _run_det("cuda", True, ld=ld)
        assert la == lb
        assert torch.equal(a.flat.data, b.flat.data)
        assert torch.equal(a.opt.m, b.opt.m) and torch.equal(a.opt.v, b.opt.v)
        c, lc = _run_det("cuda", False, ld=ld)
        torch.testing.assert_close(c.flat.data, a.flat.data, rtol=1e-4, atol=1e-5)
    finally:
        determinism.set_deterministic(False)


@pytest.mark.gpu
@pytest.mark.parametrize("preset", ["mlp_xgpu", "bert_dp8"])
def test_gpu_deterministic_mode_other_models(preset):
    """The deterministic mode covers the MLP (embedding-bag sparse backward, column sums)
    and BERT (LayerNorm / bias partial sums, token-embedding index_add_) steps too."""
    from dnn_page_vectors_amd.config import preset_config
    from dnn_page_vectors_amd.data.synthetic import SyntheticPairs, spec_from_config
    from dnn_page_vectors_amd.models import build_model
    from dnn_page_vectors_amd.ops import determinism

    cfg = preset_config(preset).replace(deterministic=True, loss_mode="in_batch")
    if preset == "bert_dp8":
        cfg = cfg.replace(bert_layers=2, batch_size=16, document_length=64, query_length=16)
    else:
        cfg = cfg.replace(batch_size=64, document_length=256, mlp_dims=(128, 128, 64), embedding_dim=128)
    pdist.set_info(pdist.DistInfo(device=torch.device("cuda")))
    try:
        runs = []
        for _ in range(2):
            torch.manual_seed(0)
            tr = Trainer(cfg, build_model(cfg, cfg.vocab_hash_size), torch.device("cuda"))
            data = SyntheticPairs(spec_from_config(cfg, cfg.vocab_hash_size, num_pages=256), "cuda", seed=3)
            losses = [float(tr.train_step(*data.batch(cfg.batch_size))["loss"]) for _ in range(3)]
            torch.cuda.synchronize()
            runs.append((losses, tr.flat.data.clone()))
        assert runs[0][0] == runs[1][0]
        assert torch.equal(runs[0][1], runs[1][1])
    finally:
        determinism.set_deterministic(False)


def test_trainers_do_not_leak_the_deterministic_mode():
    """a deterministic trainer built first must not leave a later default trainer
    (which may capture hipGraphs and use side streams) in the deterministic mode; each
    trainer's step runs in its own mode, and closing the deterministic one restores the
    previous state."""
    from dnn_page_vectors_amd.ops import determinism
    dev = "cpu"
    try:
        a, _ = _run_det(dev, True, steps=1)
        assert determinism.enabled()
        b, _ = _run_det(dev, False, steps=1)
        assert not determinism.enabled()
        g = torch.Generator().manual_seed(9)
        q = torch.randint(1, 300, (16, 12), generator=g, dtype=torch.int32)
        d = torch.randint(1, 300, (16, 4, 40), generator=g, dtype=torch.int32)
        a.train_step(q, d)
        assert determinism.enabled()
        b.train_step(q, d)
        assert not determinism.enabled()
        a.train_step(q, d)
        a.close()
        assert not determinism.enabled()
    finally:
        determinism.set_deterministic(False)


@pytest.mark.gpu
def test_graph_trainer_after_deterministic_trainer_gpu():
    """A graph-mode trainer built after a deterministic one captures its step with the
    deterministic mode OFF (no fixed-point buffer growth inside a capture)."""
    from dnn_page_vectors_amd.ops import determinism
    try:
        a, _ = _run_det("cuda", True, steps=1)
        torch.manual_seed(0)
        cfg = _cfg().replace(document_length=40, dropout_prob=(0.25, 0.5))
        b = Trainer(cfg, CDSSM(cfg, 300), torch.device("cuda"), graph=True)
        assert b.graph_mode
        g = torch.Generator().manual_seed(5)
        for _ in range(Trainer.GRAPH_WARMUP + 3):
            q = torch.randint(1, 300, (16, 12), generator=g, dtype=torch.int32).cuda()
            d = torch.randint(1, 300, (16, 4, 40), generator=g, dtype=torch.int32).cuda()
            m = b.train_step(q, d)
            assert not determinism.enabled()
        torch.cuda.synchronize()
        assert b._graph is not None and float(m["loss"]) == float(m["loss"])
        a.train_step(q, d)  # the deterministic trainer still runs in its own mode
        assert determinism.enabled()
    finally:
        determinism.set_deterministic(False)
