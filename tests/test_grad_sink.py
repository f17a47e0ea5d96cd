"""ops/grad_sink.py bookkeeping (CPU): which parameters an op may write directly."""
import torch

from dnn_page_vectors_amd.ops import grad_sink
from dnn_page_vectors_amd.ops.optim import FlatParams


def _two_layers():
    torch.manual_seed(0)
    m = torch.nn.ModuleDict({"a": torch.nn.Linear(4, 3), "b": torch.nn.Linear(3, 2)})
    return m, FlatParams(m.named_parameters())


def test_write_target_first_contribution_only(monkeypatch):
    monkeypatch.setattr(grad_sink, "ENABLED", True)
    m, flat = _two_layers()
    w = m["a"].weight
    with torch.no_grad():
        t = grad_sink.write_target(w)
        assert t is not None and t.data_ptr() == w.grad.data_ptr()
        fired = []
        remove = grad_sink.add_hook(w, lambda p: fired.append(p))
        grad_sink.done(w)
        assert fired == [w]
        assert grad_sink.write_target(w) is None          # already written this step
        assert grad_sink.accum_target(w) is not None      # accumulating kernels still may add
        flat.zero_grad()
        assert grad_sink.write_target(w) is not None
        remove()
        grad_sink.done(w)
        assert fired == [w]
    assert grad_sink.write_target(w) is None or torch.is_grad_enabled()  # grad mode on: autograd path
    monkeypatch.setattr(grad_sink, "ENABLED", False)
    with torch.no_grad():
        assert grad_sink.write_target(w) is None


def test_autograd_accumulate_marks_written(monkeypatch):
    monkeypatch.setattr(grad_sink, "ENABLED", True)
    m, flat = _two_layers()
    m["b"](m["a"](torch.randn(5, 4))).sum().backward()
    assert len(flat.written) == 4
    with torch.no_grad():
        assert grad_sink.write_target(m["a"].weight) is None


def test_mark_multi_use_finds_shared_parameters(monkeypatch):
    monkeypatch.setattr(grad_sink, "ENABLED", True)
    m, flat = _two_layers()
    x = torch.randn(5, 4)
    y = m["b"](m["a"](x)).sum() + m["a"](x).sum()
    assert grad_sink.mark_multi_use(y, flat) == 2
    with torch.no_grad():
        assert grad_sink.write_target(m["a"].weight) is None
        assert grad_sink.accum_target(m["a"].bias) is None
        assert grad_sink.write_target(m["b"].weight) is not None
    y2 = m["b"](m["a"](x)).sum()
    assert grad_sink.mark_multi_use(y2, flat) == 0


def test_embedding_tables_get_their_own_bucket():
    """parallel/ddp.py: each >= 1 MB embedding table is one bucket, so the sparse table
    backward (ops/conv_pool.py) can release it before the tower's weight gradients."""
    from dnn_page_vectors_amd.config import Configuration
    from dnn_page_vectors_amd.models.cdssm import CDSSM
    from dnn_page_vectors_amd.parallel.ddp import GradBuckets

    cfg = Configuration(feature_level="ngram", vocab_hash_size=30000)
    m = CDSSM(cfg, cfg.vocab_hash_size)
    flat = FlatParams(m.named_parameters())
    gb = GradBuckets(flat, bucket_mb=32.0)
    tables = [n for n, _ in flat.named if n.endswith("embedding")]
    assert len(tables) == 2
    for n in tables:
        bi = gb.param_bucket[n]
        assert gb.buckets[bi][2] == 1
    # every parameter is in exactly one bucket and the buckets tile disjoint ranges
    assert set(gb.param_bucket) == {n for n, _ in flat.named}
    spans = sorted((lo, hi) for lo, hi, _ in gb.buckets)
    assert all(a[1] <= b[0] for a, b in zip(spans, spans[1:]))
    assert sum(c for _, _, c in gb.buckets) == len(flat.named)
