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
