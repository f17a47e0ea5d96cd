"""Linear learning-rate warmup (Configuration.lr_warmup_steps): the HIP update reads it from the
device step buffer {step, warmup} (replayable from a hipGraph), the CPU path from the host."""
import pytest
import torch

from dnn_page_vectors_amd.ops.optim import FlatAdam, FlatParams


def _deltas(device, warmup, steps=5):
    torch.manual_seed(0)
    p = torch.nn.Parameter(torch.randn(1000, device=device))
    flat = FlatParams([("w", p)])
    opt = FlatAdam(flat, lr=1e-2, warmup=warmup)
    out = []
    for _ in range(steps):
        before = flat.data.clone()
        flat.grad.copy_(torch.ones_like(flat.grad))  # constant gradient: Adam's step = lr per element
        opt.step()
        out.append(float((before - flat.data).abs().mean()))
    return out


def _check(device):
    base = _deltas(device, 0)
    warm = _deltas(device, 4)
    for i, (b, w) in enumerate(zip(base, warm)):
        want = b * min(1.0, (i + 1) / 4)
        assert abs(w - want) <= 1e-3 * b, (i, w, want)


def test_warmup_cpu():
    _check(torch.device("cpu"))


@pytest.mark.gpu
def test_warmup_hip_device_step():
    _check(torch.device("cuda"))
