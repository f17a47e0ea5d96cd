"""Counter-based dropout masks (ops/reference.py dropout_keep_mask = the kernels' spec):
keep rate, independence between neighbouring columns / rows, determinism, both the nibble
path (p = k/16, e.g. the reference's 0.25) and the byte path (other p)."""
import pytest
import torch

from dnn_page_vectors_amd.ops import reference as ref


@pytest.mark.parametrize("p", [0.25, 0.5, 0.3, 0.1])
def test_keep_rate_and_independence(p):
    m = ref.dropout_keep_mask(1234, 4000, 104, p).float()
    thr = ref.dropout_threshold(p)
    expect = 1.0 - thr / 256.0
    assert abs(m.mean().item() - expect) < 0.01
    a = m - m.mean()
    col_corr = (a[:, :-1] * a[:, 1:]).mean() / a.var()
    row_corr = (a[:-1] * a[1:]).mean() / a.var()
    grp_corr = (a[:, :-8] * a[:, 8:]).mean() / a.var()
    for c in (col_corr, row_corr, grp_corr):
        assert abs(c.item()) < 0.02


def test_mask_deterministic_and_seed_dependent():
    a = ref.dropout_keep_mask(7, 100, 100, 0.25, row_offset=5)
    b = ref.dropout_keep_mask(7, 100, 100, 0.25, row_offset=5)
    c = ref.dropout_keep_mask(8, 100, 100, 0.25, row_offset=5)
    assert torch.equal(a, b) and not torch.equal(a, c)
    # row_offset shifts the row ids
    d = ref.dropout_keep_mask(7, 105, 100, 0.25)
    assert torch.equal(a, d[5:])
