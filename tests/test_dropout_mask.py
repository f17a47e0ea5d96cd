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


@pytest.mark.parametrize("p", [0.25, 0.125, 0.5, 0.75, 0.3])
def test_keep_rate_per_column_and_pairwise_independence(p):
    """The round-6 group hash (common.h mix24): every column's keep rate and every pairwise
    correlation of a row's 104 decisions at the statistical floor (5.5 sigma over 200k rows;
    the maximum of 5356 |N(0,1)| pairs is ~4.3 sigma)."""
    n, w = 200_000, 104
    m = ref.dropout_keep_mask(99, n, w, p).double()
    q = 1.0 - ref.dropout_threshold(p) / 256.0
    rate_sigma = (q * (1 - q) / n) ** 0.5
    assert float((m.mean(0) - q).abs().max()) < 5.5 * rate_sigma
    c = torch.corrcoef(m.t())
    c.fill_diagonal_(0.0)
    assert float(c.abs().max()) < 5.5 / n ** 0.5


def test_kept_count_distributions_binomial():
    """Higher-order check: the number of kept columns per 8-column group, per row, and the
    joint counts of two adjacent groups follow the binomial law (chi-square, p = 0.25)."""
    from math import comb

    n, w, p = 200_000, 104, 0.25
    m = ref.dropout_keep_mask(5, n, w, p).long()
    q = 0.75

    def chi2(counts, probs):
        exp = probs * n
        sel = exp > 5
        return float(((counts[sel] - exp[sel]) ** 2 / exp[sel]).sum()), int(sel.sum()) - 1

    pm = torch.tensor([comb(8, i) * q ** i * (1 - q) ** (8 - i) for i in range(9)], dtype=torch.float64)
    for g in (0, 6, 12):
        cnt = torch.bincount(m[:, 8 * g:8 * g + 8].sum(1), minlength=9).double()
        x, dof = chi2(cnt, pm)
        assert x < dof + 6 * (2 * dof) ** 0.5, (g, x, dof)
    pr = torch.tensor([comb(w, i) * q ** i * (1 - q) ** (w - i) for i in range(w + 1)], dtype=torch.float64)
    x, dof = chi2(torch.bincount(m.sum(1), minlength=w + 1).double(), pr)
    assert x < dof + 6 * (2 * dof) ** 0.5, (x, dof)
    j = m[:, :8].sum(1) * 9 + m[:, 8:16].sum(1)
    x, dof = chi2(torch.bincount(j, minlength=81).double(), torch.outer(pm, pm).reshape(-1))
    assert x < dof + 6 * (2 * dof) ** 0.5, (x, dof)
