"""bag_gemm.hip (K1 long bags: dense-count MFMA products, both operands by LDS-DMA) against plain
PyTorch fp32 / fp64 references of the same op (C = per-bag token counts):

    forward  C @ W        (split-K partial slabs, summed here as the colsum kernel would)
    backward C^T @ Gs     (dW rows stored or accumulated into a strided target)
"""
import pytest
import torch

from dnn_page_vectors_amd.ops import embedding as eops
from dnn_page_vectors_amd.ops import reference as ref

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _ids(N, L, V, seed, zipf=True):
    g = torch.Generator(device="cpu").manual_seed(seed)
    if zipf:  # Zipf over a permuted vocabulary: hot ids repeat inside a page
        r = torch.arange(1, V, dtype=torch.float64)
        p = r.pow(-1.05)
        ids = torch.multinomial(p / p.sum(), N * L, replacement=True, generator=g) + 1
        ids = torch.randperm(V, generator=g)[ids.clamp(max=V - 1)]
    else:
        ids = torch.randint(0, V, (N * L,), generator=g)
    ids = ids.view(N, L).to(torch.int32)
    ids[:, L - L // 5:] = 0  # padding tail (pad = 0 is not counted)
    ids[0, :] = 5            # a page of ONE token: count L - L // 5 (> 256 when L is long)
    if N > 1 and V > 200:    # a page whose first segment holds 64 distinct ids (> the 4 in registers)
        ids[1, :64] = torch.arange(64, dtype=torch.int32) + 64
    return ids.to(DEV)


def _dense_counts(ids, V, pad=0):
    N, L = ids.shape
    C = torch.zeros(N, V, dtype=torch.float64, device=ids.device)
    ok = ids != pad
    C.scatter_add_(1, torch.where(ok, ids, torch.zeros_like(ids)).long(), ok.double())
    return C


@pytest.mark.parametrize("N,L,V,E", [(4096, 2000, 30000, 512), (300, 130, 1000, 72), (37, 512, 65000, 128),
                                     (513, 300, 30000, 256)])
def test_bag_dense_products_match_fp64(N, L, V, E):
    """The dense-count in-tree arm (PAGEVEC_BAG_GEMM=dense, bagd_mm_kernel): the histogram's bf16
    count matrix times W (split-K partials) and C^T Gs into a strided dW, vs fp64."""
    torch.manual_seed(1)
    ids = _ids(N, L, V, seed=N + 2 * V)
    C16, lens = eops._counts(ids, V, 0)
    Cb = _dense_counts(ids, V).float().bfloat16().double()
    torch.testing.assert_close(C16[:, :V].double(), Cb, rtol=0, atol=0)

    def close(got, want):
        err = float((got.double() - want).abs().max())
        assert err <= 2e-6 * float(want.abs().max()) + 1e-5, (err, float(want.abs().max()))

    W = torch.randn(V, E, device=DEV).bfloat16()
    part = eops._dense_forward_partials(C16, W, V)
    close(part.double().sum(0), Cb @ W.double())
    gs = torch.randn(N, E, device=DEV).bfloat16()
    base = torch.full((V, E + 8), 7.0, device=DEV)
    out = base[:, :E]  # strided target, padding untouched
    eops._dense_weight_grad(C16, gs, V, out)
    close(out, Cb.t() @ gs.double())
    assert bool((base[:, E:] == 7.0).all())


def test_bag_hip_matches_library_plan_end_to_end(monkeypatch):
    """The MLP page bag (mean, bias, tanh) with its W / bias gradients: in-tree kernels vs the
    hipBLASLt counts plan vs fp32 torch."""
    V, N, L, E = 30000, 512, 2000, 512
    ids = _ids(N, L, V, seed=9)
    W0 = torch.randn(V, E, device=DEV).bfloat16().float()
    b0 = torch.randn(E, device=DEV) * 0.3
    gy = torch.randn(N, E, device=DEV)
    res = {}
    for arm in ("lib", "dense"):
        monkeypatch.setattr(eops, "BAG_GEMM", arm)
        W = W0.clone().requires_grad_(True)
        b = b0.clone().requires_grad_(True)
        y = eops.embedding_bag(ids, W, pad=0, mean=True, plan="counts", bias=b, act="tanh")
        (y * gy).sum().backward()
        res[arm] = (y.detach(), W.grad, b.grad)
    Wr = W0.clone().requires_grad_(True)
    br = b0.clone().requires_grad_(True)
    cnt = (ids != 0).sum(1, keepdim=True).clamp(min=1).float()
    yr = torch.tanh(ref.embedding_bag_sum(ids, Wr, 0) / cnt + br)
    (yr * gy).sum().backward()
    for arm in ("lib", "dense"):
        y, gW, gb = res[arm]
        torch.testing.assert_close(y, yr, rtol=2e-2, atol=2e-2)
        for got, want in ((gW, Wr.grad), (gb, br.grad)):
            err = float((got - want).abs().max() / want.abs().max())
            assert err < 2e-2, (arm, err)
    # the two device arms agree far tighter than either does with fp32 (same bf16 operands); dW:
    # the library GEMM's rounding sits ~1e-3 of the max off the in-tree fp32 sums (which match
    # fp64, test_bag_dense_products_match_fp64)
    torch.testing.assert_close(res["dense"][0], res["lib"][0], rtol=1e-4, atol=1e-4)
    err = float((res["dense"][1] - res["lib"][1]).abs().max() / res["lib"][1].abs().max())
    assert err < 2e-3, err


def test_chunked_fp8_bag_backward_dense_weight_grad(monkeypatch):
    """Config 5's fp8 bag keeps the MX fp8 forward; its bf16 weight gradient C^T G on
    bagd_mm_kernel (fp32 sums) equals the exact C^T G, tighter than the library arm's."""
    V, N, L, E = 30000, 256, 512, 512
    monkeypatch.setattr(eops, "FP8_BWD", False)
    ids = _ids(N, L, V, seed=4)
    W0 = torch.randn(V, E, device=DEV).bfloat16().float() * 0.1
    gy = torch.randn(N, E, device=DEV)
    grads = {}
    for arm in ("dense", "lib"):
        monkeypatch.setattr(eops, "BAG_GEMM", arm)
        W = W0.clone().requires_grad_(True)
        y = eops.embedding_bag(ids, W, pad=0, mean=True, plan="counts", act="tanh", fp8=True)
        (y * gy).sum().backward()
        grads[arm] = W.grad
    # the exact weight gradient: C^T (dz / len) with dz from the (fp8) forward's activation
    C = _dense_counts(ids, V)
    lens = C.sum(1, keepdim=True).clamp(min=1)
    monkeypatch.setattr(eops, "BAG_GEMM", "dense")
    W = W0.clone().requires_grad_(True)
    y = eops.embedding_bag(ids, W, pad=0, mean=True, plan="counts", act="tanh", fp8=True).detach()
    gs = ((gy * (1 - y * y)).double() / lens).float().bfloat16().double()
    want = C.float().bfloat16().double().t() @ gs
    scale = float(want.abs().max())
    err_dense = float((grads["dense"].double() - want).abs().max()) / scale
    err_lib = float((grads["lib"].double() - want).abs().max()) / scale
    # fp32 output here; the library arm of this path returns the bf16 GEMM result (2^-8)
    assert err_dense < 1e-5 and err_lib < 8e-3, (err_dense, err_lib)


@pytest.mark.parametrize("N,L", [(256, 512), (4096, 512), (300, 700)])
def test_chunked_fp8_bag_backward_on_mx_fp8(N, L, monkeypatch):
    """PAGEVEC_FP8_BWD=1 (opt-in arm): the bag weight gradient as e4m3 counts^T x e4m3
    (per-tensor scaled) dz / len on the MX fp8 MFMA, against an fp64 reference of exactly that
    quantised product (emulate_e4m3 = the device's RNE saturating conversion), and within fp8
    rounding of the exact gradient."""
    from dnn_page_vectors_amd.ops import fp8 as fops

    V, E = 30000, 512
    monkeypatch.setattr(eops, "FP8_BWD", True)
    ids = _ids(N, L, V, seed=N + L)
    W0 = torch.randn(V, E, device=DEV).bfloat16().float() * 0.1
    b0 = torch.randn(E, device=DEV) * 0.1
    gy = torch.randn(N, E, device=DEV)
    W = W0.clone().requires_grad_(True)
    b = b0.clone().requires_grad_(True)
    y = eops.embedding_bag(ids, W, pad=0, mean=True, plan="counts", act="tanh", fp8=True, bias=b)
    (y * gy).sum().backward()
    C = _dense_counts(ids, V)
    lens = C.sum(1, keepdim=True).clamp(min=1)
    yd = y.detach().double()
    dz = gy.double() * (1 - yd * yd)
    gs = (gy * (1 - y.detach() * y.detach())) / lens.float()  # fp32, as on the device
    amax = float(gs.abs().max())
    g8 = fops.emulate_e4m3(gs * (448.0 / amax)).double() * (amax / 448.0)
    c8 = fops.emulate_e4m3(C.float()).double()
    want = c8.t() @ g8
    scale = float(want.abs().max())
    err = float((W.grad.double() - want).abs().max()) / scale
    # fp32 summation order + the odd e4m3 rounding tie of dz computed with / without an FMA
    assert err < 3e-3, err
    # within fp8 rounding of the exact gradient; counts above 448 saturate in e4m3 (as in the
    # forward: _ids' page 0 repeats one token L - L // 5 times), so that reference clamps them
    exact = C.clamp(max=448.0).t() @ (dz / lens)
    assert float((W.grad.double() - exact).abs().max()) / float(exact.abs().max()) < 0.08
    torch.testing.assert_close(b.grad.double(), dz.sum(0), rtol=1e-4, atol=1e-4)
