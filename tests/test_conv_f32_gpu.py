"""dtype="fp32" (the reference's precision): the fp32 HIP conv tower (csrc/kernels/conv_pool_f32.hip,
fp32 MFMA) vs the plain-PyTorch fp32 reference of the same op (run on MI355X: pytest -m gpu)."""
import types

import pytest
import torch

from dnn_page_vectors_amd.ops import _common
from dnn_page_vectors_amd.ops import conv_pool as cops
from dnn_page_vectors_amd.ops import reference as ref

pytestmark = pytest.mark.gpu
DEV = "cuda"
FP32 = types.SimpleNamespace(dtype="fp32")


def _spy(monkeypatch):
    calls = []
    orig = cops._ConvPoolF32Fn.apply
    monkeypatch.setattr(cops._ConvPoolF32Fn, "apply", lambda *a: calls.append(1) or orig(*a))
    return calls


@pytest.mark.parametrize("N,L,V,E,p,mode", [
    (5, 130, 97, 100, 0.25, "element"),   # two segments, nibble-mode dropout (the reference's 0.25)
    (4, 1400, 300, 100, 0.3, "element"),  # eleven segments, byte-mode dropout
    (3, 64, 97, 100, 0.25, "token"),
    (6, 4, 50, 100, 0.0, "element"),      # one window per width (k = 4: one, k = 3: two)
    (7, 300, 500, 64, 0.125, "element"),  # E = 64
    (2, 5000, 120, 100, 0.25, "element"), # char-level page length
    (40, 45, 1000, 100, 0.25, "element"),
    (3, 260, 90, 112, 0.0, "element"),    # E = EMAX
])
def test_conv_f32_fwd_bwd_matches_fp32_reference(N, L, V, E, p, mode, monkeypatch):
    calls = _spy(monkeypatch)
    torch.manual_seed(0)
    F = 150
    ids = torch.randint(0, V, (N, L), dtype=torch.int32, device=DEV)
    table = (torch.randn(V, E, device=DEV) * 0.5).requires_grad_(True)
    w3 = (torch.randn(F, 3, E, device=DEV) * 0.1).requires_grad_(True)
    w4 = (torch.randn(F, 4, E, device=DEV) * 0.1).requires_grad_(True)
    b3 = (torch.randn(F, device=DEV) * 0.1).requires_grad_(True)
    b4 = (torch.randn(F, device=DEV) * 0.1).requires_grad_(True)
    seed = 4321
    with _common.precision_scope(FP32):
        pooled, argmax = cops.conv_relu_maxpool_fused(ids, table, [w3, w4], [b3, b4], p, seed, True, mode)
    assert calls, "dtype=fp32 did not take the native fp32 kernel"
    tr = table.detach().clone().requires_grad_(True)
    w3r, w4r = w3.detach().clone(), w4.detach().clone()
    x = ref.embed_dropout(ids, tr, p, seed, True, mode)
    pr, ar = ref.conv_relu_maxpool(x, [w3r, w4r], [b3.detach(), b4.detach()])
    torch.testing.assert_close(pooled, pr, rtol=1e-5, atol=2e-5)
    live = pr > 1e-4
    assert ((argmax == ar) | ~live).float().mean() > 0.999
    g = torch.randn_like(pooled)
    (pooled * g).sum().backward()
    dws, dbs, dx = ref.conv_maxpool_grads_at(x.detach(), [w3r, w4r], pooled.detach(), argmax, g)
    x.backward(dx)
    torch.testing.assert_close(b3.grad, dbs[0], rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(b4.grad, dbs[1], rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(w3.grad, dws[0], rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(w4.grad, dws[1], rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(table.grad, tr.grad, rtol=1e-4, atol=1e-5)


def test_conv_f32_eval_and_row_offset(monkeypatch):
    """Eval mode (no mask) and a nonzero flat-row offset (chunked encoders) on the fp32 path."""
    calls = _spy(monkeypatch)
    torch.manual_seed(1)
    N, L, V, E, F = 4, 90, 60, 100, 150
    ids = torch.randint(0, V, (N, L), dtype=torch.int32, device=DEV)
    table = torch.randn(V, E, device=DEV) * 0.5
    w3, w4 = torch.randn(F, 3, E, device=DEV) * 0.1, torch.randn(F, 4, E, device=DEV) * 0.1
    b3, b4 = torch.randn(F, device=DEV) * 0.1, torch.randn(F, device=DEV) * 0.1
    with _common.precision_scope(FP32):
        pe, _ = cops.conv_relu_maxpool_fused(ids, table, [w3, w4], [b3, b4], 0.25, 7, False)
        po, _ = cops.conv_relu_maxpool_fused(ids, table, [w3, w4], [b3, b4], 0.25, 7, True, row_offset=12345)
    assert len(calls) == 2
    pr, _ = ref.conv_relu_maxpool(ref.embed_dropout(ids, table, 0.25, 7, False), [w3, w4], [b3, b4])
    torch.testing.assert_close(pe, pr, rtol=1e-5, atol=2e-5)
    xo = cops._embed_dropout_offset(ids, table, 0.25, 7, True, "element", 12345)
    pro, _ = ref.conv_relu_maxpool(xo, [w3, w4], [b3, b4])
    torch.testing.assert_close(po, pro, rtol=1e-5, atol=2e-5)


@pytest.mark.parametrize("M,N,K,a_t,b_t,act,splits", [
    (300, 150, 300, False, True, "relu", 1),    # forward X W^T (CDSSM head)
    (77, 45, 130, False, True, "tanh", 1),      # ragged edges
    (300, 300, 150, False, False, "none", 1),   # dgrad dZ W
    (150, 300, 4096, True, False, "none", 8),   # wgrad dZ^T X, split-K
    (64, 64, 1000, True, True, "gelu", 1),      # both transposed
    (513, 129, 17, False, False, "none", 3),    # split-K with a short last slice
])
def test_gemm_f32_matches_fp64(M, N, K, a_t, b_t, act, splits):
    from dnn_page_vectors_amd.ops import dense as dops
    g = torch.Generator(device=DEV).manual_seed(M + N + K)
    a = torch.randn(*((K, M) if a_t else (M, K)), device=DEV, generator=g)
    b = torch.randn(*((N, K) if b_t else (K, N)), device=DEV, generator=g)
    bias = torch.randn(N, device=DEV, generator=g) if splits == 1 else None
    out = dops.gemm_f32(a, b, a_t=a_t, b_t=b_t, bias=bias, act=act, splits=splits)
    A = (a.t() if a_t else a).double()
    B = (b.t() if b_t else b).double()
    r = A @ B + (bias.double() if bias is not None else 0.0)
    r = {"relu": torch.relu, "tanh": torch.tanh, "none": lambda t: t,
         "gelu": lambda t: torch.nn.functional.gelu(t, approximate="tanh")}[act](r)
    # exact fp32 products and sums: K-length rounding only (the bf16 path would be ~1e-2)
    torch.testing.assert_close(out.double(), r, rtol=2e-5, atol=2e-5 * K ** 0.5)
    if splits == 1:  # accumulate into an existing output
        acc = torch.ones(M, N, device=DEV)
        dops.gemm_f32(a, b, a_t=a_t, b_t=b_t, out=acc, accumulate=True)
        torch.testing.assert_close(acc.double(), A @ B + 1.0, rtol=2e-5, atol=2e-5 * K ** 0.5)


def test_cdssm_fp32_step_native_matches_torch_ops(monkeypatch):
    """One dtype="fp32" CDSSM training step: the native fp32 conv tower, dense layers (fp32 MFMA
    GEMM), L2 normalisation and explicit loss give the loss and the flat gradient of the
    all-PyTorch fp32 path (PAGEVEC_F32_NATIVE=0)."""
    from dnn_page_vectors_amd.ops import dense as dops
    from dnn_page_vectors_amd.ops import loss as lops
    from dnn_page_vectors_amd.config import Configuration
    from dnn_page_vectors_amd.models import build_model
    from dnn_page_vectors_amd.parallel import dist as pdist
    from dnn_page_vectors_amd.train.trainer import Trainer

    pdist.set_info(pdist.DistInfo(device=torch.device(DEV)))
    V = 500
    cfg = Configuration(model="cdssm", feature_level="ngram", vocab_hash_size=V, query_length=12,
                        document_length=200, batch_size=32, embedding_dim=100, dtype="fp32")
    g = torch.Generator().manual_seed(4)
    q = torch.randint(1, V, (32, 12), generator=g, dtype=torch.int32).to(DEV)
    d = torch.randint(1, V, (32, cfg.J + 1, 200), generator=g, dtype=torch.int32).to(DEV)
    out = []
    for native in (False, True):
        monkeypatch.setattr(_common, "F32_NATIVE", native)
        calls = _spy(monkeypatch)
        lin, exp = [], []
        orig_lin, orig_exp = dops._LinearF32Fn.apply, lops._ExplicitFn.apply
        monkeypatch.setattr(dops._LinearF32Fn, "apply", lambda *a, o=orig_lin: lin.append(1) or o(*a))
        monkeypatch.setattr(lops._ExplicitFn, "apply", lambda *a, o=orig_exp: exp.append(1) or o(*a))
        torch.manual_seed(0)
        tr = Trainer(cfg, build_model(cfg, V), torch.device(DEV))
        m = tr.train_step(q, d)
        torch.cuda.synchronize()
        assert bool(calls) == native
        assert bool(lin) == native and bool(exp) == native, (len(lin), len(exp))
        out.append((float(m["loss"]), tr.flat.grad.clone()))
    (la, ga), (lb, gb) = out
    assert abs(la - lb) <= 1e-5 * max(1.0, abs(la))
    err = float((ga - gb).abs().max() / ga.abs().max())
    assert err < 1e-4, err


@pytest.mark.parametrize("N,L,p", [(5, 130, 0.25), (3, 5000, 0.25), (64, 45, 0.0), (2, 700, 0.3)])
def test_conv_f32_role_split_forward_bit_identical(N, L, p):
    """The role-split forward (v2, E = 100) and the one-role kernel (v1) accumulate every
    output in the same order: pooled and argmax bit-identical."""
    from dnn_page_vectors_amd.ops._common import lib

    torch.manual_seed(2)
    V, E, F = 300, 100, 150
    ids = torch.randint(0, V, (N, L), dtype=torch.int32, device=DEV)
    table = torch.randn(V, E, device=DEV) * 0.5
    w3, w4 = torch.randn(F, 3, E, device=DEV) * 0.1, torch.randn(F, 4, E, device=DEV) * 0.1
    b3, b4 = torch.randn(F, device=DEV) * 0.1, torch.randn(F, device=DEV) * 0.1
    out = []
    try:
        for v2 in (0, 1):
            lib().pv_conv_f32_set_v2(v2)
            with _common.precision_scope(FP32):
                out.append(cops.conv_relu_maxpool_fused(ids, table, [w3, w4], [b3, b4], p, 9, True))
    finally:
        lib().pv_conv_f32_set_v2(1)
    assert torch.equal(out[0][0], out[1][0])
    assert torch.equal(out[0][1], out[1][1])


@pytest.mark.parametrize("p,mode", [(0.25, "element"), (0.3, "element"), (0.25, "token")])
def test_conv_f32_mask_plane_matches_inline_hash(p, mode, monkeypatch):
    """The keep-bit plane (conv_f32_mask_kernel) and the inline hashes give the same forward
    (bit-identical) and the same gradients."""
    torch.manual_seed(3)
    N, L, V, E, F = 4, 333, 80, 100, 150
    ids = torch.randint(0, V, (N, L), dtype=torch.int32, device=DEV)
    res = []
    for use_mask in (False, True):
        monkeypatch.setattr(cops, "F32_MASK", use_mask)
        torch.manual_seed(4)
        table = (torch.randn(V, E, device=DEV) * 0.5).requires_grad_(True)
        w3 = (torch.randn(F, 3, E, device=DEV) * 0.1).requires_grad_(True)
        w4 = (torch.randn(F, 4, E, device=DEV) * 0.1).requires_grad_(True)
        b3 = torch.zeros(F, device=DEV, requires_grad=True)
        b4 = torch.zeros(F, device=DEV, requires_grad=True)
        with _common.precision_scope(FP32):
            y, a = cops.conv_relu_maxpool_fused(ids, table, [w3, w4], [b3, b4], p, 11, True, mode, row_offset=77)
        (y * torch.linspace(-1, 1, y.numel(), device=DEV).view_as(y)).sum().backward()
        res.append((y.detach(), a, table.grad, w3.grad, w4.grad))
    (y0, a0, *g0), (y1, a1, *g1) = res
    assert torch.equal(y0, y1) and torch.equal(a0, a1)
    for u, v in zip(g0, g1):
        torch.testing.assert_close(u, v, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("dxw", [0, 1])
def test_conv_f32_small_vocab_table_grad_paths(dxw):
    """Both small-vocabulary dTable kernels (wave-private LDS tables / shared table with LDS
    float atomics) against the fp32 reference, hot rows included (a 7-symbol vocabulary)."""
    from dnn_page_vectors_amd.ops._common import lib

    torch.manual_seed(5)
    N, L, V, E, F = 6, 400, 7, 100, 150
    ids = torch.randint(0, V, (N, L), dtype=torch.int32, device=DEV)
    table = (torch.randn(V, E, device=DEV) * 0.5).requires_grad_(True)
    w3 = torch.randn(F, 3, E, device=DEV) * 0.1
    w4 = torch.randn(F, 4, E, device=DEV) * 0.1
    b3, b4 = torch.zeros(F, device=DEV), torch.zeros(F, device=DEV)
    try:
        lib().pv_conv_f32_set_dxw(dxw)
        with _common.precision_scope(FP32):
            y, a = cops.conv_relu_maxpool_fused(ids, table, [w3, w4], [b3, b4], 0.25, 3, True)
        g = torch.randn_like(y)
        (y * g).sum().backward()
    finally:
        lib().pv_conv_f32_set_dxw(1)
    tr = table.detach().clone().requires_grad_(True)
    x = ref.embed_dropout(ids, tr, 0.25, 3, True)
    _, _, dx = ref.conv_maxpool_grads_at(x.detach(), [w3, w4], y.detach(), a, g)
    x.backward(dx)
    torch.testing.assert_close(table.grad, tr.grad, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("V", [1000, 150])  # global-atomic and shared-LDS-atomic table paths
def test_conv_f32_deterministic_mode_bit_identical(V):
    """Deterministic mode on the fp32 path: two backward passes give bit-identical gradients
    (the float-atomic table kernels are replaced by an ordered index_add_), close to the
    atomic path's."""
    from dnn_page_vectors_amd.ops import determinism

    torch.manual_seed(6)
    N, L, E, F = 8, 300, 100, 150
    ids = torch.randint(0, V, (N, L), dtype=torch.int32, device=DEV)
    w3 = torch.randn(F, 3, E, device=DEV) * 0.1
    w4 = torch.randn(F, 4, E, device=DEV) * 0.1
    b3, b4 = torch.zeros(F, device=DEV), torch.zeros(F, device=DEV)
    base = torch.randn(V, E, device=DEV) * 0.5

    def grads():
        table = base.clone().requires_grad_(True)
        with _common.precision_scope(FP32):
            y, _ = cops.conv_relu_maxpool_fused(ids, table, [w3, w4], [b3, b4], 0.25, 5, True)
        (y * torch.linspace(-1, 1, y.numel(), device=DEV).view_as(y)).sum().backward()
        return table.grad

    prev = determinism.set_deterministic(True)
    try:
        g1, g2 = grads(), grads()
    finally:
        determinism.restore(prev)
    g3 = grads()
    assert torch.equal(g1, g2)
    torch.testing.assert_close(g1, g3, rtol=1e-5, atol=1e-5)
