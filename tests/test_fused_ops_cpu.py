"""CPU semantics of the fused-op entry points (the reference path the HIP kernels are
checked against on the GPU): column sums with accumulate / epilogue, the bag with fused
bias + activation, and the loss ``reduce`` mode."""
import pytest
import torch

from dnn_page_vectors_amd.ops import dense as dops
from dnn_page_vectors_amd.ops import embedding as eops
from dnn_page_vectors_amd.ops import loss as lops
from dnn_page_vectors_amd.ops import reference as ref


def test_colsum_cpu_modes():
    g = torch.Generator().manual_seed(0)
    x = torch.randn(37, 6, 8, generator=g)
    torch.testing.assert_close(dops.colsum(x), x.sum(0))
    out = torch.ones(6, 8)
    dops.colsum(x, out=out, accumulate=True)
    torch.testing.assert_close(out, 1 + x.sum(0))
    scale, bias = torch.rand(6, generator=g), torch.randn(8, generator=g)
    y = dops.colsum(x, scale=scale, bias=bias, act="tanh")
    torch.testing.assert_close(y, torch.tanh(x.sum(0) * scale[:, None] + bias))


def test_embedding_bag_bias_act_cpu():
    g = torch.Generator().manual_seed(1)
    ids = torch.randint(0, 50, (9, 12), generator=g, dtype=torch.int32)
    ids[:, 8:] = 0
    W = torch.randn(50, 16, generator=g, requires_grad=True)
    b = torch.randn(16, generator=g, requires_grad=True)
    y = eops.embedding_bag(ids, W, pad=0, mean=True, bias=b, act="relu")
    cnt = (ids != 0).sum(1, keepdim=True).clamp(min=1).float()
    W2 = W.detach().clone().requires_grad_(True)
    b2 = b.detach().clone().requires_grad_(True)
    want = torch.relu(torch.nn.functional.embedding(ids.long(), W2).mul((ids != 0).unsqueeze(-1)).sum(1) / cnt + b2)
    torch.testing.assert_close(y, want)
    y.sum().backward()
    want.sum().backward()
    torch.testing.assert_close(W.grad, W2.grad)
    torch.testing.assert_close(b.grad, b2.grad)


def test_inbatch_loss_reduce_cpu():
    g = torch.Generator().manual_seed(2)
    q = torch.nn.functional.normalize(torch.randn(8, 16, generator=g), dim=1)
    d = torch.nn.functional.normalize(torch.randn(32, 16, generator=g), dim=1)
    pos = torch.arange(8, dtype=torch.int32) * 4
    per_row, P = lops.inbatch_loss(q, d, pos, 10.0, True)
    lm, P2, acc = lops.inbatch_loss(q, d, pos, 10.0, True, reduce=True)
    torch.testing.assert_close(lm, per_row.mean())
    torch.testing.assert_close(P2, P)
    torch.testing.assert_close(acc, (P > 0.5).float().mean())


def test_conv_grads_at_given_argmax_match_autograd():
    """ops/reference.py::conv_maxpool_grads_at (the GPU tests' reference backward through the
    kernel's argmax) == autograd of the reference conv when given the reference's argmax."""
    torch.manual_seed(0)
    N, L, E, F = 4, 20, 6, 5
    x = torch.randn(N, L, E, requires_grad=True)
    w3 = torch.randn(F, 3, E, requires_grad=True)
    w4 = torch.randn(F, 4, E, requires_grad=True)
    b3 = torch.randn(F, requires_grad=True)
    b4 = torch.randn(F, requires_grad=True)
    p, a = ref.conv_relu_maxpool(x, [w3, w4], [b3, b4])
    g = torch.randn_like(p)
    (p * g).sum().backward()
    dws, dbs, dx = ref.conv_maxpool_grads_at(x.detach(), [w3.detach(), w4.detach()], p.detach(), a, g)
    for got, want in ((dws[0], w3.grad), (dws[1], w4.grad), (dbs[0], b3.grad), (dbs[1], b4.grad), (dx, x.grad)):
        torch.testing.assert_close(got, want)


def test_f32_forward_plan_covers_every_window():
    """ops/conv_pool.py::f32_plan: segments are whole 128-window chunks, cover the L - 2 windows
    exactly (the kernel's launcher rejects anything else) and give every workgroup work."""
    from dnn_page_vectors_amd.ops import conv_pool as cops

    for N in (1, 3, 64, 128, 512, 4096):
        for L in (4, 5, 130, 131, 250, 1000, 5000, 20000):
            for cus in (8, 80, 256):
                nslots, nseg, sw = cops.f32_plan(N, L, cus)
                nw3 = L - 2
                assert sw % 128 == 0 and sw >= 128
                assert (nseg - 1) * sw < nw3 <= nseg * sw
                assert 1 <= nslots <= max(1, cus // 5) and nslots <= N * nseg


@pytest.mark.parametrize("p,mode", [(0.25, "element"), (0.3, "element"), (0.25, "token"), (0.0, "element")])
def test_f32_ordered_table_grad_matches_reference(p, mode):
    """ops/conv_pool.py::_f32_dtable_ordered (the fp32 table gradient of deterministic mode)
    against autograd through the reference embedding dropout + conv + max-pool."""
    from dnn_page_vectors_amd.ops import conv_pool as cops
    from dnn_page_vectors_amd.ops import reference as ref

    torch.manual_seed(0)
    N, L, V, E, F = 3, 40, 50, 16, 150
    ids = torch.randint(0, V, (N, L), dtype=torch.int32)
    table = torch.randn(V, E)
    w3, w4 = torch.randn(F, 3, E) * 0.2, torch.randn(F, 4, E) * 0.2
    b3, b4 = torch.randn(F) * 0.1, torch.randn(F) * 0.1
    seed, row_offset = 99, 1234
    tr = table.clone().requires_grad_(True)
    x = cops._embed_dropout_offset(ids, tr, p, seed, True, mode, row_offset)
    pooled, argmax = ref.conv_relu_maxpool(x, [w3, w4], [b3, b4])
    g = torch.randn_like(pooled)
    _, _, dx = ref.conv_maxpool_grads_at(x.detach(), [w3, w4], pooled, argmax, g)
    x.backward(dx)
    thr, tok, scale = cops._dropout_args(p, True, mode)
    dt = torch.zeros(V, E)
    cops._f32_dtable_ordered(g, pooled, argmax, ids, w3, w4, dt, seed, row_offset, thr, tok, scale)
    torch.testing.assert_close(dt, tr.grad, rtol=1e-5, atol=1e-5)
