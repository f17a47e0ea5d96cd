"""HIP kernel numerics vs plain-PyTorch fp32 references (run on MI355X: pytest -m gpu)."""
import pytest
import torch

from dnn_page_vectors_amd import _native
from dnn_page_vectors_amd.ops import conv_pool as cops
from dnn_page_vectors_amd.ops import dense as dops
from dnn_page_vectors_amd.ops import loss as lops
from dnn_page_vectors_amd.ops import reference as ref

pytestmark = pytest.mark.gpu
DEV = "cuda"


def bf(x):
    return x.bfloat16().float()


def test_native_hip_library_loaded():
    lib = _native.hip(required=True)
    assert lib is not None
    assert any("libpagevec_hip" in p for p in _native.loaded_libraries())


@pytest.mark.parametrize("N,L,p,mode", [(8, 37, 0.0, "element"), (5, 130, 0.25, "element"), (3, 64, 0.25, "token"),
                                        (6, 4, 0.0, "element"), (300, 45, 0.25, "element"),
                                        (12, 5000, 0.25, "element"),  # char-level page length
                                        # long-sequence table reduce (reduce7) and dW in every
                                        # compile-time dropout mode: off, element p = 0.3, token
                                        (5, 130, 0.0, "element"), (5, 130, 0.3, "element"),
                                        (4, 130, 0.25, "token"),
                                        # p = 2/16 (the chunked-CDSSM preset's 0.125): nibble >= 2
                                        (5, 130, 0.125, "element")])
def test_conv_pool_fwd_bwd(N, L, p, mode):
    torch.manual_seed(0)
    V, E, F = 97, 100, 150
    ids = torch.randint(0, V, (N, L), dtype=torch.int32, device=DEV)
    # bf16-representable operands: the kernels' bf16 copies are exact, so the fp32
    # reference sees the same values (only accumulation order differs)
    table = bf(torch.randn(V, E, device=DEV) * 0.5).requires_grad_(True)
    w3 = bf(torch.randn(F, 3, E, device=DEV) * 0.1).requires_grad_(True)
    w4 = bf(torch.randn(F, 4, E, device=DEV) * 0.1).requires_grad_(True)
    b3 = (torch.randn(F, device=DEV) * 0.1).requires_grad_(True)
    b4 = (torch.randn(F, device=DEV) * 0.1).requires_grad_(True)
    seed = 1234
    pooled, argmax = cops.conv_relu_maxpool_fused(ids, table, [w3, w4], [b3, b4], p, seed, True, mode)
    # reference on the bf16-rounded operands the kernel consumes
    tr = bf(table.detach()).requires_grad_(True)
    w3r = bf(w3.detach()).requires_grad_(True)
    w4r = bf(w4.detach()).requires_grad_(True)
    b3r = b3.detach().clone().requires_grad_(True)
    b4r = b4.detach().clone().requires_grad_(True)
    x = ref.embed_dropout(ids, tr, p, seed, True, mode)
    pr, ar = ref.conv_relu_maxpool(x, [w3r, w4r], [b3r, b4r])
    torch.testing.assert_close(pooled, pr, rtol=2e-3, atol=2e-3)
    live = pr > 1e-3
    agree = (argmax == ar) | ~live
    assert agree.float().mean() > 0.97
    g = torch.randn_like(pooled)
    (pooled * g).sum().backward()
    # the fp32 reference backward scatters through the KERNEL's argmax windows, so every
    # gradient is compared on every shape (near-ties in the forward cannot skip the check)
    xr = ref.embed_dropout(ids, tr, p, seed, True, mode)
    dws, dbs, dx = ref.conv_maxpool_grads_at(xr.detach(), [w3r.detach(), w4r.detach()], pooled.detach(), argmax,
                                             g)
    xr.backward(dx)
    torch.testing.assert_close(b3.grad, dbs[0], rtol=2e-3, atol=2e-3)
    torch.testing.assert_close(b4.grad, dbs[1], rtol=2e-3, atol=2e-3)
    torch.testing.assert_close(w3.grad, dws[0], rtol=1e-3, atol=2e-3)
    torch.testing.assert_close(w4.grad, dws[1], rtol=1e-3, atol=2e-3)
    torch.testing.assert_close(table.grad, tr.grad, rtol=1e-3, atol=2e-3)


@pytest.mark.parametrize("N,L,V,p", [(6, 130, 70000, 0.25), (3, 400, 70000, 0.0), (20, 45, 66000, 0.25)])
def test_conv_pool_bwd_word_vocab_u32_path(N, L, V, p):
    """Word-level vocabularies (dssm_cnn_v2/config.py:80-83, cnn_dssm_th.py:114-120): V >= 65535
    takes the 4-byte sort keys and the u32 reduce; dTable / dW vs the fp32 reference through
    the kernel's own argmax windows (untested on the GPU before)."""
    torch.manual_seed(3)
    E, F = 100, 150
    ids = torch.randint(0, V, (N, L), dtype=torch.int32, device=DEV)
    ids[:, ::7] = V - 1  # the top of the id range (and repeated tokens: runs in the sort)
    table = bf(torch.randn(V, E, device=DEV) * 0.5).requires_grad_(True)
    w3 = bf(torch.randn(F, 3, E, device=DEV) * 0.1).requires_grad_(True)
    w4 = bf(torch.randn(F, 4, E, device=DEV) * 0.1).requires_grad_(True)
    b3 = (torch.randn(F, device=DEV) * 0.1).requires_grad_(True)
    b4 = (torch.randn(F, device=DEV) * 0.1).requires_grad_(True)
    pooled, argmax = cops.conv_relu_maxpool_fused(ids, table, [w3, w4], [b3, b4], p, 77, True)
    g = torch.randn_like(pooled)
    (pooled * g).sum().backward()
    tr = bf(table.detach()).requires_grad_(True)
    xr = ref.embed_dropout(ids, tr, p, 77, True)
    dws, dbs, dx = ref.conv_maxpool_grads_at(xr.detach(), [bf(w3.detach()), bf(w4.detach())], pooled.detach(),
                                             argmax, g)
    xr.backward(dx)
    torch.testing.assert_close(table.grad, tr.grad, rtol=1e-3, atol=2e-3)
    torch.testing.assert_close(w3.grad, dws[0], rtol=1e-3, atol=2e-3)
    torch.testing.assert_close(w4.grad, dws[1], rtol=1e-3, atol=2e-3)
    torch.testing.assert_close(b3.grad, dbs[0], rtol=2e-3, atol=2e-3)


@pytest.mark.parametrize("V", [500, 70000])
def test_forward_emitted_keys_equal_emit_kernel(V):
    """The dTable sort keys written by the conv forward's epilogue (FWD_EMIT) give the same
    table gradient as the backward's emit kernel (2- and 4-byte keys)."""
    torch.manual_seed(4)
    E, F, N, L = 100, 150, 24, 300
    ids = torch.randint(1, V, (N, L), dtype=torch.int32, device=DEV)
    table0 = torch.randn(V, E, device=DEV) * 0.3
    w3, w4 = torch.randn(F, 3, E, device=DEV) * 0.1, torch.randn(F, 4, E, device=DEV) * 0.1
    b = [torch.randn(F, device=DEV) * 0.1, torch.randn(F, device=DEV) * 0.1]
    grads = []
    saved = cops.FWD_EMIT
    try:
        for fe in (False, True):
            cops.FWD_EMIT = fe
            t = table0.clone().requires_grad_(True)
            pooled, _ = cops.conv_relu_maxpool_fused(ids, t, [w3, w4], b, 0.25, 5, True)
            (pooled * torch.linspace(-1, 1, pooled.numel(), device=DEV).view_as(pooled)).sum().backward()
            grads.append(t.grad)
    finally:
        cops.FWD_EMIT = saved
    torch.testing.assert_close(grads[1], grads[0], rtol=1e-5, atol=1e-6)
    assert grads[0].abs().sum() > 0


@pytest.mark.parametrize("epw", [64, 512, 1024])
def test_dtable_reduce_long_runs_key_widths_agree(epw):
    """The dTable reduce (a wave walks epw sorted entries, runs carried across 64-entry
    sub-chunks) with 2-byte keys equals the 4-byte-key instantiation (the word-vocabulary
    path) at epw = 64 on Zipf-skewed ids whose hottest rows span many sub-chunks and waves
    (fp32 atomics between waves: equal up to rounding), and both match a torch fp32 scatter
    of the same sparse contributions."""
    torch.manual_seed(1)
    V, E, F, N, L = 500, 100, 150, 64, 300
    ranks = torch.arange(1, V, dtype=torch.float64)
    probs = ranks.pow(-1.1)
    ids = (torch.multinomial(probs / probs.sum(), N * L, replacement=True) + 1).view(N, L).to(torch.int32).to(DEV)
    table = bf(torch.randn(V, E, device=DEV) * 0.5)
    w3, w4 = bf(torch.randn(F, 3, E, device=DEV) * 0.1), bf(torch.randn(F, 4, E, device=DEV) * 0.1)
    b = [torch.zeros(F, device=DEV), torch.zeros(F, device=DEV)]
    grads = []
    saved = cops.REDUCE_EPW, cops.KEYS32
    try:
        for e, k32 in ((64, True), (epw, False)):
            cops.REDUCE_EPW, cops.KEYS32 = e, k32
            t = table.clone().requires_grad_(True)
            pooled, _ = cops.conv_relu_maxpool_fused(ids, t, [w3, w4], b, 0.0, 99, True)
            gp = torch.linspace(-1, 1, pooled.numel(), device=DEV).view_as(pooled)
            (pooled * gp).sum().backward()
            grads.append(t.grad)
    finally:
        cops.REDUCE_EPW, cops.KEYS32 = saved
    torch.testing.assert_close(grads[1], grads[0], rtol=1e-4, atol=3e-5)
    assert grads[0].abs().sum() > 0
    # fp32 reference of the sparse gradient: each (n, f) adds g * W[f, j] to row ids[n, a + j]
    with torch.no_grad():
        t = table.clone().requires_grad_(True)
        pooled, argmax = cops.conv_relu_maxpool_fused(ids, t, [w3, w4], b, 0.0, 99, True)
        g = gp * (pooled > 0)
        ref = torch.zeros(V, E, device=DEV)
        for k, w in ((3, w3), (4, w4)):
            sl = slice(0, F) if k == 3 else slice(F, 2 * F)
            a = argmax[:, sl].long()
            for j in range(k):
                rows = ids.gather(1, (a + j).clamp_max(L - 1)).long()
                ref.index_add_(0, rows.reshape(-1), (g[:, sl].unsqueeze(-1) * w[:, j].unsqueeze(0)).reshape(-1, E))
    torch.testing.assert_close(grads[1], ref, rtol=2e-3, atol=2e-4)


@pytest.mark.parametrize("variant", [0, 16384 + 64 + 5, 16384 + 128 + 5])
@pytest.mark.parametrize("N,L,p,mode", [(300, 45, 0.25, "element"), (40, 2000, 0.25, "element"), (7, 130, 0.25, "element"),
                                        (9, 301, 0.0, "element"), (9, 301, 0.3, "element"), (9, 301, 0.25, "token")])
def test_conv_forward_role_split_bit_identical(variant, N, L, p, mode):
    """The production v7 conv forward (768-thread workgroups: 8 MFMA waves + 4 loader waves
    that gather, mask and stage the next chunk) reproduces the v4 kernel (the previous
    production, 8 waves that all stage) bit for bit: pooled values and argmax windows, in
    every dropout mode (the A/B arm is built for p = 0.25 only)."""
    if variant != 0 and (p != 0.25 or mode != "element"):
        pytest.skip("A/B arm instantiated for the bench dropout mode only")
    torch.manual_seed(5)
    V, E, F = 500, 100, 150
    ids = torch.randint(1, V, (N, L), dtype=torch.int32, device=DEV)
    table = torch.randn(V, E, device=DEV) * 0.3
    w3, w4 = torch.randn(F, 3, E, device=DEV) * 0.1, torch.randn(F, 4, E, device=DEV) * 0.1
    b = [torch.randn(F, device=DEV) * 0.1, torch.randn(F, device=DEV) * 0.1]
    from dnn_page_vectors_amd.ops._common import lib as _lib
    lib = _lib()
    outs = []
    try:
        for v in (4096, variant):
            lib.pv_conv_set_dbg(v)
            with torch.no_grad():
                outs.append(cops.conv_relu_maxpool_fused(ids, table, [w3, w4], b, p, 11, True, mode))
            torch.cuda.synchronize()
    finally:
        lib.pv_conv_set_dbg(0)
    assert torch.equal(outs[0][0], outs[1][0])
    assert torch.equal(outs[0][1], outs[1][1])


@pytest.mark.parametrize("n,E", [(2, 100), (6, 100), (3, 37)])
def test_prep_towers_matches_per_tower_copies(n, E):
    """One-launch tower prep (pv_conv_prep_multi) == table_bf16 + pack_weights per tower, bit for bit
    (6 towers: two launches, the unshared-doc-tower v1 layout)."""
    g = torch.Generator(device=DEV).manual_seed(3)
    towers = [(torch.randn(1000 + 777 * i, E, device=DEV, generator=g), torch.randn(150, 3, E, device=DEV, generator=g),
               torch.randn(150, 4, E, device=DEV, generator=g)) for i in range(n)]
    got = cops.prep_towers(towers)
    for (t, w3, w4), (tb, pk) in zip(towers, got):
        assert torch.equal(tb, cops.table_bf16(t))
        assert torch.equal(pk, cops.pack_weights(w3, w4))


def test_conv_pool_eval_mode_no_dropout():
    V, E, F, N, L = 50, 100, 150, 4, 20
    ids = torch.randint(0, V, (N, L), dtype=torch.int32, device=DEV)
    table = torch.randn(V, E, device=DEV)
    w3, w4 = torch.randn(F, 3, E, device=DEV) * .1, torch.randn(F, 4, E, device=DEV) * .1
    b = [torch.zeros(F, device=DEV), torch.zeros(F, device=DEV)]
    a, _ = cops.conv_relu_maxpool_fused(ids, table, [w3, w4], b, 0.25, 1, False)
    r, _ = ref.conv_relu_maxpool(ref.embed_dropout(ids, bf(table), 0.25, 1, False), [bf(w3), bf(w4)], b)
    torch.testing.assert_close(a, r, rtol=2e-3, atol=2e-3)


@pytest.mark.parametrize("M,K,N,act", [(100, 300, 150, "relu"), (64, 512, 128, "none"), (33, 70, 17, "relu")])
def test_linear_act(M, K, N, act):
    x = bf(torch.randn(M, K, device=DEV)).requires_grad_(True)
    w = bf(torch.randn(N, K, device=DEV) * 0.05).requires_grad_(True)
    b = torch.randn(N, device=DEV, requires_grad=True)
    y = dops.linear_act(x, w, b, act)
    xr, wr = bf(x.detach()).requires_grad_(True), bf(w.detach()).requires_grad_(True)
    br = b.detach().clone().requires_grad_(True)
    yr = ref.linear_act(xr, wr, br, act)
    torch.testing.assert_close(y, yr, rtol=2e-3, atol=2e-3)
    g = torch.randn_like(y)
    (y * g).sum().backward()
    (yr * g).sum().backward()
    torch.testing.assert_close(b.grad, br.grad, rtol=1e-3, atol=1e-3)
    # the backward GEMMs take dz in bf16 (in-tree kernels, fp32 accumulation)
    for a_, r_ in ((w.grad, wr.grad), (x.grad, xr.grad)):
        torch.testing.assert_close(a_.float(), r_.float(), rtol=2e-2, atol=float(r_.abs().max()) * 1e-2)


@pytest.mark.parametrize("M,N,K,xbf", [(16384, 150, 300, False), (4096, 512, 512, True), (1000, 130, 70, False),
                                       (20000, 512, 128, True)])
def test_dense_backward_kernels(M, N, K, xbf):
    """dgrad on linear_act (W^T as the weight) and the split-row wgrad kernel (64 / 128
    tiles, partial slabs + column sums) vs fp32 GEMMs of the same bf16-rounded operands."""
    torch.manual_seed(5)
    dz = torch.randn(M, N, device=DEV)
    w = torch.randn(N, K, device=DEV) * 0.05
    x = torch.randn(M, K, device=DEV)
    if xbf:
        x = x.bfloat16()
    dzr, wr, xr = bf(dz), bf(w), x.float() if xbf else bf(x)
    dx = dops.dgrad_hip(dz, w)
    torch.testing.assert_close(dx, dzr @ wr, rtol=1e-3, atol=float((dzr @ wr).abs().max()) * 2e-3)
    ref_dw = dzr.t() @ xr
    for tile in (64, 128):
        dw = dops.wgrad_hip(dz, x, tile=tile)
        torch.testing.assert_close(dw, ref_dw, rtol=1e-3, atol=float(ref_dw.abs().max()) * 2e-3)
    out = torch.full((N, K), 7.0, device=DEV)
    dops.wgrad_hip(dz, x, out=out)  # overwrites a flat-gradient view
    torch.testing.assert_close(out, ref_dw, rtol=1e-3, atol=float(ref_dw.abs().max()) * 2e-3)


@pytest.mark.parametrize("grad", ["dense", "row_strided", "expanded"])
def test_l2norm(grad):
    """Backward with a dense gradient, a row-strided one (the loss kernels' padded (n, 160)
    gradient sliced to 150 columns, read in place) and a stride-0 expanded one."""
    x = torch.randn(37, 150, device=DEV, requires_grad=True)
    x2 = x.detach().clone().requires_grad_(True)
    y = dops.l2_normalize(x)
    yr = ref.l2_normalize(x2)
    torch.testing.assert_close(y, yr)
    if grad == "dense":
        g = torch.randn_like(y)
    elif grad == "row_strided":
        g = torch.randn(37, 160, device=DEV)[:, :150]
    else:
        g = torch.randn(1, 150, device=DEV).expand(37, 150)
    y.backward(g)
    yr.backward(g)
    torch.testing.assert_close(x.grad, x2.grad, rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("clip,J1,D", [(True, 4, 150), (False, 4, 150), (True, 4, 768), (True, 20, 128),
                                      (False, 64, 1024), (True, 1, 32)])
def test_explicit_loss(clip, J1, D):
    """The fused kernel's compile-time variants (D up to 1024 — BERT without projection is
    768 — and 1+J up to 64) against the fp32 expression; beyond them a loud error."""
    if J1 == 64:
        with pytest.raises(NotImplementedError):
            lops.dssm_explicit_loss(torch.zeros(2, 8, device=DEV), torch.zeros(2, 65, 8, device=DEV), 10.0)
    B = 40
    q = torch.relu(torch.randn(B, D, device=DEV))
    d = torch.relu(torch.randn(B, J1, D, device=DEV))
    qn = ref.l2_normalize(q).requires_grad_(True)
    dn = ref.l2_normalize(d).requires_grad_(True)
    loss, P = lops.dssm_explicit_loss(qn, dn, 10.0, clip)
    qn2 = qn.detach().clone().requires_grad_(True)
    dn2 = dn.detach().clone().requires_grad_(True)
    R = (qn2.unsqueeze(1) * dn2).sum(-1)
    if clip:
        R = R.clamp(0, 1)
    S = 10.0 * R
    Pr = torch.softmax(S, 1)[:, 0]
    lr = -torch.log(Pr.clamp(1e-7, 1 - 1e-7))
    torch.testing.assert_close(loss, lr, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(P, Pr, rtol=1e-4, atol=1e-5)
    loss.mean().backward()
    lr.mean().backward()
    torch.testing.assert_close(qn.grad, qn2.grad, rtol=1e-3, atol=1e-6)
    torch.testing.assert_close(dn.grad, dn2.grad, rtol=1e-3, atol=1e-6)


@pytest.mark.parametrize("B,M,D,clip", [(50, 200, 150, True), (130, 515, 128, False), (7, 7, 64, True)])
def test_inbatch_loss(B, M, D, clip):
    torch.manual_seed(1)
    q = torch.randn(B, D, device=DEV)
    dd = torch.randn(M, D, device=DEV)
    if clip:
        q, dd = q.abs(), dd.abs()
    qn = bf(ref.l2_normalize(q)).requires_grad_(True)
    dn = bf(ref.l2_normalize(dd)).requires_grad_(True)
    pos = torch.randint(0, M, (B,), device=DEV, dtype=torch.int32)
    loss, P = lops.inbatch_loss(qn, dn, pos, 10.0, clip)
    qn2 = qn.detach().clone().requires_grad_(True)
    dn2 = dn.detach().clone().requires_grad_(True)
    lr, _ = ref.inbatch_softmax_loss(qn2, dn2, pos, 10.0, clip)
    torch.testing.assert_close(loss, lr, rtol=2e-3, atol=2e-3)
    w = torch.rand(B, device=DEV)
    (loss * w).sum().backward()
    (lr * w).sum().backward()
    torch.testing.assert_close(qn.grad, qn2.grad, rtol=3e-2, atol=3e-3)
    torch.testing.assert_close(dn.grad, dn2.grad, rtol=3e-2, atol=3e-3)


@pytest.mark.parametrize("ver", [5, 3, 7])
@pytest.mark.parametrize("B,M,clip,D", [(700, 5000, True, 150), (4096, 16384, False, 150), (300, 20000, True, 150),
                                        (700, 5000, True, 128), (2048, 9000, False, 128)])
def test_inbatch_loss_split_shapes(ver, B, M, clip, D):
    """Shapes with several Y splits, >= 3 tiles per split (the ib3 LDS ring wraps), a
    partial last tile and row blocks past nx, for the kernel generations (5: ib5 on 32x32x16
    MFMAs for the query-row passes; 3: ib3, 16x16x32, everywhere; 7: the software-pipelined
    ib7 for every pass) vs the fp32 reference."""
    from dnn_page_vectors_amd.ops._common import lib as _lib

    L_ = _lib()
    old = L_.pv_ib_version()
    assert L_.pv_ib_set_version(ver) == 0
    try:
        torch.manual_seed(3)
        q = torch.randn(B, D, device=DEV)
        dd = torch.randn(M, D, device=DEV)
        # weakly correlated positives: with P+ ~ 1 the bf16-rounded positive term of dQ
        # cancels against the one-hot term (an O(1) relative error on a ~0 gradient row)
        dd[:B] = q + 2.0 * dd[:B]
        if clip:
            q, dd = q.abs(), dd.abs()
        qn = bf(ref.l2_normalize(q)).requires_grad_(True)
        dn = bf(ref.l2_normalize(dd)).requires_grad_(True)
        pos = torch.arange(B, device=DEV, dtype=torch.int32)
        loss, P = lops.inbatch_loss(qn, dn, pos, 10.0, clip)
        qn2 = qn.detach().clone().requires_grad_(True)
        dn2 = dn.detach().clone().requires_grad_(True)
        lr, _ = ref.inbatch_softmax_loss(qn2, dn2, pos, 10.0, clip)
        torch.testing.assert_close(loss, lr, rtol=2e-3, atol=2e-3)
        w = torch.rand(B, device=DEV)
        (loss * w).sum().backward()
        (lr * w).sum().backward()
        for a, b in ((qn.grad, qn2.grad), (dn.grad, dn2.grad)):
            rel = float((a - b).norm() / b.norm())
            assert rel < 3e-2, rel
            torch.testing.assert_close(a, b, rtol=5e-2, atol=float(b.abs().max()) * 2e-2)
    finally:
        L_.pv_ib_set_version(old)


def test_adam_matches_reference():
    from dnn_page_vectors_amd.ops.optim import FlatAdam, FlatParams

    torch.manual_seed(0)
    lin = torch.nn.Linear(33, 17).to(DEV)
    flat = FlatParams(lin.named_parameters())
    opt = FlatAdam(flat, lr=1e-2)
    p0 = flat.data.clone()
    m = torch.zeros_like(p0)
    v = torch.zeros_like(p0)
    for t in range(1, 4):
        flat.grad.copy_(torch.randn_like(flat.grad))
        g = flat.grad.clone()
        opt.step()
        ref.adam_keras_([p0], [g], [m], [v], t, 1e-2, 0.9, 0.999, 1e-8)
    torch.testing.assert_close(flat.data, p0, rtol=1e-5, atol=1e-6)


def test_adam_skip_flag():
    from dnn_page_vectors_amd.ops.optim import FlatAdam, FlatParams, grad_sumsq_and_finite

    lin = torch.nn.Linear(8, 4).to(DEV)
    flat = FlatParams(lin.named_parameters())
    opt = FlatAdam(flat)
    before = flat.data.clone()
    flat.grad.fill_(1.0)
    flat.grad[3] = float("nan")
    st = grad_sumsq_and_finite(flat.grad)
    assert float(st[1]) == 1.0
    opt.step(st[1:2])
    torch.testing.assert_close(flat.data, before)


def test_topk_cos():
    from dnn_page_vectors_amd.ops import topk as tops

    q = ref.l2_normalize(torch.randn(64, 150, device=DEV))
    pg = ref.l2_normalize(torch.randn(3000, 150, device=DEV))
    v, i = tops.topk_cos(q, pg, 10)
    vr, ir = tops._topk_torch(bf(q), bf(pg), 10, 1024)
    torch.testing.assert_close(v, vr, rtol=1e-3, atol=1e-3)
    assert (i[:, 0] == ir[:, 0]).float().mean() > 0.95


def test_cdssm_train_step_gpu():
    from dnn_page_vectors_amd.config import Configuration
    from dnn_page_vectors_amd.data.synthetic import SyntheticPairs, spec_from_config
    from dnn_page_vectors_amd.models.cdssm import CDSSM
    from dnn_page_vectors_amd.parallel import dist as pdist
    from dnn_page_vectors_amd.train.trainer import Trainer

    pdist.init_distributed()
    # memorising one fixed batch (dropout on): a working fwd / sparse bwd / Adam chain drives
    # the loss down fast (CPU reference: explicit 1.39 -> 0.02, in-batch 5.55 -> 0.56 in 40
    # steps); 30 steps on fresh random batches barely move the gamma=10 clipped-cosine loss
    for mode in ("explicit", "cross_gpu"):
        cfg = Configuration(feature_level="ngram", vocab_hash_size=3000, batch_size=64, query_length=45,
                            document_length=200, loss_mode=mode, lr=1e-2)
        tr = Trainer(cfg, CDSSM(cfg, 3000), torch.device(DEV))
        g = torch.Generator(device="cpu").manual_seed(0)
        pages = torch.randint(1, 3000, (512, 200), generator=g, dtype=torch.int32).to(DEV)
        idx = torch.randint(0, 512, (64, 4), generator=g).to(DEV)
        q, d = pages[idx[:, 0], :45].contiguous(), pages[idx]
        losses = [float(tr.train_step(q, d)["loss"]) for _ in range(40)]
        assert all(l == l for l in losses)
        assert losses[-1] < 0.5 * losses[0], (mode, losses[::8])


@pytest.mark.parametrize("plan,L,E", [("gather", 45, 512), ("counts", 300, 512), ("gather", 20, 64), ("counts", 20, 72),
                                      ("gather", 33, 1000)])
def test_embedding_bag(plan, L, E):
    from dnn_page_vectors_amd.ops import embedding as eops

    V, N = 1000, 33
    ids = torch.randint(0, V, (N, L), dtype=torch.int32, device=DEV)
    ids[:, L // 2:] = 0
    W = bf(torch.randn(V, E, device=DEV)).requires_grad_(True)
    Wr = W.detach().clone().requires_grad_(True)
    out = eops.embedding_bag(ids, W, pad=0, mean=True, plan=plan)
    cnt = (ids != 0).sum(1, keepdim=True).clamp(min=1).float()
    outr = ref.embedding_bag_sum(ids, Wr, 0) / cnt
    torch.testing.assert_close(out, outr, rtol=2e-2, atol=2e-2)
    g = torch.randn_like(out)
    (out * g).sum().backward()
    (outr * g).sum().backward()
    torch.testing.assert_close(W.grad, Wr.grad, rtol=2e-2, atol=2e-2)


def test_embedding_bag_sparse_backward_hot_tokens():
    """Gather plan's sparse backward (sort (token, slot) entries, sum runs, atomics): a hot
    token whose run spans hundreds of waves, pads, and the MLP query shape (N 4096, L 45,
    V 30000, E 512) against the fp32 reference."""
    from dnn_page_vectors_amd.ops import embedding as eops

    V, N, L, E = 30000, 4096, 45, 512
    g0 = torch.Generator(device=DEV).manual_seed(2)
    ids = torch.randint(1, V, (N, L), dtype=torch.int32, device=DEV, generator=g0)
    ids[torch.rand(N, L, device=DEV, generator=g0) < 0.3] = 7       # ~55k-entry run
    ids[torch.rand(N, L, device=DEV, generator=g0) < 0.4] = 0       # pads
    ids[:5] = 0                                                      # empty bags
    W = bf(torch.randn(V, E, device=DEV, generator=g0) * 0.1).requires_grad_(True)
    Wr = W.detach().clone().requires_grad_(True)
    out = eops.embedding_bag(ids, W, pad=0, mean=True, plan="gather")
    cnt = (ids != 0).sum(1, keepdim=True).clamp(min=1).float()
    outr = ref.embedding_bag_sum(ids, Wr, 0) / cnt
    torch.testing.assert_close(out, outr, rtol=2e-2, atol=2e-2)
    gy = torch.randn(N, E, device=DEV, generator=g0)
    (out * gy).sum().backward()
    (outr * gy).sum().backward()
    err = float((W.grad - Wr.grad).abs().max() / Wr.grad.abs().max())
    assert err < 1e-4, err
    assert float(W.grad[0].abs().max()) == 0.0


def test_trigram_hash_device():
    from dnn_page_vectors_amd.ops import embedding as eops

    texts = [b"statue of liberty", b"ab", b"new york city tour"]
    Lmax = 24
    buf = torch.zeros(len(texts), Lmax, dtype=torch.uint8)
    for i, t in enumerate(texts):
        buf[i, :len(t)] = torch.tensor(list(t), dtype=torch.uint8)
    lens = torch.tensor([len(t) for t in texts], dtype=torch.int32)
    got = eops.trigram_hash(buf.to(DEV), lens.to(DEV), 20, 30000).cpu()
    want = ref.fnv1a_trigram_ids(buf, lens, 20, 30000)
    assert torch.equal(got, want)
    from dnn_page_vectors_amd.data import text as T

    host = T.featurize_py([t.decode() for t in texts], "ngram", 20, hash_size=30000)
    assert got.tolist() == host


@pytest.mark.parametrize("B,N,D,k", [(100, 5000, 150, 10), (7, 300, 128, 16), (64, 64, 64, 1),
                                     (300, 3000, 768, 10), (50, 1000, 300, 5)])
def test_topk_hip_exact(B, N, D, k):
    from dnn_page_vectors_amd.ops import topk as tops

    torch.manual_seed(2)
    q = ref.l2_normalize(torch.randn(B, D, device=DEV))
    pg = ref.l2_normalize(torch.randn(N, D, device=DEV))
    v, i = tops._topk_hip(q, pg, k)
    vr, ir = tops._topk_torch(bf(q), bf(pg), k, 100000)
    torch.testing.assert_close(v, vr, rtol=1e-4, atol=1e-4)
    assert (i == ir).float().mean() > 0.97


def test_mlp_train_step_gpu():
    from dnn_page_vectors_amd.config import preset_config
    from dnn_page_vectors_amd.data.synthetic import SyntheticPairs, spec_from_config
    from dnn_page_vectors_amd.models import build_model
    from dnn_page_vectors_amd.parallel import dist as pdist
    from dnn_page_vectors_amd.train.trainer import Trainer

    pdist.init_distributed()
    cfg = preset_config("mlp_xgpu").replace(batch_size=256, document_length=400, cos_clip=False)
    tr = Trainer(cfg, build_model(cfg, cfg.vocab_hash_size), torch.device(DEV))
    data = SyntheticPairs(spec_from_config(cfg, cfg.vocab_hash_size, num_pages=2048), DEV)
    losses = [float(tr.train_step(*data.batch(256))["loss"]) for _ in range(40)]
    assert losses[-1] < losses[0] - 0.3


@pytest.mark.parametrize("D", [768, 320])  # wave-per-row LN backward / generic fallback
def test_add_layernorm_and_bias_gelu(D):
    from dnn_page_vectors_amd.ops import transformer as tops

    M = 70
    x = torch.randn(M, D, device=DEV).bfloat16().requires_grad_(True)
    r = torch.randn(M, D, device=DEV).bfloat16().requires_grad_(True)
    g = (1 + 0.1 * torch.randn(D, device=DEV)).requires_grad_(True)
    b = (0.1 * torch.randn(D, device=DEV)).requires_grad_(True)
    y = tops.add_layernorm(x, r, g, b)
    xr, rr = x.detach().float().requires_grad_(True), r.detach().float().requires_grad_(True)
    gr, br = g.detach().clone().requires_grad_(True), b.detach().clone().requires_grad_(True)
    yr = torch.nn.functional.layer_norm(xr + rr, (D,), gr, br, 1e-12)
    torch.testing.assert_close(y.float(), yr, rtol=2e-2, atol=3e-2)
    dy = torch.randn(M, D, device=DEV)
    (y.float() * dy).sum().backward()
    (yr * dy).sum().backward()
    torch.testing.assert_close(x.grad.float(), xr.grad, rtol=3e-2, atol=5e-2)
    torch.testing.assert_close(g.grad, gr.grad, rtol=3e-2, atol=1e-1)
    torch.testing.assert_close(b.grad, br.grad, rtol=3e-2, atol=1e-1)
    from dnn_page_vectors_amd.ops._common import lib

    # rows per wave of the add + LN forward (pv_ln_set_rpw): same per-row math, bit-identical,
    # with and without the dropout branch (M = 70: partial last waves)
    if D in (256, 512, 768, 1024):
        ys = []
        for rpw in (1, 2, 4):
            lib().pv_ln_set_rpw(rpw)
            try:
                with torch.no_grad():
                    ys.append((tops.add_layernorm(x, r, g, b), tops.add_layernorm(x, r, g, b, p=0.1, seed=7)))
            finally:
                lib().pv_ln_set_rpw(2)
        for a_, b_ in ys[1:]:
            assert torch.equal(a_, ys[0][0]) and torch.equal(b_, ys[0][1])
        # LN backward with / without the next-row prefetch (pv_ln_bwd_set_pf): bit-identical
        grads = []
        for pf in (0, 1):
            lib().pv_ln_bwd_set_pf(pf)
            try:
                xx, rr_ = x.detach().clone().requires_grad_(True), r.detach().clone().requires_grad_(True)
                gg, bb_ = g.detach().clone().requires_grad_(True), b.detach().clone().requires_grad_(True)
                (tops.add_layernorm(xx, rr_, gg, bb_, p=0.1, seed=7).float() * dy).sum().backward()
                grads.append((xx.grad, rr_.grad, gg.grad, bb_.grad))
            finally:
                lib().pv_ln_bwd_set_pf(1)
        for u_, v_ in zip(*grads):
            assert torch.equal(u_, v_)

    u0 = torch.randn(M, 3072, device=DEV).bfloat16()
    bb0 = torch.randn(3072, device=DEV)
    do = torch.randn(M, 3072, device=DEV)
    ur, bbr = u0.float().requires_grad_(True), bb0.clone().requires_grad_(True)
    orf = torch.nn.functional.gelu(ur + bbr, approximate="tanh")
    (orf * do).sum().backward()
    outs = {}
    for gv in (1, 2, 3):  # round-2 vector kernels / unrolled backward / unrolled both (pv_gelu_set_v)
        lib().pv_gelu_set_v(gv)
        try:
            u, bb = u0.clone().requires_grad_(True), bb0.clone().requires_grad_(True)
            o = tops.bias_gelu(u, bb)
            torch.testing.assert_close(o.float(), orf, rtol=2e-2, atol=2e-2)
            (o.float() * do).sum().backward()
            torch.testing.assert_close(bb.grad, bbr.grad, rtol=3e-2, atol=2e-1)
            torch.testing.assert_close(u.grad.float(), ur.grad, rtol=3e-2, atol=5e-2)
            outs[gv] = (o, u.grad)
        finally:
            lib().pv_gelu_set_v(2)
    for gv in (2, 3):  # same per-element math
        assert torch.equal(outs[1][0], outs[gv][0]) and torch.equal(outs[1][1], outs[gv][1])


@pytest.mark.parametrize("L", [37, 64, 300])  # generic / register (<=256) / register (<=512) softmax
def test_masked_attention(L):
    from dnn_page_vectors_amd.ops import transformer as tops

    B, H, d = 3, 4, 64
    q, k, v = (torch.randn(B, H, L, d, device=DEV).bfloat16().requires_grad_(True) for _ in range(3))
    mask = torch.ones(B, L, dtype=torch.int32, device=DEV)
    mask[1, 20:] = 0
    o = tops.attention(q, k, v, mask)
    qr, kr, vr = (t.detach().float().requires_grad_(True) for t in (q, k, v))
    s = (qr @ kr.transpose(-1, -2)) / 8.0
    s = s.masked_fill(~mask.bool()[:, None, None, :], float("-inf"))
    orf = torch.softmax(s, -1) @ vr
    torch.testing.assert_close(o.float(), orf, rtol=3e-2, atol=3e-2)
    do = torch.randn_like(orf)
    (o.float() * do).sum().backward()
    (orf * do).sum().backward()
    torch.testing.assert_close(q.grad.float(), qr.grad, rtol=5e-2, atol=5e-2)
    torch.testing.assert_close(v.grad.float(), vr.grad, rtol=5e-2, atol=5e-2)


def test_fp8_linear():
    from dnn_page_vectors_amd.ops import fp8 as fops

    torch.manual_seed(3)
    x = torch.randn(100, 512, device=DEV, requires_grad=True)
    w = (torch.randn(256, 512, device=DEV) * 0.05).requires_grad_(True)
    b = torch.randn(256, device=DEV, requires_grad=True)
    y = fops.fp8_linear(x, w, b, "tanh")
    yr = torch.tanh(torch.nn.functional.linear(fops._emulate(x.detach()), fops._emulate(w.detach()), b.detach()))
    torch.testing.assert_close(y, yr, rtol=1e-3, atol=1e-3)  # identical e4m3 rounding, fp32 accumulate
    exact = torch.tanh(torch.nn.functional.linear(x.detach(), w.detach(), b.detach()))
    assert float((y - exact).detach().abs().mean()) < 0.05  # e4m3 rounding noise only
    gy = torch.randn_like(y)
    (y * gy).sum().backward()
    # backward = bf16 GEMMs on the unquantised operands: compare with fp32 autograd through
    # the same (quantised) forward's activation mask
    xr = x.detach().clone().requires_grad_(True)
    wr = w.detach().clone().requires_grad_(True)
    br = b.detach().clone().requires_grad_(True)
    pre = torch.nn.functional.linear(xr, wr, br)
    dz = gy * (1 - y.detach() ** 2)
    (pre * dz).sum().backward()
    for got, want in ((x.grad, xr.grad), (w.grad, wr.grad), (b.grad, br.grad)):
        err = float((got - want).abs().max() / want.abs().max())
        assert err < 2e-2, err


@pytest.mark.parametrize("preset", ["bert_dp8", "longpage_fp8"])
def test_big_model_train_steps_gpu(preset):
    """Configs 4 / 5 on the HIP path: (1) the full-model parameter gradient of one step
    matches the fp32 PyTorch implementation of the same model, loss and weights (dtype
    fp32 precision scope: rocBLAS / MIOpen ops, no bf16 / fp8 kernel); (2) training on one
    fixed (memorisable) batch drives the loss down — the optimizer sees useful gradients."""
    from dnn_page_vectors_amd.config import preset_config
    from dnn_page_vectors_amd.data.synthetic import SyntheticPairs, spec_from_config
    from dnn_page_vectors_amd.models import build_model
    from dnn_page_vectors_amd.ops._common import precision_scope
    from dnn_page_vectors_amd.parallel import dist as pdist
    from dnn_page_vectors_amd.train.trainer import Trainer

    pdist.init_distributed()
    cfg = preset_config(preset)
    if preset == "bert_dp8":
        cfg = cfg.replace(bert_layers=2, batch_size=16, document_length=128, bert_dropout=0.0, lr=3e-4)
    else:
        cfg = cfg.replace(batch_size=64, document_length=2048)
    torch.manual_seed(5)
    tr = Trainer(cfg, build_model(cfg, cfg.vocab_hash_size), torch.device(DEV))
    data = SyntheticPairs(spec_from_config(cfg, cfg.vocab_hash_size, num_pages=256), DEV)
    q, d = data.batch(cfg.batch_size)

    def grad(fp32: bool) -> torch.Tensor:
        tr.flat.zero_grad()
        with precision_scope(cfg.replace(dtype="fp32", use_fp8=False) if fp32 else cfg):
            loss, _ = tr.compute_loss(q, d, 0)
            loss.backward()
        torch.cuda.synchronize()
        return tr.flat.grad.detach().clone()

    g_hip, g_ref = grad(False), grad(True)
    rel = float((g_hip - g_ref).norm() / g_ref.norm())
    cos = float(torch.nn.functional.cosine_similarity(g_hip, g_ref, dim=0))
    print(f"{preset}: grad rel err {rel:.4f} cos {cos:.5f}")
    for name, p_ in tr.flat.named:  # per-parameter view (diagnostics when the total disagrees)
        o, k, _ = tr.flat.offsets[name]
        gh, gr = g_hip[o:o + k], g_ref[o:o + k]
        print(f"  {name:40s} |g_ref| {float(gr.norm()):.3e} |g_hip| {float(gh.norm()):.3e} "
              f"rel {float((gh - gr).norm() / gr.norm().clamp_min(1e-30)):.4f}")
    assert torch.isfinite(g_hip).all()
    assert rel < (0.15 if cfg.use_fp8 else 0.05) and cos > (0.99 if cfg.use_fp8 else 0.999), (rel, cos)
    losses = [float(tr.train_step(q, d)["loss"]) for _ in range(25)]
    print(f"{preset}: loss {losses[0]:.4f} -> {losses[-1]:.4f}")
    assert all(l == l for l in losses)
    assert losses[-1] < 0.7 * losses[0], losses


@pytest.mark.parametrize("B,M,clip,block,wide,D", [(40, 160, False, 1 << 25, 0, 768), (40, 1000, True, 40 * 256, 0, 768),
                                                   (300, 3000, False, 300 * 700, 0, 768),
                                                   (64, 5000, True, 64 * 256, 0, 768),
                                                   (40, 160, False, 1 << 25, 1, 768), (40, 1000, True, 0, 1, 768),
                                                   (300, 3000, False, 0, 1, 768), (256, 2048, True, 0, 1, 768),
                                                   (33, 77, False, 0, 1, 256), (70, 300, True, 0, 1, 1024),
                                                   (50, 500, False, 0, 1, 384)])
def test_inbatch_loss_wide_rows_path(B, M, clip, block, wide, D, monkeypatch):
    """D = 768 (BERT): wide = 1, the flash kernels (loss.hip::ibw_kernel: S reduced over D
    across the workgroup's waves, never in HBM, no library GEMM); wide = 0, logits tiled over
    page-column blocks at the GEMM level (one block, or several with a partial last one)."""
    monkeypatch.setattr(lops, "IB_WIDE", bool(wide))
    if not wide:
        monkeypatch.setattr(lops, "ROWS_BLOCK_ELEMS", block)
    torch.manual_seed(4)
    qn = torch.randn(B, D, device=DEV)
    dn = torch.randn(M, D, device=DEV)
    pos = (torch.arange(B, device=DEV, dtype=torch.int32) * 3) % M
    dn[pos.long()] = qn + 0.5 * dn[pos.long()]  # positives correlated with their queries
    if clip:
        qn, dn = qn.abs(), dn.abs()
    qn = bf(ref.l2_normalize(qn)).requires_grad_(True)
    dn = bf(ref.l2_normalize(dn)).requires_grad_(True)
    if not wide:
        assert len(lops._col_blocks(B, M)) == (1 if block >= B * M else -(-M // max(256, block // B)))
    else:
        assert lops._wide_ok(D)
    loss, _ = lops.inbatch_loss(qn, dn, pos, 10.0, clip)
    q2, d2 = qn.detach().clone().requires_grad_(True), dn.detach().clone().requires_grad_(True)
    lr, _ = ref.inbatch_softmax_loss(q2, d2, pos, 10.0, clip)
    torch.testing.assert_close(loss, lr, rtol=2e-3, atol=2e-3)
    lm, _, _ = lops.inbatch_loss(qn.detach(), dn.detach(), pos, 10.0, clip, reduce=True)
    torch.testing.assert_close(lm, lr.mean(), rtol=2e-3, atol=2e-3)
    loss.mean().backward()
    lr.mean().backward()
    torch.testing.assert_close(qn.grad, q2.grad, rtol=3e-2, atol=3e-3)
    torch.testing.assert_close(dn.grad, d2.grad, rtol=3e-2, atol=3e-3)


def test_debug_kernels_flag_bad_ids_without_faulting():
    """libpagevec_hip_debug.so: out-of-range ids are recorded, not faulted on,
    and contribute zero rows exactly like the release kernels."""
    from dnn_page_vectors_amd.ops import embedding as eops

    V, E, F, N, L = 64, 100, 150, 6, 40
    torch.manual_seed(3)
    table = bf(torch.randn(V, E, device=DEV)).requires_grad_(True)
    ws = [bf(torch.randn(F, k, E, device=DEV) * 0.1).requires_grad_(True) for k in (3, 4)]
    bs = [torch.zeros(F, device=DEV, requires_grad=True) for _ in range(2)]
    ids = torch.randint(0, V, (N, L), dtype=torch.int32, device=DEV)
    _native.use_debug_kernels(True)
    try:
        _native.debug_status(reset=True)
        out, _ = cops.conv_relu_maxpool_fused(ids, table, ws, bs, 0.0, 1, True)
        out.sum().backward()
        torch.cuda.synchronize()
        assert _native.debug_status() == {}
        assert any("libpagevec_hip_debug" in p for p in _native.loaded_libraries())
        bad = ids.clone()
        bad[1, 5] = V + 7
        bad[2, 0] = -3
        table.grad = None
        out_b, _ = cops.conv_relu_maxpool_fused(bad, table, ws, bs, 0.0, 1, True)
        out_b.sum().backward()
        eops.embedding_bag(bad, table.detach(), pad=0)
        torch.cuda.synchronize()
        st = _native.debug_status()
        assert "id out of range" in st.get("convfwd", []), st
        assert "id out of range" in st.get("embed", []), st
        ref_tab = torch.cat([table.detach(), torch.zeros(1, E, device=DEV)])  # invalid -> zero row
        x = ref_tab[torch.where((bad >= 0) & (bad < V), bad.long(), torch.full_like(bad.long(), V))]
        pr, _ = ref.conv_relu_maxpool(x, [w.detach() for w in ws], [b.detach() for b in bs])
        torch.testing.assert_close(out_b, pr, rtol=2e-3, atol=2e-3)
    finally:
        _native.use_debug_kernels(False)


@pytest.mark.parametrize("L,H", [(32, 4), (37, 4), (64, 12), (65, 4), (200, 4), (256, 12), (300, 6)])
@pytest.mark.parametrize("qg,dma", [(1, 0), (2, 0), (4, 0), (1, 1), (2, 1)])
def test_fused_attention_packed_qkv(L, H, qg, dma):
    """attention.hip (online softmax fwd, dK/dV + dQ bwd) vs an fp32 reference on the same
    bf16 packed QKV, with key padding; qg = 16-row groups per wave of every kernel (the
    workgroup owns 64 qg rows; partial blocks at L = 37 / 65 / 200 / 300)."""
    from dnn_page_vectors_amd.ops import transformer as tops
    from dnn_page_vectors_amd.ops._common import lib

    lib().pv_attn_set_qg(qg, qg, qg)
    lib().pv_attn_set_fwd_dma(dma)  # forward K / V tiles by LDS-DMA
    try:
        _attention_case(L, H, tops)
    finally:
        lib().pv_attn_set_qg(0, 0, 0)
        lib().pv_attn_set_fwd_dma(0)


def _attention_case(L, H, tops):
    torch.manual_seed(L)
    N, d = 3, 64
    qkv = (torch.randn(N, L, 3 * H * d, device=DEV) * 0.5).bfloat16().requires_grad_(True)
    mask = torch.ones(N, L, dtype=torch.int32, device=DEV)
    mask[1, L // 2:] = 0
    mask[2, 5:9] = 0
    o = tops.fused_attention(qkv, mask, H)
    ref_in = qkv.detach().float().requires_grad_(True)
    q, k, v = ref_in.view(N, L, 3, H, d).permute(2, 0, 3, 1, 4)
    s = (q @ k.transpose(-1, -2)) / 8.0
    s = s.masked_fill(~mask.bool()[:, None, None, :], float("-inf"))
    orf = (torch.softmax(s, -1) @ v).transpose(1, 2).reshape(N, L, H * d)
    torch.testing.assert_close(o.float(), orf, rtol=2e-2, atol=2e-2)
    do = torch.randn_like(orf)
    (o.float() * do).sum().backward()
    (orf * do).sum().backward()
    g, gr = qkv.grad.float().view(N, L, 3, H * d), ref_in.grad.view(N, L, 3, H * d)
    for slot in range(3):
        scale = gr[:, :, slot].abs().max()
        err = (g[:, :, slot] - gr[:, :, slot]).abs().max() / scale
        assert err < 3e-2, (slot, float(err))


def test_packed_attention_qkv_projection_grads():
    """Packed query (L 32) + page (L 256) segments through the QKV projection and the fused
    attention: the projection's weight and bias gradients match fp32 torch."""
    from dnn_page_vectors_amd.ops import transformer as tops

    torch.manual_seed(5)
    H, d, Hd = 4, 64, 256
    shapes = [(6, 32), (3, 256)]
    T = sum(N * L for N, L in shapes)
    x = (torch.randn(T, Hd, device=DEV) * 0.5).bfloat16().requires_grad_(True)
    w = (torch.randn(3 * H * d, Hd, device=DEV) * 0.05).requires_grad_(True)
    b = (torch.randn(3 * H * d, device=DEV) * 0.1).requires_grad_(True)
    masks = [torch.ones(N, L, dtype=torch.int32, device=DEV) for N, L in shapes]
    masks[1][1, 200:] = 0
    out = tops.packed_attention(tops.linear(x, w, b), masks, shapes, H)
    do = torch.randn_like(out.float())
    (out.float() * do).sum().backward()
    xr = x.detach().float().requires_grad_(True)
    wr = w.detach().bfloat16().float().requires_grad_(True)
    br = b.detach().bfloat16().float().requires_grad_(True)
    qr = xr @ wr.t() + br
    outs, off = [], 0
    for (N, L), m in zip(shapes, masks):
        qkv_s = qr[off:off + N * L].view(N, L, 3, H, d).permute(2, 0, 3, 1, 4)
        s_ = (qkv_s[0] @ qkv_s[1].transpose(-1, -2)) / 8.0
        s_ = s_.masked_fill(~m.bool()[:, None, None, :], float("-inf"))
        outs.append((torch.softmax(s_, -1) @ qkv_s[2]).transpose(1, 2).reshape(N * L, H * d))
        off += N * L
    (torch.cat(outs) * do).sum().backward()
    for got, want in ((w.grad, wr.grad), (b.grad, br.grad)):
        err = (got.float() - want).abs().max() / want.abs().max()
        assert err < 3e-2, float(err)


@pytest.mark.parametrize("model", ["cdssm", "mlp"])
def test_hipgraph_step_matches_eager(model):
    """Trainer(graph=True): the captured + replayed step gives the eager trajectory (no
    dropout: identical math; replays also keep advancing Adam's device step counter)."""
    from dnn_page_vectors_amd.config import Configuration
    from dnn_page_vectors_amd.models import build_model
    from dnn_page_vectors_amd.parallel import dist as pdist
    from dnn_page_vectors_amd.train.trainer import Trainer

    pdist.set_info(pdist.DistInfo(device=torch.device(DEV)))
    cfg = Configuration(model=model, feature_level="ngram", vocab_hash_size=500, query_length=12,
                        document_length=64, batch_size=32, embedding_dim=100, dropout_prob=(0.0, 0.5),
                        loss_mode="in_batch", mlp_dims=(64, 64, 32), hidden_dims=64)
    g = torch.Generator().manual_seed(3)
    data = [(torch.randint(1, 500, (32, 12), generator=g, dtype=torch.int32).to(DEV),
             torch.randint(1, 500, (32, 4, 64), generator=g, dtype=torch.int32).to(DEV)) for _ in range(6)]
    runs = []
    for graph in (False, True):
        torch.manual_seed(0)
        tr = Trainer(cfg, build_model(cfg, 500), torch.device(DEV), graph=graph)
        losses = [float(tr.train_step(q, d)["loss"]) for q, d in data]
        runs.append((losses, tr.flat.data.clone(), tr.opt.step_count, tr._graph is not None))
    (le, pe, ce, _), (lg, pg, cg, captured) = runs
    assert captured and ce == cg == 6
    for a, b in zip(le, lg):
        assert abs(a - b) <= 1e-3 * max(1.0, abs(a)), (le, lg)
    torch.testing.assert_close(pg, pe, rtol=1e-3, atol=1e-4)


def test_hipgraph_bert_many_unfenced_replays():
    """BERT (config 4) step in a hipGraph, 40 unfenced replays over pre-built batches (the
    bench.py pattern): replays track the eager trajectory and never fault (the token
    embedding's backward is an index_add_ scatter, not torch's sort + unique_by_key)."""
    from dnn_page_vectors_amd.config import preset_config
    from dnn_page_vectors_amd.data.synthetic import SyntheticPairs, spec_from_config
    from dnn_page_vectors_amd.models import build_model
    from dnn_page_vectors_amd.parallel import dist as pdist
    from dnn_page_vectors_amd.train.trainer import Trainer

    pdist.set_info(pdist.DistInfo(device=torch.device(DEV)))
    cfg = preset_config("bert_dp8").replace(bert_layers=2, batch_size=16, document_length=64, query_length=16,
                                            bert_dropout=0.0)
    data = SyntheticPairs(spec_from_config(cfg, cfg.vocab_hash_size, num_pages=512), DEV, seed=5)
    pool = [data.batch(cfg.batch_size) for _ in range(4)]
    runs = []
    for graph in (False, True):
        torch.manual_seed(0)
        tr = Trainer(cfg, build_model(cfg, cfg.vocab_hash_size), torch.device(DEV), graph=graph, graph_fence=False)
        losses = [tr.train_step(*pool[i % 4])["loss"].clone() for i in range(40)]
        torch.cuda.synchronize()
        runs.append(([float(l) for l in losses], tr._graph is not None))
    (le, _), (lg, captured) = runs
    assert captured
    assert all(l == l for l in lg)
    for a, b in zip(le[:8], lg[:8]):
        assert abs(a - b) <= 2e-2 * max(1.0, abs(a)), (le, lg)


@pytest.mark.parametrize("T", [65536, 8192, 1000])
def test_wgrad_split_k_matches_fp32(T):
    from dnn_page_vectors_amd.ops import transformer as tf

    torch.manual_seed(7)
    dy = torch.randn(T, 768, device=DEV).to(torch.bfloat16)
    x = torch.randn(T, 384, device=DEV).to(torch.bfloat16)
    got = tf.wgrad_f32(dy, x)
    want = dy.double().t() @ x.double()
    assert got.dtype == torch.float32 and got.shape == (768, 384)
    err = (got.double() - want).abs().max() / want.abs().max()
    assert err < 1e-5, float(err)


@pytest.mark.parametrize("n", [3_000_003, 16_777_216])
def test_adam_and_sumsq_large_flat(n):
    """Large flat buffers: the unrolled (two 16-byte groups per trip) Adam path and the
    vectorised sum-of-squares, including the scalar tails."""
    from dnn_page_vectors_amd.ops._common import P, check, lib, stream

    torch.manual_seed(1)
    p = torch.randn(n, device=DEV)
    g = torch.randn(n, device=DEV)
    m = torch.randn(n, device=DEV).abs() * 0.1
    v = torch.randn(n, device=DEV).abs() * 0.01
    pr, mr, vr = p.clone(), m.clone(), v.clone()
    check(lib().pv_adam(P(p), P(g), P(m), P(v), n, 5, 1e-3, 0.9, 0.999, 1e-8, 0.0, 0, None, stream()), "pv_adam")
    ref.adam_keras_([pr], [g], [mr], [vr], 5, 1e-3, 0.9, 0.999, 1e-8)
    torch.testing.assert_close(m, mr, rtol=3e-5, atol=1e-6)  # FMA contraction vs torch's op order
    torch.testing.assert_close(v, vr, rtol=3e-5, atol=1e-6)
    torch.testing.assert_close(p, pr, rtol=1e-5, atol=1e-6)
    out = torch.zeros(2, device=DEV)
    check(lib().pv_sumsq(P(g), n, P(out), stream()), "pv_sumsq")
    want = float((g.double() ** 2).sum())
    assert abs(float(out[0]) - want) / want < 1e-4 and float(out[1]) == 0.0
    g[n // 3] = float("inf")
    out.zero_()
    check(lib().pv_sumsq(P(g[1:]), n - 1, P(out), stream()), "pv_sumsq")  # misaligned start
    assert float(out[1]) == 1.0


@pytest.mark.parametrize("D,p,with_bias", [(768, 0.1, True), (768, 0.25, False), (256, 0.0, True),
                                            (256, 0.0, False), (1024, 0.5, True)])
def test_add_layernorm_fused_dropout(D, p, with_bias):
    """LayerNorm(dropout(x + xb) + r) (wave-per-row fused kernel, counter-hash mask, folded
    linear bias) vs the fp32 reference with the same mask (ops/reference.py::dropout_keep_mask);
    gradients of x (masked), r (unmasked) and xb (column sums) from the one-pass backward."""
    from dnn_page_vectors_amd.ops import transformer as tf

    torch.manual_seed(3)
    M = 301  # odd: the 2-rows-per-wave forward recomputes (but does not store) a tail row
    x = bf(torch.randn(M, D, device=DEV)).requires_grad_(True)
    r = bf(torch.randn(M, D, device=DEV)).requires_grad_(True)
    g = (1.0 + 0.1 * torch.randn(D, device=DEV)).requires_grad_(True)
    b = (0.1 * torch.randn(D, device=DEV)).requires_grad_(True)
    xb = (0.2 * torch.randn(D, device=DEV)).requires_grad_(True) if with_bias else None
    seed = 987654
    y = tf.add_layernorm(x.to(torch.bfloat16), r.to(torch.bfloat16), g, b, 1e-12, p=p, seed=seed, bias=xb)
    x2, r2 = x.detach().clone().requires_grad_(True), r.detach().clone().requires_grad_(True)
    g2, b2 = g.detach().clone().requires_grad_(True), b.detach().clone().requires_grad_(True)
    xb2 = xb.detach().clone().requires_grad_(True) if with_bias else None
    xin = x2 + xb2 if with_bias else x2
    if p > 0:
        keep = ref.dropout_keep_mask(seed, M, D, p, device=DEV).float()
        hh = xin * keep * (256.0 / (256.0 - ref.dropout_threshold(p))) + r2
    else:
        hh = xin + r2
    yr = torch.nn.functional.layer_norm(hh, (D,), g2, b2, 1e-12)
    torch.testing.assert_close(y.float(), yr, rtol=2e-2, atol=3e-2)
    w = torch.randn(M, D, device=DEV)
    (y.float() * w).sum().backward()
    (yr * w).sum().backward()
    pairs = [(x.grad, x2.grad), (r.grad, r2.grad)] + ([(xb.grad, xb2.grad)] if with_bias else [])
    for a_, b_ in pairs:
        err = (a_.float() - b_).abs().max() / b_.abs().max()
        assert err < 3e-2, float(err)
    torch.testing.assert_close(g.grad, g2.grad, rtol=3e-2, atol=0.5)
    torch.testing.assert_close(b.grad, b2.grad, rtol=3e-2, atol=0.5)
    if p > 0:  # dropped positions get exactly zero gradient through the branch
        assert float(x.grad[keep == 0].abs().max()) == 0.0


def test_bert_packed_dual_tower_matches_separate_towers():
    """BertDualEncoder.forward packs queries and pages into one token batch (one GEMM per
    linear layer, per-group attention on offset pointers); outputs and every parameter
    gradient must match running the two towers separately (no dropout)."""
    from dnn_page_vectors_amd.config import preset_config
    from dnn_page_vectors_amd.models import build_model
    from dnn_page_vectors_amd.models.base import TwoTowerModel

    cfg = preset_config("bert_dp8").replace(bert_layers=2, bert_dropout=0.0, query_length=32, document_length=96)
    m = build_model(cfg, cfg.vocab_hash_size).to(DEV).train()
    g = torch.Generator().manual_seed(0)
    q = torch.randint(1, 30000, (8, 32), generator=g, dtype=torch.int32).to(DEV)
    d = torch.randint(1, 30000, (8, 2, 96), generator=g, dtype=torch.int32).to(DEV)
    d[:, :, 80:] = 0  # padding in the pages
    wq = torch.randn(8, 768, device=DEV)
    wd = torch.randn(8, 2, 768, device=DEV)
    grads = []
    for packed in (True, False):
        m.zero_grad(set_to_none=True)
        qv, dv = m(q, d) if packed else TwoTowerModel.forward(m, q, d)
        ((qv * wq).sum() + (dv * wd).sum()).backward()
        grads.append((qv.detach(), dv.detach(), {n: p.grad.detach().clone() for n, p in m.named_parameters()
                                                 if p.grad is not None}))
    (qa, da, ga), (qb, db, gb) = grads
    torch.testing.assert_close(qa, qb, rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(da, db, rtol=2e-2, atol=2e-2)
    assert ga.keys() == gb.keys()
    for n in ga:
        err = float((ga[n] - gb[n]).abs().max() / gb[n].abs().max().clamp_min(1e-12))
        assert err < 5e-2, (n, err)


def test_embedding_bag_counts_split_k():
    """Counts plan at a vocabulary large enough for the V-split batched GEMM (V // 8 >= 2048)."""
    from dnn_page_vectors_amd.ops import embedding as eops

    torch.manual_seed(11)
    V, N, L, E = 16384, 40, 300, 64
    ids = torch.randint(1, V, (N, L), dtype=torch.int32, device=DEV)
    ids[:, 250:] = 0
    W = bf(torch.randn(V, E, device=DEV)).requires_grad_(True)
    out = eops.embedding_bag(ids, W, plan="counts")
    Wr = W.detach().clone().requires_grad_(True)
    outr = ref.embedding_bag_sum(ids, Wr, 0) / (ids != 0).sum(1, keepdim=True).float()
    torch.testing.assert_close(out, outr, rtol=1e-2, atol=1e-2)
    g = torch.randn_like(outr)
    (out * g).sum().backward()
    (outr * g).sum().backward()
    torch.testing.assert_close(W.grad, Wr.grad, rtol=2e-2, atol=2e-2)


def test_cdssm_recall_quality_guard():
    """Training-quality guard for the headline config, on bench.py's own protocol (so it
    guards the number the driver reports): CDSSM-300d (B 4096, cross-GPU loss on one rank,
    in-batch softmax scale 40), 25 steps cycling a pool of 4 pre-built batches (bench warmup +
    timed steps), then fresh synthetic batches up to 1000 steps; Recall@10 on the bench's 2048
    held-out pairs must reach 0.38.  This protocol measures 0.443-0.452 (round-3 / round-4
    driver and builder benches); 1000 fresh-batch steps alone give 0.35-0.40 over data seeds
    and reduction modes (tools/recall_spread.py, profiles/r4_quality/).  A kernel regression
    that halves the learning signal lands near the reference-head plateau (~0.15-0.2,
    profiles/quality_r2_final.md) and fails."""
    from dnn_page_vectors_amd.config import preset_config
    from dnn_page_vectors_amd.data.synthetic import SyntheticPairs, spec_from_config
    from dnn_page_vectors_amd.eval.retrieval import recall_at_k
    from dnn_page_vectors_amd.models import build_model
    from dnn_page_vectors_amd.parallel import dist as pdist
    from dnn_page_vectors_amd.train.trainer import Trainer

    pdist.set_info(pdist.DistInfo(device=torch.device(DEV)))
    cfg = preset_config("cdssm_ngram_bf16")
    V = cfg.vocab_hash_size
    model = build_model(cfg, V)
    tr = Trainer(cfg, model, torch.device(DEV))
    data = SyntheticPairs(spec_from_config(cfg, V, num_pages=65536), DEV, seed=1337)
    pool = [data.batch(cfg.batch_size) for _ in range(4)]
    for i in range(25):
        m = tr.train_step(*pool[i % 4])
    for _ in range(1000 - 25):
        m = tr.train_step(*data.batch(cfg.batch_size))
    qe, pe = data.eval_set(2048, seed=7)
    qv, pv = model.encode(qe, "query"), model.encode(pe, "doc")
    r = recall_at_k(qv, pv, torch.arange(2048, device=DEV), k=10)
    # the HIP top-k agrees with an exact torch top-k on the same (bf16) vectors
    from dnn_page_vectors_amd.ops import topk as tops

    _, ir = tops._topk_torch(bf(qv), bf(pv), 10, 1 << 20)
    r_ref = float((ir == torch.arange(2048, device=DEV).view(-1, 1)).any(1).float().mean())
    assert float(m["loss"]) == float(m["loss"])
    print(f"recall@10 after 1000 steps: {r:.4f} (exact top-k {r_ref:.4f})")
    assert abs(r - r_ref) <= 2.0 / 2048, (r, r_ref)
    assert r >= 0.38, r


def test_resume_restores_device_adam_step(tmp_path):
    """the HIP Adam takes its bias corrections from the DEVICE step
    counter; a resumed run must continue at the same count.  Train 4 steps uninterrupted
    vs 2 steps -> checkpoint -> fresh Trainer -> resume -> 2 steps: the last update of
    both runs must agree (with t_dev restarting at 0 the resumed update is ~3x larger)."""
    from dnn_page_vectors_amd.config import Configuration
    from dnn_page_vectors_amd.io import checkpoint as ck
    from dnn_page_vectors_amd.models.cdssm import CDSSM
    from dnn_page_vectors_amd.parallel import dist as pdist
    from dnn_page_vectors_amd.train.trainer import Trainer

    pdist.set_info(pdist.DistInfo(device=torch.device(DEV)))
    cfg = Configuration(feature_level="ngram", vocab_hash_size=500, query_length=12, document_length=64,
                        batch_size=32, loss_mode="explicit", experiment_root_directory=str(tmp_path))
    g = torch.Generator().manual_seed(4)
    data = [(torch.randint(1, 500, (32, 12), generator=g, dtype=torch.int32).to(DEV),
             torch.randint(1, 500, (32, 4, 64), generator=g, dtype=torch.int32).to(DEV)) for _ in range(4)]
    ta = Trainer(cfg, CDSSM(cfg, 500), torch.device(DEV))
    for q, d in data[:3]:
        ta.train_step(q, d)
    before_a = ta.flat.data.clone()
    ta.train_step(*data[3])
    delta_a = ta.flat.data - before_a

    tb = Trainer(cfg, CDSSM(cfg, 500), torch.device(DEV))
    for q, d in data[:2]:
        tb.train_step(q, d)
    ck.save_epoch(tb, str(tmp_path / "ck"), 1)
    tc = Trainer(cfg, CDSSM(cfg, 500), torch.device(DEV))
    assert ck.resume(tc, str(tmp_path / "ck"))
    assert tc.opt.step_count == 2 and float(tc.opt.t_dev[0]) == 2.0
    tc.train_step(*data[2])
    before_c = tc.flat.data.clone()
    tc.train_step(*data[3])
    delta_c = tc.flat.data - before_c
    torch.cuda.synchronize()
    assert float(tc.opt.t_dev[0]) == 4.0
    rel = float((delta_c - delta_a).norm() / delta_a.norm())
    assert rel < 0.05, rel
    torch.testing.assert_close(tc.flat.data, ta.flat.data, rtol=1e-3, atol=2e-4)


@pytest.mark.parametrize("n,kbytes,end_bit", [(1, 2, 15), (100, 2, 15), (4095, 2, 15), (4096, 4, 15), (4097, 2, 8),
                                              (1_000_003, 2, 15), (17_203_200, 2, 15), (300_001, 4, 23),
                                              (70_000, 4, 32), (184_320, 2, 15), (2_000_000, 4, 20)])
def test_radix_sort_matches_stable_sort(n, kbytes, end_bit):
    """The dTable sort (radix_sort.hip) == torch's stable sort: same keys, same input
    positions (stability) — Zipf-skewed keys with a sentinel."""
    g = torch.Generator().manual_seed(n)
    hi = min(1 << end_bit, 60000 if kbytes == 2 else 1 << 31)
    k = (torch.rand(n, generator=g) ** 3 * (hi - 1)).long()  # skewed toward small keys
    k[::7] = hi - 1  # many equal keys (the dead-entry sentinel pattern)
    if kbytes == 4 and end_bit == 32:
        k = torch.randint(0, 1 << 32, (n,), generator=g, dtype=torch.int64)
    dt = torch.int16 if kbytes == 2 else torch.int32
    keys = k.to(torch.int64)
    kin = (keys - (1 << 16) * (keys >= (1 << 15)) if kbytes == 2 else keys - (1 << 32) * (keys >= (1 << 31))).to(dt)
    kin = kin.to(DEV)
    skeys = torch.empty_like(kin)
    svals = torch.empty(n, dtype=torch.int32, device=DEV)
    cops.sort_pairs_iota(kin, skeys, svals, end_bit)
    ref_k, ref_i = torch.sort(keys, stable=True)
    mask = (1 << 16) - 1 if kbytes == 2 else (1 << 32) - 1
    got_k = skeys.cpu().to(torch.int64) & mask
    assert torch.equal(got_k, ref_k)
    assert torch.equal(svals.cpu().to(torch.int64), ref_i)


def test_hipgraph_cdssm_unfenced_fresh_batches():
    """CDSSM steps replayed from a hipGraph with NO per-replay sync while eager work (a fresh
    synthetic batch, i.e. new allocations) runs between replays: the pattern that faulted in
    rocPRIM's memset-reset onesweep sort after ~97 replays.  The in-tree radix sort makes the
    captured step self-contained; 160 replays must run clean and keep learning signal finite."""
    from dnn_page_vectors_amd.config import preset_config
    from dnn_page_vectors_amd.data.synthetic import SyntheticPairs, spec_from_config
    from dnn_page_vectors_amd.models import build_model
    from dnn_page_vectors_amd.parallel import dist as pdist
    from dnn_page_vectors_amd.train.trainer import Trainer

    pdist.set_info(pdist.DistInfo(device=torch.device(DEV)))
    cfg = preset_config("cdssm_ngram_bf16").replace(batch_size=128, document_length=512)
    data = SyntheticPairs(spec_from_config(cfg, cfg.vocab_hash_size, num_pages=8192), DEV, seed=3)
    tr = Trainer(cfg, build_model(cfg, cfg.vocab_hash_size), torch.device(DEV), graph=True, graph_fence=False)
    losses = []
    for _ in range(160):
        q, d = data.batch(cfg.batch_size)
        losses.append(tr.train_step(q, d)["loss"].clone())
    torch.cuda.synchronize()
    assert tr._graph is not None
    vals = [float(l) for l in losses]
    assert all(v == v and v < 50 for v in vals), vals[-5:]


@pytest.mark.parametrize("model", ["cdssm", "mlp", "bert"])
def test_direct_flat_grad_writes_match_autograd(model, monkeypatch):
    """ops/grad_sink.py: ops writing parameter gradients straight into the flat buffer give
    the gradients autograd's AccumulateGrad path gives (one step, same data and init)."""
    from dnn_page_vectors_amd.config import Configuration, preset_config
    from dnn_page_vectors_amd.models import build_model
    from dnn_page_vectors_amd.ops import grad_sink
    from dnn_page_vectors_amd.parallel import dist as pdist
    from dnn_page_vectors_amd.train.trainer import Trainer

    pdist.set_info(pdist.DistInfo(device=torch.device(DEV)))
    if model == "bert":
        cfg = preset_config("bert_dp8").replace(bert_layers=2, batch_size=16, document_length=64, query_length=16,
                                                bert_dropout=0.0)
        V = cfg.vocab_hash_size
    else:
        cfg = Configuration(model=model, feature_level="ngram", vocab_hash_size=500, query_length=12,
                            document_length=64, batch_size=32, embedding_dim=100, dropout_prob=(0.0, 0.5),
                            loss_mode="in_batch", mlp_dims=(64, 64, 32), hidden_dims=64)
        V = 500
    if model == "bert":
        from dnn_page_vectors_amd.data.synthetic import SyntheticPairs, spec_from_config

        q, d = SyntheticPairs(spec_from_config(cfg, V, num_pages=512), DEV, seed=5).batch(cfg.batch_size)
    else:
        g = torch.Generator().manual_seed(4)
        q = torch.randint(1, V, (32, 12), generator=g, dtype=torch.int32).to(DEV)
        d = torch.randint(1, V, (32, 4, 64), generator=g, dtype=torch.int32).to(DEV)
    grads = []
    for enabled in (False, True):
        monkeypatch.setattr(grad_sink, "ENABLED", enabled)
        torch.manual_seed(0)
        tr = Trainer(cfg, build_model(cfg, V), torch.device(DEV))
        tr.train_step(q, d)
        torch.cuda.synchronize()
        grads.append((tr.flat.grad.clone(), len(tr.flat.written)))
    (ga, _), (gb, n_written) = grads
    assert n_written == len(tr.flat.named)
    assert float(ga.abs().sum()) > 0
    err = float((ga - gb).abs().max() / ga.abs().max())
    assert err < 1e-2, err


def test_direct_grad_weight_used_twice(monkeypatch):
    """A weight reached by two ops in one backward: the first writes the flat gradient, the
    second falls back to autograd's accumulate (grad_sink.write_target's written set)."""
    from dnn_page_vectors_amd.ops import grad_sink
    from dnn_page_vectors_amd.ops.optim import FlatParams

    x1 = bf(torch.randn(256, 96, device=DEV))
    x2 = bf(torch.randn(128, 96, device=DEV))
    res = []
    for enabled in (True, False):
        monkeypatch.setattr(grad_sink, "ENABLED", enabled)
        torch.manual_seed(1)
        lin = torch.nn.Linear(96, 64).to(DEV)
        lin.weight.data = bf(lin.weight.data)
        flat = FlatParams(lin.named_parameters())
        flat.zero_grad()
        y = dops.linear_act(x1, lin.weight, lin.bias, "relu").sum() + dops.linear_act(x2, lin.weight, lin.bias,
                                                                                       "tanh").sum()
        y.backward()
        assert lin.weight.grad.data_ptr() == flat.grad.data_ptr()
        res.append((lin.weight.grad.clone(), lin.bias.grad.clone(), lin.weight.detach().clone(),
                    lin.bias.detach().clone()))
    (gw, gb, w0, b0), (gw2, gb2, _, _) = res
    torch.testing.assert_close(gw, gw2, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(gb, gb2, rtol=1e-5, atol=1e-5)
    wr = w0.requires_grad_(True)
    br = b0.requires_grad_(True)
    (torch.relu(x1 @ wr.t() + br).sum() + torch.tanh(x2 @ wr.t() + br).sum()).backward()
    for got, want in ((gw, wr.grad), (gb, br.grad)):
        err = float((got - want).abs().max() / want.abs().max())
        assert err < 2e-2, err


@pytest.mark.parametrize("torch_style,E", [(False, 96), (True, 96), (False, 20), (False, 60), (True, 300)])
def test_lazy_embedding_adam_matches_cpu(torch_style, E):
    """FlatAdam(lazy=[table]): untouched embedding rows keep weights and moments; touched rows
    and every other parameter get the dense update (HIP segmented step vs the CPU path)."""
    from dnn_page_vectors_amd.ops.optim import FlatAdam, FlatParams

    def make(dev):
        torch.manual_seed(0)
        m = torch.nn.ModuleDict({"lin": torch.nn.Linear(33, 17), "tok": torch.nn.Embedding(301, E)})
        return m.to(dev)

    res = []
    for dev in ("cpu", DEV):
        m = make(dev)
        flat = FlatParams(m.named_parameters())
        opt = FlatAdam(flat, lr=1e-2, torch_style=torch_style, lazy=["tok.weight"])
        assert opt.lazy
        g = torch.Generator().manual_seed(1)
        for t in range(4):
            gr = torch.randn(flat.numel, generator=g)
            o, k, _ = flat.offsets["tok.weight"]
            tab = gr[o:o + k].view(301, E)
            tab[torch.arange(301) % (t + 2) != 0] = 0.0   # a different row subset each step
            gr[o + k:o + (k + 63) // 64 * 64] = 0.0        # alignment padding carries no gradient
            flat.grad.copy_(gr.to(dev))
            opt.step()
        res.append((flat.data.cpu(), opt.m.cpu(), opt.v.cpu()))
    for a, b in zip(res[0], res[1]):
        torch.testing.assert_close(b, a, rtol=1e-5, atol=1e-6)
    # rows never touched (odd rows with t+2 in {2,3,4,5} all skipping them: rows % 60 == 1) keep init
    o, k, _ = flat.offsets["tok.weight"]
    mv = res[1][1][o:o + k].view(301, E)
    never = [r for r in range(301) if all(r % (t + 2) != 0 for t in range(4))]
    assert never and float(mv[never].abs().max()) == 0.0


@pytest.mark.parametrize("R,shape,dt", [(4096, (512,), torch.float32), (65536, (768,), torch.bfloat16),
                                        (8, (4096, 512), torch.float32), (3, (100,), torch.float32),
                                        (1000, (36,), torch.bfloat16), (16384, (150,), torch.float32),
                                        (777, (3, 50), torch.float32), (65, (30,), torch.bfloat16),
                                        # wide and not 4-aligned: element loads at 16 quads per block
                                        (2, (513, 129), torch.float32), (3, (4099,), torch.bfloat16)])
def test_colsum_modes(R, shape, dt):
    """dense.hip::colsum_kernel (bias gradients, split-K sums) vs the fp32 torch sum:
    overwrite, accumulate into a non-zero buffer, and the scale / bias / activation epilogue."""
    g0 = torch.Generator(device=DEV).manual_seed(0)
    x = torch.randn(R, *shape, device=DEV, generator=g0).to(dt)
    want = x.float().sum(0)
    got = dops.colsum(x)
    torch.testing.assert_close(got, want, rtol=1e-4, atol=1e-3)
    base = torch.randn(*shape, device=DEV, generator=g0)
    acc = base.clone()
    dops.colsum(x, out=acc, accumulate=True)
    torch.testing.assert_close(acc, base + want, rtol=1e-4, atol=1e-3)
    if len(shape) == 2:
        scale = torch.rand(shape[0], device=DEV, generator=g0)
        bias = torch.randn(shape[1], device=DEV, generator=g0)
        y = dops.colsum(x, scale=scale, bias=bias, act="tanh")
        torch.testing.assert_close(y, torch.tanh(want * scale[:, None] + bias), rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("plan,L,act", [("gather", 45, "tanh"), ("counts", 300, "tanh"), ("gather", 20, "relu"),
                                        ("counts", 2000, "relu")])
def test_embedding_bag_fused_bias_act(plan, L, act):
    """act(mean bag + bias) with the bias / activation in the producing kernel (gather
    epilogue, split-K column-sum epilogue): values and W / bias gradients vs fp32 torch."""
    from dnn_page_vectors_amd.ops import embedding as eops

    V, N, E = 30000, 96, 512
    g0 = torch.Generator(device=DEV).manual_seed(3)
    ids = torch.randint(1, V, (N, L), dtype=torch.int32, device=DEV, generator=g0)
    ids[:, L // 3:] *= (torch.rand(N, L - L // 3, device=DEV, generator=g0) < 0.5).int()
    W = bf(torch.randn(V, E, device=DEV, generator=g0)).requires_grad_(True)
    b = (torch.randn(E, device=DEV, generator=g0) * 0.3).requires_grad_(True)
    Wr = W.detach().clone().requires_grad_(True)
    br = b.detach().clone().requires_grad_(True)
    y = eops.embedding_bag(ids, W, pad=0, mean=True, plan=plan, bias=b, act=act)
    cnt = (ids != 0).sum(1, keepdim=True).clamp(min=1).float()
    pre = ref.embedding_bag_sum(ids, Wr, 0) / cnt + br
    yr = torch.tanh(pre) if act == "tanh" else torch.relu(pre)
    torch.testing.assert_close(y, yr, rtol=2e-2, atol=2e-2)
    gy = torch.randn_like(yr)
    (y * gy).sum().backward()
    (yr * gy).sum().backward()
    for got, want in ((W.grad, Wr.grad), (b.grad, br.grad)):
        err = float((got - want).abs().max() / want.abs().max())
        assert err < 2e-2, err


@pytest.mark.parametrize("with_dq", [True, False])
def test_inbatch_loss_reduce_matches_mean(with_dq):
    """inbatch_loss(reduce=True): mean loss / accuracy from the loss_stats kernel and the
    fused backward prologue (ib_grad_scale) equal per-row loss -> torch mean -> backward."""
    B, M, D = 300, 1200, 150
    g0 = torch.Generator(device=DEV).manual_seed(5)
    q0 = torch.nn.functional.normalize(torch.randn(B, D, device=DEV, generator=g0), dim=1)
    d0 = torch.nn.functional.normalize(torch.randn(M, D, device=DEV, generator=g0), dim=1)
    d0[::4][:B] = torch.nn.functional.normalize(q0 + 0.5 * d0[::4][:B], dim=1)
    pos = torch.arange(B, device=DEV, dtype=torch.int32) * 4
    res = []
    for reduce in (False, True):
        q = q0.clone().requires_grad_(with_dq)
        d = d0.clone().requires_grad_(True)
        out = lops.inbatch_loss(q, d, pos, 10.0, True, reduce=reduce)
        if reduce:
            loss, P, acc = out
        else:
            loss, P = out
            loss, acc = loss.mean(), (P > 0.5).float().mean()
        loss.backward()
        res.append((float(loss), float(acc), q.grad, d.grad))
    (l0, a0, gq0, gd0), (l1, a1, gq1, gd1) = res
    assert abs(l0 - l1) < 1e-5 * max(1.0, abs(l0)) and a0 == a1
    torch.testing.assert_close(gd1, gd0, rtol=1e-5, atol=1e-7)
    if with_dq:
        torch.testing.assert_close(gq1, gq0, rtol=1e-5, atol=1e-7)


def test_adam_bf16_mirror_tracks_weights():
    """FlatAdam(mirror=...): the update kernel writes bf16(p) with every step (dense and lazy
    segments); mirror_for() serves it only while it is current."""
    from dnn_page_vectors_amd.models.base import bump_generation
    from dnn_page_vectors_amd.ops.optim import FlatAdam, FlatParams, mirror_for

    torch.manual_seed(0)
    m = torch.nn.ModuleDict({"lin": torch.nn.Linear(33, 17), "tok": torch.nn.Embedding(301, 96),
                             "tok2": torch.nn.Embedding(50, 40)}).to(DEV)
    flat = FlatParams(m.named_parameters())
    opt = FlatAdam(flat, lr=1e-2, lazy=["tok2.weight"], mirror=["tok.weight", "lin.weight", "tok2.weight"])
    for name in ("tok.weight", "lin.weight", "tok2.weight"):
        p = dict(flat.named)[name]
        assert mirror_for(p) is not None
    for _ in range(3):
        flat.grad.copy_(torch.randn_like(flat.grad))
        opt.step()
        bump_generation()
        for name in ("tok.weight", "lin.weight", "tok2.weight"):
            p = dict(flat.named)[name]
            mm = mirror_for(p)
            assert mm is not None and torch.equal(mm, p.detach().to(torch.bfloat16)), name
    bump_generation()  # e.g. a checkpoint load: stale until refreshed
    assert mirror_for(m.tok.weight) is None
    with torch.no_grad():
        m.tok.weight.mul_(0.5)
    opt.refresh_mirrors()
    assert torch.equal(mirror_for(m.tok.weight), m.tok.weight.detach().to(torch.bfloat16))


@pytest.mark.parametrize("preset", ["mlp", "bert"])
def test_bf16_mirror_training_matches_cast(preset):
    """Same trajectory with the optimizer-written bf16 weights as with per-step casts."""
    from dnn_page_vectors_amd.config import Configuration, preset_config
    from dnn_page_vectors_amd.data.synthetic import SyntheticPairs, spec_from_config
    from dnn_page_vectors_amd.models import build_model
    from dnn_page_vectors_amd.parallel import dist as pdist
    from dnn_page_vectors_amd.train.trainer import Trainer

    pdist.set_info(pdist.DistInfo(device=torch.device(DEV)))
    if preset == "bert":
        cfg = preset_config("bert_dp8").replace(bert_layers=2, batch_size=16, document_length=64, query_length=16,
                                                bert_dropout=0.0)
    else:
        cfg = Configuration(model="mlp", feature_level="ngram", vocab_hash_size=500, query_length=12,
                            document_length=64, batch_size=32, embedding_dim=64, loss_mode="in_batch",
                            mlp_dims=(64, 64, 32))
    data = SyntheticPairs(spec_from_config(cfg, cfg.vocab_hash_size, num_pages=512), DEV, seed=5)
    pool = [data.batch(cfg.batch_size) for _ in range(4)]
    runs = []
    for mirror in (False, True):
        torch.manual_seed(0)
        tr = Trainer(cfg.replace(optimizer_bf16_mirror=mirror), build_model(cfg, cfg.vocab_hash_size),
                     torch.device(DEV))
        assert bool(tr.opt.mirrors) == mirror
        runs.append([float(tr.train_step(*pool[i % 4])["loss"]) for i in range(5)])
    for a, b in zip(*runs):
        assert abs(a - b) <= 1e-3 * max(1.0, abs(a)), runs


@pytest.mark.parametrize("V,L", [(30000, 2000), (1001, 300), (38000, 64)])
def test_bag_counts_matrix_exact(V, L):
    """LDS-histogram count matrix (16-bit packed counters below V 40960, u32 otherwise) vs a
    bincount reference: every entry, pads excluded, odd / even neighbours and repeats."""
    from dnn_page_vectors_amd.ops import embedding as eops

    N = 37
    g0 = torch.Generator(device=DEV).manual_seed(9)
    ids = torch.randint(1, V, (N, L), dtype=torch.int32, device=DEV, generator=g0)
    ids[:, ::7] = 5           # a repeated token (count L/7 <= 286)
    ids[:, 1::11] = 6         # its odd neighbour
    ids[:, L // 2:] *= (torch.rand(N, L - L // 2, device=DEV, generator=g0) < 0.5).int()  # pads
    C, lens = eops._counts(ids, V, 0)
    ref_c = torch.zeros(N, V, device=DEV)
    ref_c.scatter_add_(1, ids.long(), torch.ones(N, L, device=DEV))
    ref_c[:, 0] = 0
    got = C[:, :V].float()
    torch.testing.assert_close(got, ref_c.bfloat16().float(), rtol=0, atol=0)
    torch.testing.assert_close(lens, (ids != 0).sum(1).float(), rtol=0, atol=0)


def test_bert_residual_link_matches_autograd_sum(monkeypatch):
    """ops/transformer.py::ResidualLink: the residual gradient added in the linear layer's dX
    GEMM equals autograd's separate sum (2-layer BERT, every parameter and the input)."""
    from dnn_page_vectors_amd.models.bert_dual import BertEncoder
    from dnn_page_vectors_amd.ops import transformer as tops

    g = torch.Generator().manual_seed(0)
    ids = torch.randint(1, 500, (6, 40), generator=g).to(DEV)
    ids[:, 30:] = 0
    grads = []
    for fuse in (False, True):
        monkeypatch.setattr(tops, "RESID_FUSE", fuse)
        enc = BertEncoder(500, 256, 512, 4, 2, 64, 32, torch.Generator().manual_seed(1)).to(DEV)
        out = enc(ids, 0.0, True)
        (out.float() * torch.linspace(-1, 1, out.numel(), device=DEV).view_as(out)).sum().backward()
        grads.append({n: p.grad.detach().clone() for n, p in enc.named_parameters() if p.grad is not None})
    assert grads[0].keys() == grads[1].keys() and len(grads[0]) > 10
    for n in grads[0]:
        a, b = grads[0][n].float(), grads[1][n].float()
        err = float((a - b).abs().max() / a.abs().max().clamp_min(1e-12))
        assert err < 3e-2, (n, err)


def test_conv_weight_rows_kernel_matches_torch_layout():
    """pv_conv_weight_rows (one launch) == the zero-filled [2F][4][EP] bf16 layout built with
    torch ops (the backward's dTable operand)."""
    torch.manual_seed(3)
    F, E = 150, 100
    w3 = torch.randn(F, 3, E, device=DEV)
    w4 = torch.randn(F, 4, E, device=DEV)
    got = cops._weight_rows(w3, w4, cops.EP)
    ref_rows = torch.zeros(2 * F, 4, cops.EP, dtype=torch.bfloat16, device=DEV)
    ref_rows[:F, :3, :E] = w3
    ref_rows[F:, :, :E] = w4
    assert torch.equal(got, ref_rows)


@pytest.mark.parametrize("CL", [512, 7])
def test_chunk_mean_pool_matches_torch(CL):
    """chunkpool.hip masked mean over non-empty chunks (fwd + bwd) == the torch expression,
    with empty chunks and a page whose chunks are all padding."""
    torch.manual_seed(5)
    N, C, D = 6, 8, 128
    ids = torch.randint(1, 1000, (N, C * CL), dtype=torch.int32, device=DEV)
    ids.view(N, C, CL)[1, 3] = 0          # one empty chunk
    ids.view(N, C, CL)[2, 5:] = 0         # trailing empty chunks
    ids[4] = 0                            # an all-padding page -> zeros
    ids.view(N, C, CL)[0, 2, :-1] = 0     # one non-pad id keeps a chunk alive
    v = torch.randn(N, C, D, device=DEV, requires_grad=True)
    out = dops.chunk_mean_pool(v, ids, CL)
    live = (ids.view(N, C, CL) != 0).any(dim=2).unsqueeze(2).float()
    v2 = v.detach().clone().requires_grad_(True)
    ref_out = (v2 * live).sum(1) / live.sum(1).clamp(min=1.0)
    torch.testing.assert_close(out, ref_out, rtol=1e-5, atol=1e-6)
    g = torch.randn(N, D, device=DEV)
    (out * g).sum().backward()
    (ref_out * g).sum().backward()
    torch.testing.assert_close(v.grad, v2.grad, rtol=1e-5, atol=1e-6)
    assert torch.all(out[4] == 0)


def test_colsum_bag_mean_length_epilogue():
    """colsum mode 3 (scale_is_len): act(sum / max(len, 1) + bias) -- the split-K bag-mean
    epilogue of the counts GEMM, with zero-length bags."""
    torch.manual_seed(6)
    S, N, E = 8, 37, 512
    x = torch.randn(S, N, E, device=DEV)
    lens = torch.randint(0, 50, (N,), device=DEV).float()
    lens[3] = 0.0
    bias = torch.randn(E, device=DEV)
    y = dops.colsum(x, scale=lens, bias=bias, act="tanh", scale_is_len=True)
    ref_y = torch.tanh(x.sum(0) / lens.clamp(min=1.0)[:, None] + bias)
    torch.testing.assert_close(y, ref_y, rtol=1e-5, atol=1e-5)


def test_cdssm_training_curve_hip_matches_torch():
    """Training-curve parity: CDSSM (B 512, pages 256 tokens, cross-GPU loss on one rank)
    trained 300 steps from the same initial weights on the same batches with the same
    dropout masks, once through the HIP kernels (bf16 MFMA, sparse argmax backward, counting
    sort, fused Adam) and once through eager fp32 PyTorch ops.  Loss curves and the final
    Recall@10 must agree within run-to-run noise: the HIP backward learns exactly what the
    framework-reference model learns (the CDSSM-vs-MLP quality gap is the model, not the
    kernels)."""
    import copy

    from dnn_page_vectors_amd.config import preset_config
    from dnn_page_vectors_amd.data.synthetic import SyntheticPairs, spec_from_config
    from dnn_page_vectors_amd.eval.retrieval import recall_at_k
    from dnn_page_vectors_amd.models import build_model
    from dnn_page_vectors_amd.parallel import dist as pdist
    from dnn_page_vectors_amd.train.trainer import Trainer

    pdist.set_info(pdist.DistInfo(device=torch.device(DEV)))
    base = preset_config("cdssm_ngram_bf16").replace(batch_size=512, document_length=256)
    V = base.vocab_hash_size
    torch.manual_seed(21)
    m0 = build_model(base, V)
    out = {}
    # the fp32 arm's F.conv1d through PyTorch's native (unfold + GEMM) convolution: MIOpen
    # would search / compile kernels for every new shape on a fresh box first
    cudnn_prev = torch.backends.cudnn.enabled
    torch.backends.cudnn.enabled = False
    try:
        for dtype in ("bf16", "fp32"):
            cfg = base.replace(dtype=dtype)
            model = copy.deepcopy(m0)
            model.cfg = cfg
            tr = Trainer(cfg, model, torch.device(DEV))
            data = SyntheticPairs(spec_from_config(cfg, V, num_pages=8192), DEV, seed=77)
            losses = []
            for i in range(300):
                losses.append(float(tr.train_step(*data.batch(cfg.batch_size))["loss"]))
                if i % 50 == 0:
                    print(f"{dtype} step {i} loss {losses[-1]:.4f}", flush=True)
            qe, pe = data.eval_set(1024)
            r = recall_at_k(model.encode(qe, "query"), model.encode(pe, "doc"), torch.arange(1024, device=DEV),
                            k=10)
            out[dtype] = (losses, r)
    finally:
        torch.backends.cudnn.enabled = cudnn_prev
    (lh, rh), (lt, rt) = out["bf16"], out["fp32"]
    tail_h, tail_t = sum(lh[-50:]) / 50, sum(lt[-50:]) / 50
    print(f"HIP bf16: loss {lh[0]:.3f} -> {tail_h:.3f}, R@10 {rh:.3f} | torch fp32: loss {lt[0]:.3f} -> "
          f"{tail_t:.3f}, R@10 {rt:.3f}")
    assert abs(lh[0] - lt[0]) < 0.02 * lt[0]
    assert tail_h < 0.9 * lh[0] and tail_t < 0.9 * lt[0]  # both learn
    assert abs(tail_h - tail_t) < 0.05 * tail_t, (tail_h, tail_t)
    assert abs(rh - rt) < 0.05, (rh, rt)


def _curve_parity(preset, overrides, steps, num_pages=4096, eval_pairs=1024, seed=21):
    """Train the same initial model on the same batches (same dropout seeds) through the HIP
    kernels (bf16) and through eager fp32 PyTorch ops; -> {dtype: (losses, Recall@10)}."""
    import copy

    from dnn_page_vectors_amd.config import preset_config
    from dnn_page_vectors_amd.data.synthetic import SyntheticPairs, spec_from_config
    from dnn_page_vectors_amd.eval.retrieval import recall_at_k
    from dnn_page_vectors_amd.models import build_model
    from dnn_page_vectors_amd.parallel import dist as pdist
    from dnn_page_vectors_amd.train.trainer import Trainer

    pdist.set_info(pdist.DistInfo(device=torch.device(DEV)))
    base = preset_config(preset).replace(**overrides)
    V = base.vocab_hash_size
    torch.manual_seed(seed)
    m0 = build_model(base, V)
    out = {}
    cudnn_prev = torch.backends.cudnn.enabled
    torch.backends.cudnn.enabled = False  # fp32 arm: no MIOpen kernel search on a fresh box
    try:
        for dtype in ("bf16", "fp32"):
            cfg = base.replace(dtype=dtype)
            model = copy.deepcopy(m0)
            model.cfg = cfg
            tr = Trainer(cfg, model, torch.device(DEV))
            data = SyntheticPairs(spec_from_config(cfg, V, num_pages=num_pages), DEV, seed=77)
            losses = [float(tr.train_step(*data.batch(cfg.batch_size))["loss"]) for _ in range(steps)]
            qe, pe = data.eval_set(eval_pairs)
            with torch.no_grad():
                r = recall_at_k(model.encode(qe, "query"), model.encode(pe, "doc"),
                                torch.arange(eval_pairs, device=DEV), k=10)
            out[dtype] = (losses, r)
    finally:
        torch.backends.cudnn.enabled = cudnn_prev
    return out


@pytest.mark.parametrize("preset,overrides,steps,learn,pages", [
    # lr 1e-3 (the preset's 3e-3 is tuned for the 500-step recall protocol): at 3e-3 the bf16 and
    # fp32 trajectories drift apart run to run with the float-atomic summation order (tails
    # 0.477 vs 0.430 in one run, within 8% in the next); the kernels' parity is the question here
    ("longpage_cdssm", dict(batch_size=128, num_chunks=4, chunk_len=256, document_length=1024, lr=1e-3), 200, 0.97,
     512),
    ("bert_dp8", dict(bert_layers=2, batch_size=32, document_length=64, query_length=16, lr=3e-4), 200, 0.9, 256),
])
def test_new_config_training_curve_hip_matches_torch(preset, overrides, steps, learn, pages):
    """the fp32-torch parity arm for the chunked-CDSSM (config 5, conv chunk
    encoder) and BERT (config 4) presets, as for the CDSSM headline: the HIP step (bf16 MFMA,
    fused kernels) learns what the fp32 PyTorch implementation of the same model learns, so a
    quality gap between presets is the model / recipe, not the kernels."""
    out = _curve_parity(preset, overrides, steps, num_pages=pages)  # a small page pool: it can be learned
    (lh, rh), (lt, rt) = out["bf16"], out["fp32"]
    k = max(10, steps // 6)
    tail_h, tail_t = sum(lh[-k:]) / k, sum(lt[-k:]) / k
    print(f"{preset} HIP bf16: loss {lh[0]:.3f} -> {tail_h:.3f}, R@10 {rh:.3f} | torch fp32: loss {lt[0]:.3f} -> "
          f"{tail_t:.3f}, R@10 {rt:.3f}")
    assert abs(lh[0] - lt[0]) < 0.02 * lt[0]
    assert tail_h < learn * lh[0] and tail_t < learn * lt[0]  # both learn
    # the tails agree within 8% of each other or within 2% of the starting loss: bf16 and fp32
    # trajectories of a fast-learning preset drift a little apart over 200 steps (chunked CDSSM
    # at ~1/12 of its initial loss: 0.401 vs 0.451 in one run, 0.416 vs 0.409 in another)
    assert abs(tail_h - tail_t) < max(0.08 * tail_t, 0.02 * lt[0]), (tail_h, tail_t)
    assert abs(rh - rt) < 0.08, (rh, rt)


def _mx_k_of(hyp: str, l: int, j: int) -> int:
    """k index of byte j (0..31) of lane l's 32-byte operand under a layout hypothesis."""
    g = l >> 4
    if hyp == "contig32":      # lane group g holds k 32g .. 32g+31
        return 32 * g + j
    if hyp == "halves16":      # k 16g + j (j < 16), 64 + 16g + j - 16
        return 16 * g + j if j < 16 else 64 + 16 * g + (j - 16)
    if hyp == "chunks8":       # four K=32 sub-ops: byte j of chunk c = j // 8 -> k 32c + 8g + j % 8
        return 32 * (j // 8) + 8 * g + (j % 8)
    raise ValueError(hyp)


def test_mx_fp8_mfma_layout():
    """v_mfma_scale_f32_16x16x128_f8f6f4 (e4m3 x e4m3, e8m0 scales): which byte of which lane
    is which k (the MX GEMM's operand packing) and which 32-k block a lane's scale byte
    scales.  Exact check with small-integer e4m3 data against host references of the
    candidate layouts; C in the standard 16x16 layout (row 4 (l >> 4) + r, col l & 15)."""
    from dnn_page_vectors_amd.ops._common import P, check, lib, stream

    g = torch.Generator().manual_seed(0)
    a = torch.randint(-4, 5, (64, 32), generator=g).float()   # lane-major raw operand values
    b = torch.randint(-4, 5, (64, 32), generator=g).float()
    ea = torch.randint(-2, 3, (64,), generator=g)
    eb = torch.randint(-2, 3, (64,), generator=g)

    def run(sa_exp, sb_exp):
        ad = a.to(torch.float8_e4m3fn).view(torch.uint8).to(DEV)
        bd = b.to(torch.float8_e4m3fn).view(torch.uint8).to(DEV)
        sad = (127 + sa_exp).to(torch.int32).to(DEV)
        sbd = (127 + sb_exp).to(torch.int32).to(DEV)
        c = torch.empty(64, 4, device=DEV)
        check(lib().pv_mx_probe(P(ad), P(bd), P(sad), P(sbd), P(c), stream(c.device)), "pv_mx_probe")
        torch.cuda.synchronize()
        got = torch.empty(16, 16)
        cc = c.cpu()
        for l in range(64):
            for r in range(4):
                got[4 * (l >> 4) + r, l & 15] = cc[l, r]
        return got

    def ref(hyp, sa_exp, sb_exp, scale_block):
        A = torch.zeros(16, 128)
        B = torch.zeros(128, 16)
        for l in range(64):
            for j in range(32):
                k = _mx_k_of(hyp, l, j)
                A[l & 15, k] = a[l, j] * 2.0 ** float(sa_exp[scale_block(l, k)])
                B[k, l & 15] = b[l, j] * 2.0 ** float(sb_exp[scale_block(l, k)])
        return A @ B

    zero = torch.zeros(64, dtype=torch.long)
    got1 = run(zero, zero)
    layouts = [h for h in ("contig32", "halves16", "chunks8") if torch.equal(got1, ref(h, zero, zero, lambda l, k: 0))]
    print("MX layouts matching unit-scale data:", layouts)
    assert layouts, "no candidate layout matches"
    got2 = run(ea, eb)
    # candidate scale owners: the lane holding (row l & 15, k-block k // 32)
    def owner(l, k):
        return (l & 15) + 16 * (k // 32)
    scaled = [h for h in layouts if torch.equal(got2, ref(h, ea, eb, owner))]
    print("MX layouts matching per-(row, 32-k block) scales owned by lane row + 16 * block:", scaled)
    assert scaled, (got2, [ref(h, ea, eb, owner) for h in layouts])


@pytest.mark.parametrize("M,N,K,ks", [(256, 128, 128, 1), (300, 136, 1024, 1), (1000, 520, 768, None),
                                      (4096, 512, 30080, None), (64, 1000, 2048, 2)])
def test_gemm_mx8(M, N, K, ks):
    """gemm_mx8.hip (v_mfma_scale_f32_16x16x128_f8f6f4, e4m3 x e4m3, unit block scales):
    C = alpha * (*alpha_ptr) * A8 . B8^T, edge tiles and split-K partials, against fp32 torch
    on the dequantised operands (products exact in fp32; only the summation order differs)."""
    from dnn_page_vectors_amd.ops import fp8 as fops

    g = torch.Generator().manual_seed(M + 3 * N + K)
    A = fops.emulate_e4m3(torch.randn(M, K, generator=g) * 8)
    B = fops.emulate_e4m3(torch.randn(N, K, generator=g) * 8)
    a8 = A.to(torch.float8_e4m3fn).view(torch.uint8).to(DEV)
    b8 = B.to(torch.float8_e4m3fn).view(torch.uint8).to(DEV)
    amax = torch.tensor([3.0], device=DEV)
    from dnn_page_vectors_amd.ops._common import lib

    outs = []
    for ns in (2, 3):  # staging buffers: same MFMA order, bit-identical results
        lib().pv_gemm_mx8_set_stages(ns)
        try:
            outs.append(fops.gemm_mx8(a8, b8, 0.25, amax, ksplit=ks))
        finally:
            lib().pv_gemm_mx8_set_stages(2)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])
    out = outs[1]
    c = out.sum(0) if out.dim() == 3 else out
    want = 0.75 * (A.double() @ B.double().t())
    err = float((c.cpu().double() - want).abs().max() / want.abs().max())
    print(f"mx8 {M}x{N}x{K} ks={ks}: max rel err {err:.2e}")
    assert err < 2e-4, err  # the MFMA's internal sum of a 128-k block is not a plain fp32 chain


def test_quant_fp8_t_and_counts8():
    """The MX bag's operands: W^T in e4m3 (per-tensor 448 / amax, zero K padding) and the
    e4m3 + bf16 count rows of one histogram kernel (exact <= 16, e4m3 rounding above)."""
    from dnn_page_vectors_amd.ops import embedding as eops
    from dnn_page_vectors_amd.ops import fp8 as fops

    g = torch.Generator().manual_seed(1)
    V, E = 1000, 96
    W = torch.randn(V, E, generator=g) * 0.05
    w8, amax = fops.quantize_t(W.to(DEV), 1024)
    torch.cuda.synchronize()
    a = float(W.abs().max())
    assert abs(float(amax) - a) < 1e-7
    want = fops.emulate_e4m3(W.t() * (448.0 / a))
    got = w8.cpu().view(torch.float8_e4m3fn).float()
    assert torch.equal(got[:, :V], want) and not got[:, V:].any()
    ids = torch.randint(1, 40, (16, 700), generator=g, dtype=torch.int32)
    ids[:, :300] = 5          # one token 300 times: e4m3 rounds 300 -> 288
    ids[3] = 0                # an all-padding bag
    C8, C16, lens = eops._counts8(ids.to(DEV), V, 0, True)
    torch.cuda.synchronize()
    C = torch.zeros(16, V)
    C.scatter_add_(1, ids.long(), (ids != 0).float())
    C[:, 0] = 0
    # bf16 counts: exact up to 256 (the 300+ repeats round like torch's bf16 cast)
    assert torch.equal(C16.cpu().float()[:, :V], C.bfloat16().float()) and not C16.cpu()[:, V:].float().any()
    assert torch.equal(C8.cpu().view(torch.float8_e4m3fn).float()[:, :V], fops.emulate_e4m3(C))
    assert torch.equal(lens.cpu(), C.sum(1))


def test_fp8_bag_matches_reference():
    """embedding_bag(fp8=True) on the GPU (e4m3 counts x e4m3 W^T on the MX MFMA + split-K
    column-sum epilogue: mean, bias, tanh) against the CPU reference with the same
    quantisation, forward and weight gradient (e4m3 C^T x e4m3 G, PAGEVEC_FP8_BWD)."""
    from dnn_page_vectors_amd.ops import embedding as eops

    g = torch.Generator().manual_seed(2)
    N, L, V, E = 512, 512, 30000, 512
    # Zipf-like ids: frequent tokens repeat > 16 times per bag (the rounded counts)
    ranks = torch.arange(1, V, dtype=torch.float64)
    p = (1.0 / ranks) / (1.0 / ranks).sum()
    ids = (torch.multinomial(p, N * L, replacement=True, generator=g) + 1).view(N, L).to(torch.int32)
    ids[:, 400:] = 0
    W = (torch.randn(V, E, generator=g) * 0.05).requires_grad_(True)
    b = (torch.randn(E, generator=g) * 0.1).requires_grad_(True)
    out_ref = eops.embedding_bag(ids, W, pad=0, mean=True, bias=b, act="tanh", fp8=True)
    gy = torch.randn(N, E, generator=g)
    (out_ref * gy).sum().backward()
    Wd = W.detach().to(DEV).requires_grad_(True)
    bd = b.detach().to(DEV).requires_grad_(True)
    out = eops.embedding_bag(ids.to(DEV), Wd, pad=0, mean=True, bias=bd, act="tanh", fp8=True)
    (out * gy.to(DEV)).sum().backward()
    torch.cuda.synchronize()
    err = float((out.detach().cpu() - out_ref.detach()).abs().max())
    assert err < 2e-4, err
    exact = eops.embedding_bag(ids, W.detach(), pad=0, mean=True, bias=b.detach(), act="tanh")
    qerr = float((out.detach().cpu() - exact).abs().max() / exact.abs().max())
    print(f"fp8 bag vs reference-quantised {err:.2e}, vs exact fp32 (quantisation) {qerr:.3f}")
    assert qerr < 0.08
    gw = float((Wd.grad.cpu() - W.grad).abs().max() / W.grad.abs().max())
    # FP8_BWD (opt-in arm): both sides quantise the gradient to e4m3 per tensor — the odd
    # rounding tie differs (fp32 dz computed with / without FMAs); default: the exact C^T G
    # on both sides (bf16 dz on the GPU)
    assert gw < (5e-3 if eops.FP8_BWD else 1e-2), gw
    torch.testing.assert_close(bd.grad.cpu(), b.grad, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("side", [False, True])
def test_conv_pool_backward_dw_stream_placement(side, monkeypatch):
    """dW on the calling stream (default) or on the side stream (PAGEVEC_DW_STREAM=1): the
    same gradients (float-atomic sums: to rounding)."""
    torch.manual_seed(11)
    N, L, V, E, F = 64, 300, 500, 100, 150
    ids = torch.randint(0, V, (N, L), dtype=torch.int32, device=DEV)
    base = [bf(torch.randn(V, E, device=DEV) * 0.5), bf(torch.randn(F, 3, E, device=DEV) * 0.1),
            bf(torch.randn(F, 4, E, device=DEV) * 0.1), torch.randn(F, device=DEV) * 0.1,
            torch.randn(F, device=DEV) * 0.1]
    grads = []
    for s in (False, side):
        monkeypatch.setattr(cops, "DW_SIDE_STREAM", s)
        t, w3, w4, b3, b4 = [x.clone().requires_grad_(True) for x in base]
        y, _ = cops.conv_relu_maxpool_fused(ids, t, [w3, w4], [b3, b4], 0.25, 3, True)
        (y * torch.linspace(-1, 1, y.numel(), device=DEV).view_as(y)).sum().backward()
        torch.cuda.synchronize()
        grads.append([t.grad, w3.grad, w4.grad, b3.grad, b4.grad])
    for u, v in zip(*grads):
        torch.testing.assert_close(u, v, rtol=1e-4, atol=1e-5)


def test_bert_embed_fused_matches_unfused(monkeypatch):
    """transformer.hip::bert_embed_* (the packed front end: one gather + position / type add +
    bf16 cast; word rows by atomics, position / type rows by per-group sums) against the
    per-group torch path of BertEncoder.forward_multi: forward bit-identical, gradients equal up
    to the summation order."""
    from dnn_page_vectors_amd.ops import transformer as tops

    torch.manual_seed(3)
    V, H, Lmax = 500, 64, 40
    word0 = torch.randn(V, H, device=DEV) * 0.1
    pos0 = torch.randn(Lmax, H, device=DEV) * 0.1
    typ0 = torch.randn(2, H, device=DEV) * 0.1
    q = torch.randint(1, V, (7, 12), device=DEV)
    d = torch.randint(0, V, (5, 33), device=DEV)
    d[:, 20:] = 0  # padding tail
    gy = torch.randn(7 * 12 + 5 * 33, H, device=DEV)  # one upstream gradient for both arms
    gy[7 * 12:].view(5, 33, H)[:, 20:] = 0  # padding rows carry no gradient, as in the model
    out = {}
    for fused in (True, False):
        monkeypatch.setattr(tops, "BERT_EMBED", fused)
        word, pos, typ = (t.clone().requires_grad_(True) for t in (word0, pos0, typ0))
        x = tops.bert_embed(word, pos, typ, [q, d])
        if x is None:
            xs = [(word[i.long()] + pos[:i.shape[1]].unsqueeze(0) + typ[0]).to(torch.bfloat16).reshape(-1, H)
                  for i in (q, d)]
            x = torch.cat(xs, 0)
        (x.float() * gy).sum().backward()
        out[fused] = (x, word.grad, pos.grad, typ.grad)
    assert torch.equal(out[True][0], out[False][0])
    for a, b in zip(out[True][1:], out[False][1:]):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("fused_shapes", [False, True])
def test_attention_bias_grad_link(monkeypatch, fused_shapes):
    """attention.hip::pv_attn_bwd2's per-workgroup dQ / dK / dV column sums (BiasGradLink) give
    the qkv bias gradient of the linear feeding the attention: against the colsum of dqkv (the
    unlinked path) — equal up to bf16 rounding of dqkv before the sum; every other gradient
    bit-identical."""
    from dnn_page_vectors_amd.ops import transformer as tops

    torch.manual_seed(5)
    H, Hd = 4, 256
    shapes = [(6, 32), (5, 100)] if fused_shapes else [(3, 77)]
    T = sum(n * l for n, l in shapes)
    x0 = torch.randn(T, Hd, device=DEV)
    w0 = torch.randn(3 * Hd, Hd, device=DEV) * 0.05
    b0 = torch.randn(3 * Hd, device=DEV) * 0.1
    masks = []
    for n, l in shapes:
        m = torch.ones(n, l, dtype=torch.int32, device=DEV)
        m[0, l // 2:] = 0
        masks.append(m)
    gy = torch.randn(T, Hd, device=DEV)
    out = {}
    for linked in (True, False):
        monkeypatch.setattr(tops, "ATTN_BGRAD", linked)
        x, w, b = (t.clone().requires_grad_(True) for t in (x0, w0, b0))
        bl = tops.BiasGradLink()
        qkv = tops.linear(x, w, b, bias_link=bl)
        if fused_shapes:
            a = tops.packed_attention(qkv, masks, shapes, H, bias_link=bl)
        else:
            n, l = shapes[0]
            a = tops.fused_attention(qkv.view(n, l, -1), masks[0], H, bias_link=bl).reshape(T, -1)
        (a.float() * gy).sum().backward()
        assert bl.part is None  # consumed by the linear's backward
        out[linked] = (x.grad, w.grad, b.grad)
    assert torch.equal(out[True][0], out[False][0])
    assert torch.equal(out[True][1], out[False][1])
    ref = out[False][2]
    err = (out[True][2] - ref).abs().max().item()
    assert err <= 1e-2 * ref.abs().max().item() + 1e-4, err


@pytest.mark.parametrize("B,M,clip,D", [(700, 5000, True, 150), (2048, 9000, False, 128), (300, 20000, True, 150),
                                        (513, 4097, True, 150)])
@pytest.mark.parametrize("ver", [7])
def test_inbatch_loss_ib7_matches_ib5(B, M, clip, D, ver):
    """loss.hip::ib7_kernel (next tile's S product beside this tile's epilogue, 4-slot ring,
    peeled partial tile) does ib5's arithmetic in ib5's order: the loss and the query-side gradient (ib5 in generation 5) bit-identical; the
    page-side gradient (ib3 in generation 5, a different summation order) against generation 5
    to fp32 rounding."""
    from dnn_page_vectors_amd.ops._common import lib as _lib

    L_ = _lib()
    old = L_.pv_ib_version()
    torch.manual_seed(11)
    q = torch.randn(B, D, device=DEV)
    dd = torch.randn(M, D, device=DEV)
    dd[:B] = q + 2.0 * dd[:B]
    if clip:
        q, dd = q.abs(), dd.abs()
    qn0 = bf(ref.l2_normalize(q))
    dn0 = bf(ref.l2_normalize(dd))
    pos = torch.arange(B, device=DEV, dtype=torch.int32)
    w = torch.rand(B, device=DEV)
    res = {}
    try:
        for v in (5, ver):
            assert L_.pv_ib_set_version(v) == 0
            qn = qn0.clone().requires_grad_(True)
            dn = dn0.clone().requires_grad_(True)
            loss, P = lops.inbatch_loss(qn, dn, pos, 10.0, clip)
            (loss * w).sum().backward()
            torch.cuda.synchronize()
            res[v] = (loss.detach(), qn.grad, dn.grad)
    finally:
        L_.pv_ib_set_version(old)
    assert torch.equal(res[5][0], res[ver][0])
    assert torch.equal(res[5][1], res[ver][1])
    torch.testing.assert_close(res[ver][2], res[5][2], rtol=1e-4, atol=1e-6)


def test_adam_grid_cap_bit_identical():
    """The dense Adam launch's workgroup cap changes only how the stream is split over
    workgroups: the update is bit-identical."""
    from dnn_page_vectors_amd.ops._common import P, lib, stream

    L_ = lib()
    torch.manual_seed(2)
    n = 1_000_003
    base = [torch.randn(n, device=DEV) * 0.01 for _ in range(4)]
    base[3].abs_()
    outs = []
    try:
        for cap in (4096, 1024, 16384):
            L_.pv_adam_set_grid(cap)
            p, g, m, v = (x.clone() for x in base)
            t = torch.zeros(2, device=DEV)  # {step, warmup steps} (optim.hip warmup_scale reads both)
            for _ in range(3):
                assert L_.pv_adam_dev(P(p), P(g), P(m), P(v), n, P(t), 1e-3, 0.9, 0.999, 1e-7, 0.0, 0, None,
                                      stream(p.device)) == 0
            torch.cuda.synchronize()
            outs.append((p, m, v))
    finally:
        L_.pv_adam_set_grid(16384)  # the default
    for o in outs[1:]:
        for a, b in zip(outs[0], o):
            assert torch.equal(a, b)


def test_loss_generation_default_is_ib7():
    """The loss-kernel generation in effect by default is ib7 (no environment switch)."""
    from dnn_page_vectors_amd.ops._common import lib as _lib

    assert _lib().pv_ib_version() == 7


@pytest.mark.parametrize("L", [45, 50, 20, 4])
@pytest.mark.parametrize("p,mode", [(0.25, "element"), (0.0, "element"), (0.3, "token")])
def test_conv_short_chunk_bit_identical(L, p, mode):
    """conv_pool_fwd.hip: sequences of <= 50 tokens (the query tower) run the v7 kernel with one
    48-row chunk instead of 112 rows — pooled values and argmax windows bit-identical, and the
    training step's gradients (sort keys emitted by the same loader waves) equal up to the
    backward's float-atomic summation order."""
    from dnn_page_vectors_amd.ops._common import lib as _lib

    torch.manual_seed(7)
    V, E, F, N = 700, 100, 150, 300
    ids = torch.randint(1, V, (N, L), dtype=torch.int32, device=DEV)
    table0 = torch.randn(V, E, device=DEV) * 0.3
    w30, w40 = torch.randn(F, 3, E, device=DEV) * 0.1, torch.randn(F, 4, E, device=DEV) * 0.1
    b0 = [torch.randn(F, device=DEV) * 0.1, torch.randn(F, device=DEV) * 0.1]
    gy = torch.randn(N, 2 * F, device=DEV)
    lib = _lib()
    outs = []
    try:
        for short in (0, 1):
            lib.pv_conv_set_short(short)
            table, w3, w4 = (t.clone().requires_grad_(True) for t in (table0, w30, w40))
            b = [t.clone().requires_grad_(True) for t in b0]
            pooled, arg = cops.conv_relu_maxpool_fused(ids, table, [w3, w4], b, p, 11, True, mode)
            (pooled * gy).sum().backward()
            torch.cuda.synchronize()
            outs.append((pooled.detach(), arg, table.grad, w3.grad, w4.grad, b[0].grad, b[1].grad))
    finally:
        lib.pv_conv_set_short(1)
    assert torch.equal(outs[0][0], outs[1][0])
    assert torch.equal(outs[0][1], outs[1][1])
    for a, c in zip(outs[0][2:], outs[1][2:]):
        torch.testing.assert_close(a, c, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("B,M,clip,D", [(4096, 16384, True, 150), (700, 5000, False, 128), (300, 1200, True, 150)])
def test_inbatch_fused_glue_matches_unfused(B, M, clip, D, monkeypatch):
    """ops/loss.py FUSED_GLUE: the one-launch forward finish (positive logit, loss / P+, U split
    sum, batch mean loss + accuracy by a last-workgroup ticket) and the backward with the
    positive pair folded into the prologue and the dD split sum equal the round-5 launches
    (ib_pos x 2, ib_rowsum, ib_split_reduce x 2, loss_stats, ib_grad_scale) to fp32 rounding;
    a second call re-uses the re-armed ticket."""
    torch.manual_seed(21)
    q = torch.randn(B, D, device=DEV)
    dd = torch.randn(M, D, device=DEV)
    dd[::4][:B] = q + 2.0 * dd[::4][:B]
    if clip:
        q, dd = q.abs(), dd.abs()
    qn0 = bf(ref.l2_normalize(q))
    dn0 = bf(ref.l2_normalize(dd))
    pos = torch.arange(B, device=DEV, dtype=torch.int32) * 4
    res = {}
    for fused in (False, True, True):
        monkeypatch.setattr(lops, "FUSED_GLUE", fused)
        qn = qn0.clone().requires_grad_(True)
        dn = dn0.clone().requires_grad_(True)
        lm, P, acc = lops.inbatch_loss(qn, dn, pos, 10.0, clip, reduce=True)
        lm.backward()
        torch.cuda.synchronize()
        res.setdefault(fused, []).append((float(lm), float(acc), P.detach(), qn.grad, dn.grad))
    base = res[False][0]
    for got in res[True]:
        assert abs(got[0] - base[0]) <= 1e-5 * abs(base[0]) and got[1] == base[1]
        torch.testing.assert_close(got[2], base[2], rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(got[3], base[3], rtol=1e-4, atol=1e-6)
        torch.testing.assert_close(got[4], base[4], rtol=1e-4, atol=1e-6)
    assert res[True][0][0] == res[True][1][0]  # deterministic finish, ticket re-armed
