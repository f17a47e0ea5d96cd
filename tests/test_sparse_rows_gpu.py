"""Row-sparse embedding gradients on the device (parallel/sparse_rows.py + optim.hip::pv_adam_rows)
against the dense table gradient with LazyAdam, through the HIP conv / bag kernels that write the
table gradient (ops/grad_sink.py direct writes included).  ADVICE r4: the micro's old check read
rows 0-3 only."""
import pytest
import torch

from dnn_page_vectors_amd.config import Configuration
from dnn_page_vectors_amd.data.synthetic import SyntheticPairs, spec_from_config
from dnn_page_vectors_amd.models import build_model
from dnn_page_vectors_amd.train.trainer import Trainer

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _cfg(model: str, sparse: bool) -> Configuration:
    common = dict(feature_level="ngram", vocab_hash_size=120_000, batch_size=64, query_length=20,
                  document_length=130, loss_mode="in_batch", lazy_embedding_adam=True,
                  sparse_embedding_grad=sparse, seed=5)
    if model == "mlp":
        return Configuration(model="mlp", embedding_dim=128, mlp_dims=(128, 64, 32), J=0, cos_clip=False,
                             lr=3e-3, **common)
    return Configuration(model="cdssm", **common)


@pytest.mark.parametrize("model", ["cdssm", "mlp"])
def test_sparse_embedding_grad_matches_lazy_dense_gpu(model):
    V = 120_000
    res = {}
    for sparse in (False, True):
        cfg = _cfg(model, sparse)
        m = build_model(cfg, V)
        tr = Trainer(cfg, m, DEV)
        init = tr.flat.data.detach().clone()
        data = SyntheticPairs(spec_from_config(cfg, V, num_pages=512), DEV, seed=11)
        batches = [data.batch(cfg.batch_size) for _ in range(4)]
        for q, d in batches:
            tr.train_step(q, d)
        torch.cuda.synchronize()
        # per tower: the query table sees the query ids only, the page tables the page ids
        touched = {"query": torch.unique(torch.cat([q.reshape(-1) for q, _ in batches]).long()),
                   "doc": torch.unique(torch.cat([d.reshape(-1) for _, d in batches]).long())}
        tabs = {}
        for name, p in tr.flat.named:
            if p.dim() == 2 and name.rsplit(".", 1)[-1] == "embedding":
                o, k, _ = tr.flat.offsets[name]
                tabs[name] = (o, k, p.shape)
        res[sparse] = (tr.flat.data.detach().clone(), init, tabs, touched,
                       tr.flat.grad.detach().clone() if tr.flat.grad is not None else None)
    (dd, di, tabs, touched, _), (sd, si, _, _, sg) = res[False], res[True]
    assert torch.equal(di, si)  # same initial parameters
    assert tabs, "no embedding tables registered"
    # the whole flat buffer (towers AND every table row) agrees with the dense lazy run; the two
    # runs sum the same gradients in different orders (atomics), hence the tolerance
    torch.testing.assert_close(sd, dd, rtol=2e-4, atol=2e-6)
    for name, (o, k, shape) in tabs.items():
        V_, E = shape
        s_tab, i_tab = sd[o:o + k].view(V_, E), si[o:o + k].view(V_, E)
        mask = torch.ones(V_, dtype=torch.bool, device=DEV)
        tt = touched["query" if name.startswith("query") else "doc"]
        mask[tt[tt < V_]] = False
        # rows no batch touched keep their initial weights bit for bit (lazy: no moment decay)
        assert torch.equal(s_tab[mask], i_tab[mask]), name
        # and the touched rows moved
        moved = (s_tab[~mask] != i_tab[~mask]).any(dim=1).float().mean()
        assert moved > 0.5, (name, float(moved))
        # the last step's table gradient lives only in rows that step touched
        if sg is not None:
            g_tab = sg[o:o + k].view(V_, E)
            assert not g_tab[mask].any(), name


def test_no_grad_forward_skips_dtable_key_sort(monkeypatch):
    """the forward key emit / early sort only runs when a backward can follow — not
    for eval / encode batches under torch.no_grad (needs_input_grad alone says requires_grad)."""
    from dnn_page_vectors_amd.ops import conv_pool as cops

    calls = []
    real = cops.sort_pairs_iota
    monkeypatch.setattr(cops, "sort_pairs_iota", lambda *a, **k: (calls.append(1), real(*a, **k))[1])
    cfg = Configuration(feature_level="ngram", vocab_hash_size=30000, batch_size=16, query_length=45,
                        document_length=2000, loss_mode="in_batch")
    m = build_model(cfg, 30000).to(DEV)
    ids = torch.randint(1, 30000, (16, 2000), device=DEV, dtype=torch.int32)
    with torch.no_grad():
        m.encode(ids, "doc")
    torch.cuda.synchronize()
    assert not calls, "key sort ran under no_grad"
    t = m.doc_towers[0]
    pooled, _ = cops.conv_relu_maxpool_fused(ids, t.embedding, list(t.conv_w), list(t.conv_b), 0.25, 1, True)
    pooled.sum().backward()
    torch.cuda.synchronize()
    assert calls, "the training forward no longer sorts its keys early (EARLY_SORT path)"
