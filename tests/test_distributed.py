"""Multi-process data parallelism on CPU (gloo, world_size 2 / 4 / 8) — the fake cluster of SURVEY §4.2.

* all_gather_autograd: summed gradients of every rank's loss w.r.t. its local page
  vectors equal the single-process gradient of the summed loss (backward = reduce-scatter).
* DP training (bucketed all-reduce): 2 ranks x B/2 == 1 process x B after 3 steps, for
  the explicit-negative and the cross-GPU in-batch loss.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _env(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))


def _gather_worker(rank, world, port, q):
    _env(rank, world, port)
    from dnn_page_vectors_amd.parallel import dist as pdist

    pdist.init_distributed(device="cpu")
    torch.manual_seed(0)
    X = torch.randn(world * 3, 5)
    local = X[rank * 3:(rank + 1) * 3].clone().requires_grad_(True)
    g = pdist.all_gather_autograd(local)
    w = torch.arange(g.numel(), dtype=torch.float32).view_as(g) * (rank + 1)
    (g * w).sum().backward()
    q.put((rank, local.grad.detach().numpy().copy()))
    pdist.destroy()


@pytest.mark.parametrize("world", [2, 4, 8])
def test_all_gather_autograd_gloo(world):
    port = _port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_gather_worker, args=(r, world, port, q)) for r in range(world)]
    [p.start() for p in ps]
    res = dict(q.get(timeout=120) for _ in ps)
    [p.join(timeout=60) for p in ps]
    base = torch.arange(world * 3 * 5, dtype=torch.float32).view(world * 3, 5)
    full = base * (world * (world + 1) // 2)  # sum over ranks r of d(sum(g*w_r))/dg, w_r = base*(r+1)
    for r in range(world):
        torch.testing.assert_close(torch.from_numpy(res[r]), full[r * 3:(r + 1) * 3])


def _cfg(mode, B):
    from dnn_page_vectors_amd.config import Configuration

    return Configuration(feature_level="ngram", vocab_hash_size=150, query_length=8, document_length=16,
                         batch_size=B, embedding_dim=12, hidden_dims=16, dropout_prob=(0.0, 0.5), loss_mode=mode,
                         grad_bucket_mb=0.05)


def _data(B):
    g = torch.Generator().manual_seed(42)
    out = []
    for _ in range(3):
        q = torch.randint(1, 150, (B, 8), generator=g, dtype=torch.int32)
        d = torch.randint(1, 150, (B, 4, 16), generator=g, dtype=torch.int32)
        out.append((q, d))
    return out


def _dp_worker(rank, world, port, mode, q, B=8):
    _env(rank, world, port)
    from dnn_page_vectors_amd.models.cdssm import CDSSM
    from dnn_page_vectors_amd.parallel import dist as pdist
    from dnn_page_vectors_amd.train.trainer import Trainer

    pdist.init_distributed(device="cpu")
    cfg = _cfg(mode, B // world)
    tr = Trainer(cfg, CDSSM(cfg, 150))
    assert len(tr.buckets.buckets) > 1  # several buckets, launched from grad hooks
    for qa, da in _data(B):
        sl = slice(rank * B // world, (rank + 1) * B // world)
        tr.train_step(qa[sl], da[sl])
    q.put((rank, tr.flat.data.detach().numpy().copy()))
    pdist.destroy()


@pytest.mark.parametrize("mode,world", [("explicit", 2), ("cross_gpu", 2), ("cross_gpu", 4), ("cross_gpu", 8)])
def test_data_parallel_matches_single_process(mode, world):
    from dnn_page_vectors_amd.models.cdssm import CDSSM
    from dnn_page_vectors_amd.parallel import dist as pdist
    from dnn_page_vectors_amd.train.trainer import Trainer

    B = 16 if world == 8 else 8  # two queries per rank at W = 8 (the driver's node size)
    port = _port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_dp_worker, args=(r, world, port, mode, q, B)) for r in range(world)]
    [p.start() for p in ps]
    res = {r: torch.from_numpy(v) for r, v in (q.get(timeout=300) for _ in ps)}
    [p.join(timeout=60) for p in ps]
    # single process reference (cross_gpu with one rank == in-batch over the whole batch)
    pdist.set_info(pdist.DistInfo())
    cfg = _cfg("in_batch" if mode == "cross_gpu" else mode, B)
    tr = Trainer(cfg, CDSSM(cfg, 150))
    for qa, da in _data(B):
        tr.train_step(qa, da)
    for r in range(1, world):
        torch.testing.assert_close(res[0], res[r], rtol=0, atol=0)
    torch.testing.assert_close(res[0], tr.flat.data, rtol=1e-4, atol=3e-5)  # Adam amplifies summation-order noise


def _placement_worker(rank, world, port, q):
    _env(rank, world, port)
    from dnn_page_vectors_amd.models.cdssm import CDSSM
    from dnn_page_vectors_amd.parallel import dist as pdist
    from dnn_page_vectors_amd.train.trainer import Trainer

    pdist.init_distributed(device="cpu")
    cfg = _cfg("explicit", 8).replace(placement="tower")
    tr = Trainer(cfg, CDSSM(cfg, 150))
    losses = []
    for qa, da in _data(8):  # every rank sees the whole batch; the 4 doc slots are split 2 + 2
        losses.append(float(tr.train_step(qa, da)["loss"]))
    q.put((rank, (tr.flat.data.detach().numpy().copy(), losses)))
    pdist.destroy()


def test_tower_placement_matches_single_process():
    """P9 (cnn_dssm_tf.py:139-158): doc slots on different ranks == one process (no dropout)."""
    from dnn_page_vectors_amd.models.cdssm import CDSSM
    from dnn_page_vectors_amd.parallel import dist as pdist
    from dnn_page_vectors_amd.train.trainer import Trainer

    world, port = 2, _port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_placement_worker, args=(r, world, port, q)) for r in range(world)]
    [p.start() for p in ps]
    res = {r: (torch.from_numpy(v[0]), v[1]) for r, v in (q.get(timeout=300) for _ in ps)}
    [p.join(timeout=60) for p in ps]
    pdist.set_info(pdist.DistInfo())
    cfg = _cfg("explicit", 8)
    tr = Trainer(cfg, CDSSM(cfg, 150))
    losses = [float(tr.train_step(qa, da)["loss"]) for qa, da in _data(8)]
    assert res[0][1] == res[1][1]  # identical head on every rank
    for a, b in zip(res[0][1], losses):
        assert abs(a - b) < 1e-5
    torch.testing.assert_close(res[0][0], res[1][0], rtol=0, atol=0)
    torch.testing.assert_close(res[0][0], tr.flat.data, rtol=1e-4, atol=3e-5)


def _tower_sharded_worker(rank, world, port, q):
    _env(rank, world, port)
    from dnn_page_vectors_amd.models.cdssm import CDSSM
    from dnn_page_vectors_amd.parallel import dist as pdist
    from dnn_page_vectors_amd.train.trainer import Trainer

    pdist.init_distributed(device="cpu")
    cfg = _cfg("explicit", 4).replace(placement="tower")
    tr = Trainer(cfg, CDSSM(cfg, 150))
    qa, da = _data(8)[0]
    sl = slice(rank * 4, (rank + 1) * 4)  # a data-parallel shard: different batch per rank
    try:
        tr.train_step(qa[sl], da[sl])
        q.put((rank, "no error"))
    except ValueError as e:
        q.put((rank, str(e)))
    pdist.destroy()


def test_tower_placement_rejects_sharded_batches():
    """tower placement pairs this rank's queries with other ranks' doc slots, so
    sharded (per-rank) batches must be refused instead of training on mismatched pairs."""
    world, port = 2, _port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_tower_sharded_worker, args=(r, world, port, q)) for r in range(world)]
    [p.start() for p in ps]
    res = dict(q.get(timeout=300) for _ in ps)
    [p.join(timeout=60) for p in ps]
    for r in range(world):
        assert "SAME batch" in res[r], res


def test_cli_train_tower_placement_two_ranks(tmp_path):
    """`train --synthetic --set placement=tower` under the launcher (gloo, 2 ranks): the CLI
    must feed every rank the same batch (the trainer's replica check would raise otherwise)
    and both ranks end with identical weights."""
    import json
    import subprocess
    import sys
    import textwrap

    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    script = tmp_path / "w.py"
    script.write_text(textwrap.dedent(f"""
        import os, sys, torch
        from dnn_page_vectors_amd import cli
        rc = cli.main(["train", "--synthetic", "--synthetic-pages", "256",
                       "--set", "experiment_root_directory={tmp_path}", "--set", "feature_level=ngram",
                       "--set", "vocab_hash_size=150", "--set", "query_length=8", "--set", "document_length=16",
                       "--set", "batch_size=8", "--set", "embedding_dim=12", "--set", "hidden_dims=16",
                       "--set", "num_train_samples=32", "--set", "num_validation_samples=8", "--set", "nb_epoch=1",
                       "--set", "placement=tower", "--set", "loss_mode=explicit", "--set", "reuse_experiment_timestamp=True"])
        sys.exit(rc)
    """))
    env = dict(os.environ, PYTHONPATH=repo, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    r = subprocess.run([sys.executable, "-m", "dnn_page_vectors_amd.launch", "--nproc", "2", "--", str(script)],
                       env=env, cwd=str(tmp_path), capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    hist = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])["history"]
    assert len(hist["loss"]) == 1 and hist["loss"][0] == hist["loss"][0]


def _recall_worker(rank, world, port, q):
    _env(rank, world, port)
    from dnn_page_vectors_amd.eval.retrieval import distributed_recall_table
    from dnn_page_vectors_amd.parallel import dist as pdist

    pdist.init_distributed(device="cpu")
    Q, P, n = _recall_data(world)
    sl = slice(rank * n, (rank + 1) * n)
    r = distributed_recall_table(Q[sl], P[sl], torch.arange(n), ks=(1, 5, 10))
    q.put((rank, r))
    pdist.destroy()


def _recall_data(world, n=24, D=8):
    g = torch.Generator().manual_seed(3)
    P = torch.nn.functional.normalize(torch.randn(world * n, D, generator=g), dim=1)
    Q = torch.nn.functional.normalize(P + 0.9 * torch.randn(world * n, D, generator=g), dim=1)
    return Q, P, n


@pytest.mark.parametrize("world", [2, 4])
def test_distributed_recall_matches_single_process(world):
    """W ranks, each with its own queries and pages: Recall@k over the all-gathered pages
    equals the single-process Recall@k on the concatenated collection."""
    from dnn_page_vectors_amd.eval.retrieval import recall_table

    Q, P, n = _recall_data(world)
    want = recall_table(Q, P, torch.arange(world * n), ks=(1, 5, 10))
    assert 0.0 < want["recall@1"] < 1.0  # a non-trivial case
    port = _port()
    ctx = mp.get_context("spawn")
    qq = ctx.Queue()
    ps = [ctx.Process(target=_recall_worker, args=(r, world, port, qq)) for r in range(world)]
    [p.start() for p in ps]
    res = dict(qq.get(timeout=120) for _ in ps)
    [p.join(timeout=60) for p in ps]
    for r in range(world):
        assert res[r] == pytest.approx(want), (r, res[r], want)


def test_buckets_never_mix_towers():
    """A bucket holds one top-level module's parameters only (query tower vs doc towers),
    even when the open bucket is tiny: its all-reduce waits on one tower's streams."""
    from dnn_page_vectors_amd.models.cdssm import CDSSM
    from dnn_page_vectors_amd.ops.optim import FlatParams
    from dnn_page_vectors_amd.parallel.ddp import GradBuckets

    cfg = _cfg("explicit", 4)
    flat = FlatParams(CDSSM(cfg, 150).named_parameters())

    b = GradBuckets.__new__(GradBuckets)  # constructed without a process group (world size 1)
    import dnn_page_vectors_amd.parallel.ddp as ddp
    orig = ddp.dist
    try:
        ddp.dist = type("D", (), {"is_initialized": staticmethod(lambda: False),
                                  "get_world_size": staticmethod(lambda: 1)})
        b.__init__(flat, bucket_mb=64.0)
    finally:
        ddp.dist = orig
    owner = {}
    for name, bi in b.param_bucket.items():
        owner.setdefault(bi, set()).add(name.split(".", 1)[0])
    assert len(b.buckets) >= 2
    assert all(len(mods) == 1 for mods in owner.values()), owner


def _sparse_data(B, V):
    g = torch.Generator().manual_seed(43)
    return [(torch.randint(1, V, (B, 8), generator=g, dtype=torch.int32),
             torch.randint(1, V, (B, 4, 16), generator=g, dtype=torch.int32)) for _ in range(3)]


def _sparse_worker(rank, world, port, q, V, sparse, cap=-1):
    _env(rank, world, port)
    from dnn_page_vectors_amd.models.cdssm import CDSSM
    from dnn_page_vectors_amd.parallel import dist as pdist
    from dnn_page_vectors_amd.train.trainer import Trainer

    pdist.init_distributed(device="cpu")
    B = 8
    cfg = _cfg("cross_gpu", B // world).replace(sparse_embedding_grad=sparse, lazy_embedding_adam=True,
                                                sparse_rows_capacity=cap)
    tr = Trainer(cfg, CDSSM(cfg, V))
    init = tr.flat.data.detach().clone()
    if sparse:
        assert tr.buckets.sparse_bucket  # the tables' buckets are row exchanges
    for qa, da in _sparse_data(B, V):
        sl = slice(rank * B // world, (rank + 1) * B // world)
        tr.train_step(qa[sl], da[sl])
    err = ""
    if sparse:
        try:
            tr.sparse.check()
        except RuntimeError as e:
            err = str(e)
    if err:  # every step overflowed: each was skipped like a non-finite one (no partial update)
        assert torch.equal(tr.flat.data, init), "an overflowing step updated the parameters"
    q.put((rank, tr.flat.data.detach().numpy().copy(), err))
    pdist.destroy()


def _run_sparse(world, V, sparse, cap=-1):
    port = _port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_sparse_worker, args=(r, world, port, q, V, sparse, cap)) for r in range(world)]
    [p.start() for p in ps]
    res = {r: (torch.from_numpy(v), e) for r, v, e in (q.get(timeout=300) for _ in ps)}
    [p.join(timeout=60) for p in ps]
    return res


@pytest.mark.parametrize("world", [2, 4])
def test_sparse_embedding_grad_dp_equals_dense(world):
    """SURVEY §5.8 / VERDICT r3: on a 200k-row vocabulary the touched-row exchange (all-gather
    of ids + rows, LazyAdam over the union rows) gives the same parameters as the dense
    bucket all-reduce with LazyAdam, and as one process with the whole batch."""
    from dnn_page_vectors_amd.models.cdssm import CDSSM
    from dnn_page_vectors_amd.parallel import dist as pdist
    from dnn_page_vectors_amd.train.trainer import Trainer

    V = 200_000
    out = {}
    for sparse in (True, False):
        res = _run_sparse(world, V, sparse)
        for r in range(1, world):
            torch.testing.assert_close(res[0][0], res[r][0], rtol=0, atol=0)
        assert all(not e for _, e in res.values())
        out[sparse] = res[0][0]
    torch.testing.assert_close(out[True], out[False], rtol=1e-5, atol=1e-6)
    pdist.set_info(pdist.DistInfo())
    cfg = _cfg("in_batch", 8).replace(sparse_embedding_grad=True, lazy_embedding_adam=True)
    tr = Trainer(cfg, CDSSM(cfg, V))
    for qa, da in _sparse_data(8, V):
        tr.train_step(qa, da)
    torch.testing.assert_close(out[True], tr.flat.data, rtol=1e-4, atol=3e-5)


def test_sparse_rows_capacity_modes():
    """The exchange's padding (Configuration.sparse_rows_capacity): exact per-step sizing (0,
    host sync) and a fixed capacity with room give the auto mode's parameters; a capacity below
    the distinct-row count drops rows, the step is skipped on the device (parameters unchanged)
    and every rank's check() says so."""
    V, world = 200_000, 2
    auto = _run_sparse(world, V, True, -1)[0][0]
    for cap in (0, 4096):
        res = _run_sparse(world, V, True, cap)
        assert all(not e for _, e in res.values()), cap
        torch.testing.assert_close(res[0][0], auto, rtol=1e-6, atol=1e-7)
    res = _run_sparse(world, V, True, 8)
    assert all("beyond the exchange capacity" in e for _, e in res.values())


def test_unique_rows_fixed_size():
    from dnn_page_vectors_amd.parallel.sparse_rows import unique_rows

    g = torch.Generator().manual_seed(0)
    ids = torch.randint(-3, 60, (500,), generator=g)
    want = torch.unique(ids[(ids >= 0) & (ids < 50)]).to(torch.int32)
    ov = torch.zeros((), dtype=torch.int64)
    got = unique_rows(ids, 50, 64, ov)
    assert got.shape == (64,) and int(ov) == 0
    torch.testing.assert_close(got[:want.numel()], want)
    assert bool((got[want.numel():] == -1).all())
    got = unique_rows(ids, 50, 10, ov)  # capacity below the distinct count: first 10, rest counted
    torch.testing.assert_close(got, want[:10])
    assert int(ov) == want.numel() - 10
    assert unique_rows(ids[:0], 50, 4).tolist() == [-1] * 4


def _agree_worker(rank, world, port, q):
    """Capture agreement (Trainer._capture_agreed): rank 1's capture fails, every rank must fall
    back to eager steps together; pdist.all_agree itself for all-true / one-false inputs."""
    _env(rank, world, port)
    from dnn_page_vectors_amd.config import preset_config
    from dnn_page_vectors_amd.models import build_model
    from dnn_page_vectors_amd.parallel import dist as pdist
    from dnn_page_vectors_amd.train.trainer import Trainer

    pdist.init_distributed(device="cpu")
    res = {"all_true": pdist.all_agree(True), "one_false": pdist.all_agree(rank != world - 1)}
    cfg = preset_config("cdssm_ngram_bf16").replace(batch_size=4, query_length=8, document_length=16,
                                                    vocab_hash_size=200)
    tr = Trainer(cfg, build_model(cfg, cfg.vocab_hash_size), torch.device("cpu"))
    tr.graph_mode = True  # as on a GPU run with graph_distributed=True

    def fake_capture(q_, d_, key):
        if rank == 1:
            raise RuntimeError("capture failed (injected)")
        tr._graph = object()  # rank 0 'captured' its graph

    tr._capture = fake_capture
    ok = tr._capture_agreed(None, None, ("k",))
    res.update(ok=ok, graph_mode=tr.graph_mode, graph=tr._graph is not None, status=tr.graph_status)
    q.put((rank, res))
    pdist.destroy()


@pytest.mark.parametrize("world", [2, 4])
def test_capture_outcome_agreed_across_ranks(world):
    port = _port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_agree_worker, args=(r, world, port, q)) for r in range(world)]
    [p.start() for p in ps]
    res = dict(q.get(timeout=180) for _ in ps)
    [p.join(timeout=60) for p in ps]
    for r in range(world):
        x = res[r]
        assert x["all_true"] is True and x["one_false"] is False
        assert x["ok"] is False and x["graph_mode"] is False and x["graph"] is False, (r, x)
        assert x["status"].startswith("eager (capture failed on"), x["status"]
    assert "injected" in res[1]["status"] and "another rank" in res[0]["status"]
