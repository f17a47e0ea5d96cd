#!/usr/bin/env python3
"""Headline benchmark: CDSSM-300d training throughput (pairs/sec, whole job) + Recall@10.

Config (BASELINE.json config 2): CDSSM with 2 x 150 conv filters
(k = 3, 4 -> 300-d pooled) -> Dense 150, 30k hashed letter-trigram ids, query 45 /
page 2000 tokens (reference ngram lengths, dssm_cnn_v2/config.py:88-91), J = 3 explicit
negatives per query (reference), bf16 MFMA compute with fp32 master weights, per-GPU
batch 4096 (weak scaling), cross-GPU in-batch negatives: every query is scored against
ALL W * 4096 * (1 + J) page vectors of the step (all-gathered over RCCL).  Synthetic
data: a device-resident pool of pre-featurized batches (no dataset/network available),
random-init weights.  Each timed step = forward + backward + gradient all-reduce +
Adam update.  After the timed steps the run continues UNTIMED on fresh synthetic batches
up to --quality-steps optimizer steps (default 1000 for cdssm / mlp) and reports Recall@10
of that trained model on held-out query/page pairs (`recall_at_10`, `recall_after_steps`).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...     (one rank per GPU, RCCL)

Launch: with ``--gpus N > 1`` and no torchrun environment (``WORLD_SIZE`` unset) this
process never touches the GPU: it spawns N fresh rank processes of itself through
``dnn_page_vectors_amd.launch`` (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 /
a free MASTER_PORT, ``HSA_ENABLE_IPC_MODE_LEGACY=0`` for RCCL's dmabuf IPC), waits for them
and exits with the first non-zero rank status.  Under torchrun the ranks come from the
environment.  Either way every rank checks ``world_size == --gpus`` and, on GPUs, that the
process group runs on RCCL (``backend == "nccl"``; ``PAGEVEC_DIST_BACKEND=gloo`` is the
explicit one-GPU rehearsal override), and rank 0 reports ``n_gpus`` = the world size.

``--dry-run``: the same launch / process-group / timing / JSON path on the CPU (gloo,
eager PyTorch ops, a tiny config-1-sized model) — the CPU test of the multi-rank launch.

Rank 0 prints ONE JSON line (driver contract).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

# RCCL on this driver needs dmabuf IPC: set before anything can initialise HIP
os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
# Multi-rank: the step uses four streams (page tower, query tower, one side stream each) and
# RCCL adds its own; with HIP's default 4 hardware queues two of them would share a queue, and
# a side-stream kernel queued behind a collective waits for the other ranks.  8 queues keep
# them apart (neutral at one rank: 6.94-6.96 vs 6.93-6.94 ms, profiles/r4_prune/hwq_ab.txt).
# A node that exports the default 4 explicitly gets 8 as well; the value in effect is recorded
# in the JSON (runtime_knobs).
if int(os.environ.get("WORLD_SIZE", "1")) > 1 and int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4) < 8:
    os.environ["GPU_MAX_HW_QUEUES"] = "8"

import torch  # noqa: E402


# fp32 gradient megabytes per model (parallel/topology.py picks the RCCL message
# class from it before the process group exists)
GRAD_MB = {"cdssm": 12.6, "mlp": 126.0, "bert": 440.0, "chunked": 126.0, "chunked_cdssm": 12.6, "cdssm_char": 0.5}

MODEL_DESC = {
    "cdssm": "CDSSM-300d (conv 2x150, k=3,4 -> dense 150), 30k hashed tri-grams, Lq=45, Ld=2000, J=3",
    "mlp": "Two-tower MLP 512-512-128, 30k hashed tri-grams, Lq=45, Ld=2000, in-batch/cross-GPU negatives",
    "bert": "BERT-base dual encoder (12L/768H/12A, shared), Lq=32, Ld=256, cross-GPU negatives",
    "cdssm_char": "CDSSM-300d (conv 2x150, k=3,4 -> dense 150), char level (reference run config), ~100-symbol "
                  "vocab, Lq=250, Ld=5000, J=3; bf16 HIP kernels instead of the reference's fp32 (precision "
                  "override)",
    "chunked": "Long-page chunked encoder, 4096 tokens = 8x512 chunks, MLP 512-512-128 fp8 e4m3, mean-pool",
    "chunked_cdssm": "Long-page chunked encoder, 4096 tokens = 8x512 chunks, CDSSM conv tower per chunk (fused "
                     "conv kernel), mean-pool",
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--set", action="append", default=[], metavar="KEY=VALUE",
                    help="Configuration overrides for A/B runs (recorded in the JSON config)")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=4096, help="per-GPU batch (queries)")
    ap.add_argument("--loss", default=None, choices=["cross_gpu", "explicit", "in_batch"],
                    help="default: cross_gpu (cdssm headline); explicit J=3 for cdssm_char (reference head)")
    ap.add_argument("--backend", default="hip", choices=["hip", "torch"],
                    help="torch = eager PyTorch-ROCm implementation of the same model (baseline stand-in)")
    ap.add_argument("--recall", type=int, default=2048, help="held-out pairs for Recall@10 (0 = skip)")
    ap.add_argument("--pool", type=int, default=-1,
                    help="pre-featurized batches kept in HBM for the timed steps; -1 = auto: 4, BERT one per "
                         "timed / warmup step up to 32 (the 110 M-parameter towers memorise a 4-batch pool "
                         "repeated over 25 steps: Recall@10 0.27-0.34 after 200 steps vs 0.41-0.42 without "
                         "the repeats, profiles/r5_bq3/)")
    ap.add_argument("--eager-compare", type=int, default=1,
                    help="also time the eager PyTorch-ROCm implementation of the same model (batch 512, "
                         "single GPU only) and report the speedup")
    ap.add_argument("--graph", type=int, default=-1,
                    help="capture the training step in a hipGraph after 2 eager steps (single process only); "
                         "-1 = auto: on for the mlp / chunked / chunked_cdssm / bert steps, off for cdssm (its "
                         "graph serialises the side streams: eager 6.74-6.82 vs graph 7.24 ms)")
    ap.add_argument("--quality-steps", type=int, default=-1,
                    help="after the timed steps, keep training (untimed, fresh synthetic batches, eager) until "
                         "this many optimizer steps in total, then measure Recall@10 on held-out pairs; "
                         "-1 = auto (1000 for cdssm / mlp, 500 for chunked / cdssm_char, 200 for bert)")
    ap.add_argument("--deterministic", type=int, default=0,
                    help="deterministic reduction mode (ops/determinism.py): order-free fixed-point "
                         "gradient sums, one stream, no hipGraph")
    ap.add_argument("--dry-run", action="store_true",
                    help="CPU rehearsal of the launch / process group / JSON path (gloo, eager ops, tiny model)")
    ap.add_argument("--dtype", default=None, choices=["bf16", "fp32"],
                    help="compute precision (default: the preset's; bf16 for cdssm_char). fp32 = the "
                         "reference's precision: fp32-MFMA conv kernels (conv_pool_f32.hip), fp32 PyTorch ops elsewhere")
    ap.add_argument("--model", default="cdssm", choices=["cdssm", "mlp", "bert", "chunked", "chunked_cdssm",
                                                         "cdssm_char"],
                    help="cdssm = headline (config 2); mlp = config 3; bert = config 4; chunked = config 5; "
                         "cdssm_char = the reference's default run (char level, 250 / 5000 tokens), per-GPU "
                         "batch --batch (default 1024 here)")
    return ap.parse_args()


def _eager_pairs_per_s(cfg, V, dev, batch=512, steps=3, warmup=2):
    """Same model/loss/optimizer through plain PyTorch-ROCm ops (F.embedding, F.conv1d via
    MIOpen, autograd, torch matmul) — BASELINE.md's stand-in for the reference, which
    cannot run here (Python 2 + Keras 1 + Theano)."""
    try:
        from dnn_page_vectors_amd.data.synthetic import SyntheticPairs, spec_from_config
        from dnn_page_vectors_amd.models import build_model
        from dnn_page_vectors_amd.ops._common import get_backend, set_backend
        from dnn_page_vectors_amd.train.trainer import Trainer

        prev = get_backend()
        set_backend("torch")
        try:
            c = cfg.replace(batch_size=batch)
            tr = Trainer(c, build_model(c, V), dev)
            gen = SyntheticPairs(spec_from_config(c, V, num_pages=2048), dev, seed=7)
            b = gen.batch(batch)
            for _ in range(warmup):
                tr.train_step(*b)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(steps):
                tr.train_step(*b)
            torch.cuda.synchronize()
            return batch * steps / (time.perf_counter() - t0)
        finally:
            set_backend(prev)
            torch.cuda.empty_cache()
    except Exception as e:  # the comparison is informational only
        print(f"eager comparison skipped: {e}", file=sys.stderr)
        return None


def _sync(dev) -> None:
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


def _spawn_ranks(a) -> int:
    """--gpus N > 1 without a torchrun environment: N fresh rank processes of this script
    (this process has not initialised HIP and never will)."""
    from dnn_page_vectors_amd.launch import launch

    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    return launch([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], a.gpus, env=env)


def _rank_stats(trainer, marks, local_dt, steps, dev, pdist):
    """Per-rank step-time spread and exposed communication, gathered to every rank: the numbers
    that tell stragglers, RCCL and compute apart when a multi-GPU run scales poorly.

    step_ms: GPU time from a step's first to its last enqueued work (CUDA events; host clock on
    the CPU); exposed_allreduce_ms: GPU time the step's stream spends after its backward waiting
    for the bucketed gradient all-reduces to land (0 at one rank, None when not measured)."""
    import statistics

    ev = trainer.step_events
    trainer.step_events = None
    if ev:
        step_ms = [e0.elapsed_time(e3) for e0, _, _, e3 in ev]
        comm = [e1.elapsed_time(e2) for _, e1, e2, _ in ev if e1 is not None]
    else:
        step_ms = [1e3 * (b - a_) for a_, b in zip(marks[:-1], marks[1:])]
        comm = []
    med_comm = statistics.median(comm) if comm else -1.0
    local = [statistics.median(step_ms), min(step_ms), max(step_ms), med_comm, 1e3 * local_dt / steps]
    g = pdist.gather_floats(local, dev)  # (world, 5)
    col = lambda j: [round(float(x), 3) for x in g[:, j]]  # noqa: E731
    med = col(0)
    out = {
        "step_ms_median_per_rank": med,
        "step_ms_min_per_rank": col(1),
        "step_ms_max_per_rank": col(2),
        "wall_ms_per_step_per_rank": col(4),
        "step_ms_rank_spread": {"min": min(med), "median": round(statistics.median(med), 3), "max": max(med)},
        "exposed_allreduce_ms_median_per_rank": None if float(g[:, 3].min()) < 0 else col(3),
        "step_probe": "cuda events" if ev else "host clock",
    }
    return out


def _lib_stamp(backend):
    """Link stamp of the kernel library this run loaded (and whether it matches the sources)."""
    if backend != "hip":
        return None
    from dnn_page_vectors_amd import _build

    path = os.environ.get("PAGEVEC_HIP_LIB")
    if path:
        return {"path": path, "variant": True}
    return {"stamp": _build.hip_stamp(), "matches_sources": not _build.hip_stale()}


def _rccl_version():
    try:
        v = torch.cuda.nccl.version()
        return ".".join(str(x) for x in v) if isinstance(v, tuple) else str(v)
    except Exception:  # noqa: BLE001 - informational
        return None


def main():
    a = parse()
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(_spawn_ranks(a))
    from dnn_page_vectors_amd.config import preset_config
    from dnn_page_vectors_amd.data.synthetic import SyntheticPairs, spec_from_config
    from dnn_page_vectors_amd.eval.retrieval import distributed_recall_table, recall_at_k
    from dnn_page_vectors_amd.models import build_model
    from dnn_page_vectors_amd.models.cdssm import cdssm_flops_per_sample
    from dnn_page_vectors_amd.ops._common import set_backend
    from dnn_page_vectors_amd.parallel import dist as pdist
    from dnn_page_vectors_amd.train.trainer import Trainer
    from dnn_page_vectors_amd.utils import knobs

    from dnn_page_vectors_amd.parallel import topology

    # xGMI message-class policy (parallel/topology.py): RCCL environment defaults must be in
    # place before the communicator is created (eager device_id init inside init_distributed)
    topology.apply_env(GRAD_MB[a.model], int(os.environ.get("WORLD_SIZE", "1")))
    info = pdist.init_distributed(device="cpu" if a.dry_run else None)
    if info.world_size != a.gpus:
        raise SystemExit(f"bench.py: world size {info.world_size} != --gpus {a.gpus} (launch N ranks with "
                         f"`bench.py --gpus N` or torchrun --nproc-per-node N)")
    if info.world_size > 1 and info.device.type == "cuda" and info.backend != "nccl" \
            and os.environ.get("PAGEVEC_DIST_BACKEND") != info.backend:
        raise SystemExit(f"bench.py: multi-GPU runs use RCCL (backend 'nccl'), got {info.backend!r}")
    if a.dry_run:  # CPU rehearsal: eager PyTorch ops, a tiny model, no quality phase
        a.backend, a.graph, a.eager_compare, a.quality_steps = "torch", 0, 0, 0
        a.recall = min(a.recall, 64)
    if a.backend == "torch":
        set_backend("torch")
    preset = {"cdssm": "cdssm_ngram_bf16", "mlp": "mlp_xgpu", "bert": "bert_dp8", "chunked": "longpage_fp8",
              "chunked_cdssm": "longpage_cdssm", "cdssm_char": "reference_char"}[a.model]
    cfg = preset_config(preset)
    if a.loss is None:
        a.loss = "explicit" if a.model == "cdssm_char" else "cross_gpu"
    if a.model == "cdssm_char":  # reference run config (char, 250 / 5000) on the HIP fast path
        cfg = cfg.replace(dtype=a.dtype or "bf16", vocab_hash_size=100)
        if a.batch == 4096:
            a.batch = 1024
    batch = a.batch if a.model in ("cdssm", "cdssm_char") or a.batch != 4096 else cfg.batch_size
    cfg = cfg.replace(batch_size=batch, loss_mode=a.loss if a.model in ("cdssm", "cdssm_char") else cfg.loss_mode,
                      deterministic=bool(a.deterministic))
    a.batch = batch
    if a.dtype is not None:
        cfg = cfg.replace(dtype=a.dtype)
    if a.set:
        cfg = cfg.override(a.set)
    if a.dry_run:
        a.batch = min(a.batch, 16)
        cfg = cfg.replace(batch_size=a.batch, query_length=12, document_length=32, vocab_hash_size=1000)
    V = cfg.vocab_hash_size
    dev = info.device
    model = build_model(cfg, V)
    # the capture happens after 2 eager steps: only inside the untimed warmup
    if a.graph < 0:
        # cdssm: a graph serialises the query tower / dW side streams (6.74-6.82 eager vs 7.24 ms
        # graph, profiles/r5_graph_ab/); chunked_cdssm's eager step is bimodal (1.08 / 1.41 ms),
        # its graph step steady at 1.13-1.14 ms
        a.graph = 0 if a.model in ("cdssm", "cdssm_char") else 1
    if a.quality_steps < 0:
        a.quality_steps = {"cdssm": 1000, "mlp": 1000, "chunked": 500, "chunked_cdssm": 500, "cdssm_char": 500,
                           "bert": 200}[a.model]
    # pre-built device-resident batches and nothing eager between replays: no per-replay fence
    trainer = Trainer(cfg, model, dev, graph=bool(a.graph) and a.warmup > Trainer.GRAPH_WARMUP, graph_fence=False)

    # 65536 distinct synthetic pages (the quality phase draws fresh batches from them; a
    # smaller pool lets the towers memorise training pages instead of generalising)
    spec = spec_from_config(cfg, V, num_pages=512 if a.dry_run else 65536)
    data = SyntheticPairs(spec, dev, seed=1337 + info.rank)
    if a.pool < 0:
        a.pool = min(32, a.warmup + a.steps) if a.model == "bert" else 4
    pool = [data.batch(a.batch) for _ in range(max(1, a.pool))]
    _sync(dev)

    def step(i):
        q, d = pool[i % len(pool)]
        return trainer.train_step(q, d)

    # the whole loop on the trainer's high-priority stream (Trainer.stream_context): the query
    # tower and side streams keep normal priority, and consecutive steps need no stream hand-off
    sctx = trainer.stream_context()
    sctx.__enter__()
    for i in range(a.warmup):
        m = step(i)
    _sync(dev)
    pdist.barrier()
    _sync(dev)
    # per-step probes: GPU events around every timed step and around the wait for the bucketed
    # gradient all-reduces (the exposed communication of the step); host marks on the CPU
    probe = dev.type == "cuda"
    if probe:
        trainer.step_events = []
    marks = []
    t0 = time.perf_counter()
    for i in range(a.steps):
        marks.append(time.perf_counter())
        m = step(a.warmup + i)
    _sync(dev)
    marks.append(time.perf_counter())
    pdist.barrier()
    _sync(dev)
    dt = time.perf_counter() - t0
    local_dt = dt
    t = torch.tensor([dt], device=dev, dtype=torch.float64)
    pdist.all_reduce_max_(t)
    dt = float(t[0])
    final_loss = float(m["loss"])
    rank_stats = _rank_stats(trainer, marks, local_dt, a.steps, dev, pdist)

    # quality phase (untimed): continue on fresh batches so Recall@10 reflects a trained model
    done = a.warmup + a.steps
    graph_used = trainer._graph is not None
    for i in range(max(0, a.quality_steps - done)):
        m = trainer.train_step(*data.batch(a.batch))
        if info.rank == 0 and (i + 1) % 100 == 0:
            print(f"quality step {done + i + 1}: loss {float(m['loss']):.4f}", file=sys.stderr, flush=True)
    quality_loss = float(m["loss"])
    _sync(dev)
    sctx.__exit__(None, None, None)

    recall = recall_local = None
    if a.recall > 0:
        # every rank encodes its own held-out pairs (rank-specific pages, one shared vocabulary);
        # Recall@10 ranks each query against the pages of ALL ranks (all-gathered page vectors)
        qe, pe = data.eval_set(a.recall, seed=7 + 1000 * info.rank)
        qv = model.encode(qe, "query")
        pv = model.encode(pe, "doc")
        rel = torch.arange(a.recall, device=dev)
        recall_local = recall_at_k(qv, pv, rel, k=10)
        recall = distributed_recall_table(qv, pv, rel, ks=(10,))["recall@10"]

    W = info.world_size
    eager = None
    if a.eager_compare and W == 1 and a.backend == "hip" and a.model == "cdssm":
        eager = _eager_pairs_per_s(cfg, V, dev)

    pairs = a.batch * W * a.steps
    value = pairs / dt
    # forward model FLOPs per pair (the CDSSM backward is sparse — gradients reach only the
    # argmax windows — so a dense "3 x forward" count would overstate the work done)
    if a.model in ("cdssm", "cdssm_char"):
        per_pair = cdssm_flops_per_sample(cfg)
        train_mult = None
    elif a.model == "chunked_cdssm":  # query tower + (1+J) pages x num_chunks conv towers of chunk_len
        C = -(-cfg.document_length // cfg.chunk_len)
        per_pair = cdssm_flops_per_sample(cfg.replace(document_length=cfg.chunk_len, J=(1 + cfg.J) * C - 1))
        train_mult = None
    elif a.model == "bert":
        from dnn_page_vectors_amd.models.bert_dual import bert_flops_per_token
        per_pair = (cfg.query_length * bert_flops_per_token(cfg, cfg.query_length) +
                    (1 + cfg.J) * cfg.document_length * bert_flops_per_token(cfg, cfg.document_length))
        train_mult = 3.0  # dense backward: 2 x forward
    else:  # mlp (config 3) / chunked with the MLP chunk encoder (config 5): towers of bag + dense
        from dnn_page_vectors_amd.models.mlp_dssm import mlp_bag_gemm_flops, mlp_tower_flops

        dims = cfg.mlp_dims
        if a.model == "chunked":
            C = -(-cfg.document_length // cfg.chunk_len)
            page = C * mlp_tower_flops(cfg.chunk_len, dims)
            long_bags = C  # chunk bags through the counts GEMM
        else:
            page = mlp_tower_flops(cfg.document_length, dims)
            long_bags = 1
        per_pair = mlp_tower_flops(cfg.query_length, dims) + (1 + cfg.J) * page
        train_mult = None
        # what the MFMAs execute for the long bags (dense counts row x table, fwd + the C^T G
        # weight gradient), to put the step against the bf16 / fp8 MFMA roofline
        exec_pair = (1 + cfg.J) * long_bags * 2 * mlp_bag_gemm_flops(V, dims[0])
    flops = per_pair * a.batch * W * a.steps / dt
    if info.is_main:
        out = {
            "metric": "pairs/sec (whole node) + Recall@10, DSSM-300d" if a.model == "cdssm"
                      else f"pairs/sec (whole node), {a.model}",
            "value": round(value, 1),
            "unit": "pairs/s",
            "n_gpus": W,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(1000.0 * dt / a.steps, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp32" if cfg.dtype == "fp32" else
                     "fp8_e4m3 MFMA (bf16 elsewhere)" if a.model == "chunked" else "bf16",
            "data": "synthetic (device-resident pre-featurized Zipf trigram-id pages; random-init weights)",
            "config": {"model": MODEL_DESC[a.model] if a.model != "cdssm_char" or cfg.dtype != "fp32" else
                       MODEL_DESC[a.model].split("; bf16")[0] + "; fp32 (reference precision)",
                       "global_batch": a.batch * W, "seq_len": cfg.document_length,
                       "parallelism": f"dp{W}", "loss": a.loss, "backend": a.backend,
                       "softmax_scale": (cfg.inbatch_gamma or cfg.GAMMA) if a.loss != "explicit" else cfg.GAMMA,
                       "deterministic": bool(a.deterministic),
                       "dist_backend": info.backend,
                       "comm": topology.report(topology.grad_mb(model),
                                               trainer.buckets.bucket_mb if trainer.buckets is not None else
                                               topology.bucket_mb(topology.grad_mb(model), cfg.grad_bucket_mb)),
                       "launch": "torchrun-env" if os.environ.get("TORCHELASTIC_RUN_ID") else
                                 ("bench-spawn" if W > 1 else "single"),
                       "rccl_env": {k: v for k, v in sorted(os.environ.items())
                                    if k.startswith(("NCCL_", "RCCL_")) and "SOCKET" not in k},
                       **({"overrides": list(a.set)} if a.set else {})},
            "recall_at_10": None if recall is None else round(recall, 4),
            "recall_candidates": a.recall * W if recall is not None else None,
            "recall_at_10_rank_local": None if recall_local is None else round(recall_local, 4),
            "recall_after_steps": max(done, a.quality_steps),
            "final_loss": round(final_loss, 4),
            "loss_after_quality_steps": round(quality_loss, 4),
            "fwd_model_tflops": round(flops / 1e12, 1),
            "train_model_tflops": round(flops * train_mult / 1e12, 1) if train_mult else None,
            "peak_hbm_gb": round(torch.cuda.max_memory_allocated() / 1e9, 1) if dev.type == "cuda" else None,
            "hip_graph": graph_used,
            "graph_status": trainer.graph_status,
            "per_rank": rank_stats,
            "ranks_seen": W,
            "rccl_version": _rccl_version() if info.backend == "nccl" else None,
            "native_lib_stamp": _lib_stamp(a.backend),
            "runtime_knobs": knobs.in_effect(),
        }
        if a.model in ("mlp", "chunked"):
            out["bag_gemm_executed_tflops"] = round(exec_pair * a.batch * W * a.steps / dt / 1e12, 1)
        if a.dry_run:
            out["dry_run"] = True
            out["data"] = "synthetic (CPU dry run: gloo, eager PyTorch ops, tiny model; not a measurement)"
        if eager:
            out["eager_pytorch_pairs_per_s"] = round(eager, 1)
            out["speedup_vs_eager_pytorch"] = round(value / eager, 1)
        print(json.dumps(out), flush=True)
    pdist.destroy()


if __name__ == "__main__":
    main()
