"""Command line: ``python -m dnn_page_vectors_amd {setup,w2v,train,encode,eval,serve,bench}``.

The reference has no CLI — each script runs at module level with hard-coded settings
(SURVEY §5.6).  Every subcommand here takes ``--preset``, ``--config file.yaml`` and
``--set key=value`` overrides of the Configuration fields (config.py).
"""
from __future__ import annotations

import argparse
import json
import logging
import os
import sys
from typing import List, Optional

log = logging.getLogger("pagevec")


def _config(a):
    from .config import Configuration, preset_config

    if a.config:
        cfg = Configuration.from_yaml(a.config)
    elif a.preset:
        cfg = preset_config(a.preset)
    else:
        cfg = Configuration()
    if a.set:
        cfg = cfg.override(a.set)
    return cfg


def _common(p):
    p.add_argument("--preset", default=None)
    p.add_argument("--config", default=None)
    p.add_argument("--set", action="append", default=[], metavar="KEY=VALUE")


def cmd_setup(a) -> int:
    from .experiment import SetupExperiment

    cfg = _config(a)
    exp = SetupExperiment(cfg)
    exp.create_workspace()
    if a.input:
        exp.import_dataset(a.input, link=a.link)
    if os.path.exists(cfg.input_dataset):
        nt, nv = exp.split_dataset_file()
        log.info("split: %d train / %d validation rows", nt, nv)
        if cfg.vocab_hash_size <= 1:
            v = exp.build_vocabulary()
            log.info("vocabulary: %d tokens", len(v))
    cfg.save_json(os.path.join(cfg.data_path, "config.json"))
    print(json.dumps({"data_path": cfg.data_path}))
    return 0


def _featurizer(cfg):
    from .data.featurize import Featurizer

    if cfg.vocab_hash_size > 1:
        return Featurizer(cfg.feature_level, hash_size=cfg.vocab_hash_size, html=cfg.html_normalize,
                          nthreads=cfg.num_workers)
    from .io.vocab import load_vocab

    return Featurizer(cfg.feature_level, vocab=load_vocab(cfg), html=cfg.html_normalize, nthreads=cfg.num_workers)


def cmd_train(a) -> int:
    import torch

    from .data.dataset import JsonlPairDataset, PairLoader, SyntheticLoader
    from .data.synthetic import SyntheticPairs, spec_from_config
    from .io import checkpoint as ck
    from .models import build_model
    from .ops._common import set_backend
    from .parallel import dist as pdist
    from .train.trainer import Trainer
    from .utils.metrics import MetricsLogger

    cfg = _config(a)
    from .parallel import topology  # RCCL defaults for the job's message class, before the communicator exists

    world = int(os.environ.get("WORLD_SIZE", "1"))
    gmb = 0.0
    if world > 1:
        # the gradient size of the model this job will train: the real vocabulary (a word-level
        # config's vocab_hash_size is <= 1), parameters on the meta device (no allocation)
        V0 = (cfg.vocab_hash_size if cfg.vocab_hash_size > 1 else 1000) if a.synthetic else _featurizer(cfg).num_ids
        with torch.device("meta"):
            gmb = topology.grad_mb(build_model(cfg, V0))
    topology.apply_env(gmb, world)
    info = pdist.init_distributed()
    if cfg.backend != "auto":
        set_backend(cfg.backend)
    torch.manual_seed(cfg.seed)
    # placement=tower (P9, cnn_dssm_tf.py:139-158) splits the J+1 doc SLOTS of one batch over
    # the ranks and scores every rank's queries against the gathered slots: every rank must
    # see the SAME batch (unsharded loader, rank-independent synthetic seed); data parallel
    # gives each rank its own shard
    replicated = getattr(cfg, "placement", "dp") == "tower"
    d_rank, d_world = (0, 1) if replicated else (info.rank, info.world_size)
    if a.synthetic:
        V = cfg.vocab_hash_size if cfg.vocab_hash_size > 1 else 1000
        gen = SyntheticPairs(spec_from_config(cfg, V, num_pages=a.synthetic_pages), info.device,
                             seed=cfg.seed + d_rank)
        steps = max(1, cfg.num_train_samples // (cfg.batch_size * d_world))
        train_loader = SyntheticLoader(gen, cfg.batch_size, steps)
        val_loader = SyntheticLoader(gen, cfg.batch_size, max(1, cfg.num_validation_samples // cfg.batch_size))
    elif a.validation_split is not None:
        # v1 data path (dssm_cnn/cnn_dssm.py:201): one in-memory file, pad to the dataset max,
        # Keras validation_split (last fraction) + per-epoch shuffle
        from .data.dataset import InMemoryPairs

        fz = _featurizer(cfg)
        V = fz.num_ids
        mem = InMemoryPairs(a.data or cfg.model_training_data, fz, cfg.query_length, cfg.document_length,
                            cfg.num_negative_examples, validation_split=a.validation_split)
        cfg = cfg.replace(query_length=mem.query_length, document_length=mem.document_length)
        train_loader = mem.train_loader(cfg.batch_size, shuffle=True, seed=cfg.seed, device=info.device,
                                        rank=d_rank, world_size=d_world)
        val_loader = mem.val_loader(cfg.batch_size, device=info.device, rank=d_rank, world_size=d_world)
        steps = max(1, train_loader.num_batches())
        log.info("in-memory data: %d train / %d validation rows, padded to %d / %d tokens", mem.n_train,
                 mem.n_val, mem.query_length, mem.document_length)
    else:
        fz = _featurizer(cfg)
        V = fz.num_ids
        tr = JsonlPairDataset(a.data or cfg.model_training_data, fz, cfg.query_length, cfg.document_length,
                              cfg.num_negative_examples)
        va = JsonlPairDataset(cfg.model_validation_data, fz, cfg.query_length, cfg.document_length,
                              cfg.num_negative_examples)
        train_loader = PairLoader(tr, cfg.batch_size, shuffle=a.shuffle, seed=cfg.seed, rank=d_rank,
                                  world_size=d_world, prefetch=cfg.prefetch, device=info.device)
        # validation keeps the last partial batch (Keras evaluates every row; each rank gets the
        # same row count, so the partial batch has one shape on every rank)
        val_loader = PairLoader(va, cfg.batch_size, rank=d_rank, world_size=d_world, device=info.device,
                                drop_last=False)
        steps = min(train_loader.num_batches(), max(1, cfg.num_train_samples // (cfg.batch_size * d_world)))
    model = build_model(cfg, V)
    if cfg.feature_level == "word" and cfg.vocab_hash_size <= 1 and os.path.exists(cfg.word_vectors_file):
        from .io.vectors import cached_word_vectors, init_embedding_
        from .io.vocab import load_vocab

        W = cached_word_vectors(cfg, load_vocab(cfg))
        for t in [model.query_tower, *model.doc_towers]:
            init_embedding_(t.embedding, W)
    metrics = MetricsLogger(os.path.join(cfg.trained_model_dir, "metrics.jsonl"), enabled=info.is_main)
    trainer = Trainer(cfg, model, info.device, metrics)
    if a.resume and ck.resume(trainer, cfg.trained_model_dir):
        log.info("resumed at epoch %d step %d", trainer.epoch, trainer.step)
    hist = trainer.fit(lambda ep: train_loader.epoch_iter(ep), steps_per_epoch=steps,
                       validation_batches=lambda ep: val_loader.epoch_iter(0, fresh=True),
                       callbacks=[ck.ModelCheckpoint(cfg.trained_model_dir)])
    ck.save_final(trainer, cfg.trained_model_dir)
    if info.is_main:
        print(json.dumps({"history": hist, "model_dir": cfg.trained_model_dir}))
    pdist.destroy()
    return 0


def cmd_w2v(a) -> int:
    """Train word vectors on the experiment's text (reference train_word2vec,
    dssm_cnn_v2/w2v.py:8-53) and write them where ``train`` looks for pretrained vectors
    (``word_vectors_file``, word2vec text format); the model itself goes to
    ``vectors/word2vec_models/<name>`` (loaded instead of retrained when present)."""
    from .data.featurize import iter_jsonl_texts
    from .data.text import split_features
    from .models.word2vec import Word2Vec, model_name

    cfg = _config(a)
    files = a.input or [f for f in (cfg.model_training_data, cfg.model_validation_data) if os.path.exists(f)]
    if not files:
        raise SystemExit("no training text: run `setup` first or pass --input")
    path = os.path.join(cfg.vectors_directory, "word2vec_models", model_name(cfg.embedding_dim, a.min_count, a.window))
    if Word2Vec.exists(path) and not a.force:
        model = Word2Vec.load(path)
    else:
        sents = [split_features(t, "word") for fn in files for row in iter_jsonl_texts(fn, cfg.num_negative_examples)
                 for t in row]
        model = Word2Vec(sents, size=cfg.embedding_dim, window=a.window, min_count=a.min_count, sample=1e-3,
                         sg=int(a.sg), iter=a.iter, seed=cfg.seed)
        model.init_sims(replace=True)
        model.save(path)
    os.makedirs(os.path.dirname(cfg.word_vectors_file), exist_ok=True)
    model.save_word2vec_format(cfg.word_vectors_file)
    print(json.dumps({"model": path, "vectors": cfg.word_vectors_file, "words": len(model.index2word),
                      "dim": model.vector_size}))
    return 0


def cmd_encode(a) -> int:
    import numpy as np
    import torch

    from .io import checkpoint as ck
    from .models import build_model

    cfg = _config(a)
    dev = torch.device("cuda" if torch.cuda.device_count() > 0 else "cpu")
    fz = _featurizer(cfg)
    model = build_model(cfg, fz.num_ids).to(dev)
    ck.load_weights(model, a.weights or os.path.join(cfg.trained_model_dir, ck.FINAL_WEIGHTS))
    with open(a.input, encoding="utf-8") as f:
        texts = [l.rstrip("\n") for l in f]
    L = cfg.query_length if a.tower == "query" else cfg.document_length
    ids = torch.from_numpy(fz(texts, L)).to(dev)
    vec = model.encode(ids, a.tower).float().cpu().numpy()
    np.save(a.output, vec)
    print(json.dumps({"vectors": a.output, "shape": list(vec.shape)}))
    return 0


def cmd_eval(a) -> int:
    """Recall@1/10/100.  ``--data FILE`` (or ``--data validation``: the experiment's
    model_validation_data): real {'q', 'doc_corr', 'doc_incorr'} rows, every query ranked
    against all distinct pages of the file; without --data: held-out synthetic pairs.
    Under a multi-rank launch (launch.py / torchrun) the rows are sharded and the page
    vectors all-gathered (eval/retrieval.py::distributed_recall_table)."""
    import torch

    from .eval.retrieval import evaluate_pairs_dataset, recall_table
    from .io import checkpoint as ck
    from .models import build_model
    from .parallel import dist as pdist

    cfg = _config(a)
    info = pdist.init_distributed()
    dev = info.device
    if a.data:
        from .data.dataset import JsonlPairDataset

        path = cfg.model_validation_data if a.data == "validation" else a.data
        fz = _featurizer(cfg)
        model = build_model(cfg, fz.num_ids).to(dev)
        weights = a.weights or os.path.join(cfg.trained_model_dir, ck.FINAL_WEIGHTS)
        if os.path.exists(weights) or a.weights:
            ck.load_weights(model, weights)
        ds = JsonlPairDataset(path, fz, cfg.query_length, cfg.document_length, cfg.num_negative_examples)
        r = evaluate_pairs_dataset(model, ds, dev, max_rows=a.max_rows, include_negatives=not a.no_negatives)
        r.update(data=path, skipped_rows=ds.skipped)
        kind = "jsonl_retrieval"
    else:
        from .data.synthetic import SyntheticPairs, spec_from_config

        V = cfg.vocab_hash_size if cfg.vocab_hash_size > 1 else 1000
        model = build_model(cfg, V).to(dev)
        if a.weights:
            ck.load_weights(model, a.weights)
        gen = SyntheticPairs(spec_from_config(cfg, V, num_pages=1024), dev, seed=cfg.seed)
        q, p = gen.eval_set(a.pages)
        r = recall_table(model.encode(q, "query"), model.encode(p, "doc"), torch.arange(a.pages, device=dev))
        kind = "synthetic_retrieval"
    if info.is_main:
        if a.metrics:
            from .utils.metrics import MetricsLogger

            MetricsLogger(a.metrics).log(eval=kind, pages=a.pages, weights=a.weights, **r)
        print(json.dumps(r))
    pdist.destroy()
    return 0


def cmd_serve(a) -> int:
    """HTTP serving (serve/server.py): encode, index pages, search by query text."""
    import uvicorn

    from .serve.server import build_service, create_app

    from .io.checkpoint import FINAL_WEIGHTS

    cfg = _config(a)
    final = os.path.join(cfg.trained_model_dir, FINAL_WEIGHTS)
    weights = a.weights or (final if os.path.exists(final) else None)
    engine, index = build_service(cfg, weights, max_batch=a.max_batch, max_wait_ms=a.max_wait_ms,
                                  index_path=a.index)
    if a.pages:
        batch_ids, batch_txt = [], []
        with open(a.pages, encoding="utf-8") as f:
            for line in f:
                if not line.strip():
                    continue
                rec = json.loads(line)
                batch_ids.append(rec["id"])
                batch_txt.append(rec["text"])
                if len(batch_txt) == a.max_batch:
                    index.add(engine.encode(batch_txt, "doc"), batch_ids, normalize=False)
                    batch_ids, batch_txt = [], []
        if batch_txt:
            index.add(engine.encode(batch_txt, "doc"), batch_ids, normalize=False)
        log.info("indexed %d pages", len(index))
    if a.save_dir:
        os.makedirs(a.save_dir, exist_ok=True)
    uvicorn.run(create_app(engine, index, save_dir=a.save_dir, max_items=a.max_items), host=a.host, port=a.port, log_level="info")
    engine.close()
    return 0


def main(argv: Optional[List[str]] = None) -> int:
    from .log import setup_logging

    setup_logging()
    ap = argparse.ArgumentParser(prog="dnn_page_vectors_amd")
    sub = ap.add_subparsers(dest="cmd", required=True)
    p = sub.add_parser("setup", help="create the workspace, import + split the dataset, build the vocab")
    _common(p)
    p.add_argument("--input", default=None, help="local JSONL dataset to import")
    p.add_argument("--link", action="store_true")
    p.set_defaults(fn=cmd_setup)
    p = sub.add_parser("w2v", help="train word2vec vectors on the experiment text (reference w2v.py)")
    _common(p)
    p.add_argument("--input", action="append", default=None, help="JSONL file(s); default: the train/val split")
    p.add_argument("--window", type=int, default=10)
    p.add_argument("--min-count", type=int, default=1)
    p.add_argument("--iter", type=int, default=5)
    p.add_argument("--sg", action="store_true", help="skip-gram instead of CBOW")
    p.add_argument("--force", action="store_true", help="retrain even if the model exists")
    p.set_defaults(fn=cmd_w2v)
    p = sub.add_parser("train")
    _common(p)
    p.add_argument("--synthetic", action="store_true")
    p.add_argument("--synthetic-pages", type=int, default=65536)
    p.add_argument("--shuffle", action="store_true")
    p.add_argument("--resume", action="store_true")
    p.add_argument("--data", default=None, help="training JSONL (default: the experiment's model_training_data)")
    p.add_argument("--validation-split", type=float, default=None,
                   help="v1 in-memory mode: hold out the last fraction of --data for validation (Keras "
                        "validation_split), pad to the dataset's longest text, shuffle every epoch")
    p.set_defaults(fn=cmd_train)
    p = sub.add_parser("encode")
    _common(p)
    p.add_argument("--input", required=True)
    p.add_argument("--output", required=True)
    p.add_argument("--tower", default="doc", choices=["doc", "query"])
    p.add_argument("--weights", default=None)
    p.set_defaults(fn=cmd_encode)
    p = sub.add_parser("eval")
    _common(p)
    p.add_argument("--weights", default=None)
    p.add_argument("--pages", type=int, default=2048, help="synthetic pairs (without --data)")
    p.add_argument("--data", default=None,
                   help="JSONL {'q','doc_corr','doc_incorr'} file to evaluate on, or 'validation' for the "
                        "experiment's model_validation_data")
    p.add_argument("--max-rows", type=int, default=0, help="evaluate the first N rows only (0 = all)")
    p.add_argument("--no-negatives", action="store_true", help="rank against the positive pages only")
    p.add_argument("--metrics", default=None, help="append the eval record to this metrics JSONL")
    p.set_defaults(fn=cmd_eval)
    p = sub.add_parser("serve", help="HTTP page-vector service: /encode, /index/add, /search")
    _common(p)
    p.add_argument("--weights", default=None)
    p.add_argument("--pages", default=None, help='JSONL {"id": ..., "text": ...} to index at startup')
    p.add_argument("--index", default=None, help="saved PageIndex path to load")
    p.add_argument("--host", default="127.0.0.1")
    p.add_argument("--port", type=int, default=8000)
    p.add_argument("--max-batch", type=int, default=4096)
    p.add_argument("--max-wait-ms", type=float, default=2.0)
    p.add_argument("--save-dir", default=None,
                   help="directory POST /index/save may write into (default: saving over HTTP disabled)")
    p.add_argument("--max-items", type=int, default=4096, help="max texts / pages / queries per request")
    p.set_defaults(fn=cmd_serve)
    p = sub.add_parser("bench", help="run bench.py (headline benchmark)")
    p.add_argument("rest", nargs=argparse.REMAINDER)
    p.set_defaults(fn=lambda a: __import__("subprocess").call([sys.executable, os.path.join(
        os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bench.py")] + a.rest))
    a = ap.parse_args(argv)
    return int(a.fn(a) or 0)


if __name__ == "__main__":
    sys.exit(main())
