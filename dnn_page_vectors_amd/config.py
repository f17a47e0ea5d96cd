"""Typed experiment configuration.

Mirrors the reference's hard-coded attribute bag ``Configuration``
(``dssm_cnn_v2/config.py:8-91``) with the *same field names*, plus the trainer
module constants of ``dssm_cnn_v2/cnn_dssm_th.py:28-54`` (``embedding_dim``,
``batch_size``, ``nb_epoch``, ``filter_sizes``, ``num_filters``,
``dropout_prob``, ``hidden_dims``, ``J``, ``GAMMA``, ...).

Differences from the reference (documented, deliberate):

* everything is overridable: ``Configuration.from_yaml(path)``,
  ``cfg.override(["batch_size=4096", "feature_level=ngram"])`` (CLI ``--set``);
* ``query_length``/``document_length`` are derived from ``feature_level``
  exactly as in ``config.py:80-91`` unless explicitly set;
* the experiment timestamp follows ``config.py:21-35`` (fixed string when
  ``reuse_experiment_timestamp`` else a ``_TIMESTAMP`` JSON file);
* S3 URIs are kept for reference but the workspace setup copies from local
  paths (there is no network on the GPU box);
* pickles become JSON / safetensors (see ``io/checkpoint.py``).
"""
from __future__ import annotations

import dataclasses
import json
import logging
import os
from dataclasses import dataclass, field, fields
from typing import Any, Dict, List, Optional, Sequence, Tuple

from .utils.fs import create_dir, get_current_date_time

# (query_length, document_length) per feature level, config.py:80-91
FEATURE_LEVEL_LENGTHS: Dict[str, Tuple[int, int]] = {
    "word": (20, 975),
    "char": (250, 5000),
    "ngram": (45, 2000),
}

FIXED_TIMESTAMP = "2016-09-16T23-04-38"  # config.py:23-24


@dataclass
class Configuration:
    # ---- experiment layout (config.py:17-75) ---------------------------------
    experiment_root_directory: str = "/tmp/pagevec_project_data"
    reuse_experiment_timestamp: bool = True
    experiment_name: str = "dssm_cnn_v2"
    feature_level: str = "char"          # word | ngram | char
    default_ngram: int = 3
    word_vectors: str = "fast"            # fast | word2vec
    input_dataset_s3_path: str = "s3://ankit-test/ebs_backup/lstm/model_training_data.txt"
    word2vec_wordvector_s3_path: str = "s3://ankit-test/vectors_final/vectors_wholecorpus100.txt"
    fast_wordvector_s3_path: str = "s3://ankit-test/fast_model/full_model.vec"
    create_data_dump: bool = True
    num_negative_examples: int = 3
    train_validation_split: float = 0.2
    query_length: Optional[int] = None
    document_length: Optional[int] = None

    # ---- featurization (new) -------------------------------------------------
    # 0 => exact vocabulary (reference); >0 => hashed ids in [1, vocab_hash_size)
    vocab_hash_size: int = 0
    html_normalize: bool = False          # utils/word2vec_normalizer.py mode

    # ---- model hyper-parameters (cnn_dssm_th.py:28-44) -----------------------
    model: str = "cdssm"                  # cdssm | mlp | bert | chunked | lstm
    embedding_dim: int = 100
    batch_size: int = 128
    nb_epoch: int = 5
    filter_sizes: Tuple[int, ...] = (3, 4)
    num_filters: int = 150
    dropout_prob: Tuple[float, ...] = (0.25, 0.5)
    hidden_dims: int = 150
    J: int = 3
    GAMMA: float = 10.0
    num_train_samples: int = 16000
    num_validation_samples: int = 4000
    embeddings_pickled: bool = False
    vocab_pickled: bool = False
    embedding_weights_masking: bool = False
    share_doc_tower: bool = True          # v1 (dssm_cnn/cnn_dssm.py:160-168) used 5 unshared towers
    final_dropout: bool = False           # v1 Dropout(0.5) before the last ReLU (dssm_cnn/cnn_dssm.py:149)
    embed_dropout_mode: str = "element"   # element (Keras-exact) | token (row mask) | none

    # MLP tower (config 1 / 3): trigram bag -> dense stack
    mlp_dims: Tuple[int, ...] = (512, 512, 128)
    mlp_act: str = "tanh"                 # DSSM hidden activation (tanh | relu)
    # BERT dual encoder (config 4)
    bert_layers: int = 12
    bert_hidden: int = 768
    bert_heads: int = 12
    bert_intermediate: int = 3072
    bert_vocab: int = 30522
    bert_max_len: int = 512
    bert_out_dim: int = 0                 # 0 => CLS vector (768), else projection
    bert_dropout: float = 0.1
    # chunked long-page encoder (config 5)
    chunk_len: int = 512
    num_chunks: int = 8
    chunk_encoder: str = "mlp"           # mlp | cdssm
    cdssm_act: str = "relu"              # the CDSSM tower's Dense activation: relu (reference) | tanh
    chunk_pool: str = "auto"             # auto = mean of the chunk vectors | max (cdssm: max of the chunks' conv features)
    use_fp8: bool = False
    # LSTM legacy tower (old_scripts/lstm.py:125-200)
    lstm_output_size: int = 64
    lstm_dense_units: int = 32
    lstm_conv: bool = False               # lstm_new.py: Conv1D(64,3)+MaxPool(2) before the LSTM

    # ---- training (new) ------------------------------------------------------
    loss_mode: str = "explicit"          # explicit (J negatives, parity) | in_batch | cross_gpu
    cos_clip: bool = True                 # R = clip(cos, 0, 1) as RTH/RTF (cnn_dssm_th.py:76-78)
    # softmax scale of the in-batch / cross-GPU losses (new modes: the reference's GAMMA = 10
    # belongs to its 4-way head); 0 = GAMMA
    inbatch_gamma: float = 0.0
    lr: float = 1e-3                      # Keras 1 Adam defaults
    beta1: float = 0.9
    beta2: float = 0.999
    adam_eps: float = 1e-8
    lazy_embedding_adam: bool = False    # Adam skips embedding rows with an all-zero gradient (large vocabularies)
    # row-sparse embedding gradients (parallel/sparse_rows.py): only the touched rows are zeroed,
    # exchanged between data-parallel ranks (all-gather of ids + rows, not a dense all-reduce)
    # and updated (LazyAdam) — for million-row word vocabularies
    sparse_embedding_grad: bool = False
    # padding of the row exchange: -1 = min(V, noted ids) agreed once (no per-step host sync:
    # capturable), 0 = exact per-step maximum (a host sync per table and step), > 0 = rows
    sparse_rows_capacity: int = -1
    optimizer_bf16_mirror: bool = True   # the Adam kernel also writes the bf16 compute copies of big weights
    # compute precision (ops/_common.py::precision_scope): bf16 = the HIP kernels (bf16 MFMA
    # operands, fp32 accumulation / master weights); fp32 = the reference's precision, no bf16
    # anywhere: the CDSSM conv tower on fp32-MFMA kernels (conv_pool_f32.hip), the other ops
    # through PyTorch's fp32 ops.  CPU runs compute fp32 either way.
    dtype: str = "bf16"
    seed: int = 1337                      # np.random.seed(1337), cnn_dssm_th.py:20
    backend: str = "auto"                 # auto | hip | torch  (op implementation)
    grad_bucket_mb: float = 32.0
    lr_warmup_steps: int = 0              # linear learning-rate warmup (0 = none; Keras had none)
    # graph mode on a data-parallel run captures the whole step INCLUDING its RCCL collectives
    # (page / query gathers, bucketed gradient all-reduces) in the hipGraph.  Opt-in (round 6):
    # it is verified on a world-1 RCCL group only (tests/test_rccl_gpu.py), no multi-rank run has
    # replayed it yet; when on, the ranks agree on the capture outcome and all fall back to eager
    # steps if any rank's capture failed (Trainer._capture_agreed)
    graph_distributed: bool = False
    query_stream: bool = True             # query tower (fwd, hence bwd) on a side HIP stream
    deterministic: bool = False           # order-free (fixed-point) GPU reductions, one stream (ops/determinism.py)
    placement: str = "dp"                # dp (data parallel) | tower (slots over ranks, cnn_dssm_tf.py:139-158)
    log_every: int = 10
    skip_nonfinite: bool = True
    prefetch: int = 2                     # featurized batches the loader thread keeps ahead (pinned)
    num_workers: int = 0                  # featurizer threads per batch (C++ pool); 0 = min(16, CPUs)
    # saved-config format: 2 = dtype 'fp32' selects the reference-precision path (in
    # version-1 files, written before the field existed, 'fp32' was the no-op default)
    config_version: int = 2

    # --------------------------------------------------------------------------
    def __post_init__(self) -> None:
        self.filter_sizes = tuple(int(x) for x in self.filter_sizes)
        self.dropout_prob = tuple(float(x) for x in self.dropout_prob)
        self.mlp_dims = tuple(int(x) for x in self.mlp_dims)
        if self.feature_level not in FEATURE_LEVEL_LENGTHS:
            raise ValueError(f"feature_level must be one of {sorted(FEATURE_LEVEL_LENGTHS)}")
        ql, dl = FEATURE_LEVEL_LENGTHS[self.feature_level]
        if self.query_length is None:
            self.query_length = ql
        if self.document_length is None:
            self.document_length = dl
        if self.dtype not in ("bf16", "fp32"):
            raise ValueError(f"dtype must be 'bf16' (HIP kernels) or 'fp32' (reference precision), got {self.dtype!r}")
        if self.use_fp8 and self.dtype != "bf16":
            raise ValueError("use_fp8 (fp8 chunk GEMMs) runs on the HIP path: it needs dtype='bf16'")
        if self.chunk_encoder not in ("mlp", "cdssm"):
            raise ValueError(f"chunk_encoder must be 'mlp' or 'cdssm', got {self.chunk_encoder!r}")
        if self.num_workers < 0 or self.prefetch < 1:
            raise ValueError("num_workers must be >= 0 (0 = auto) and prefetch >= 1")

    # ---- derived paths (config.py:41-75) --------------------------------------
    @property
    def timestamp(self) -> str:
        if self.reuse_experiment_timestamp:
            return FIXED_TIMESTAMP
        tsf = os.path.join(self.experiment_root_directory, "_TIMESTAMP")
        if os.path.exists(tsf):
            with open(tsf) as f:
                return json.load(f)["project_timestamp"]
        ts = get_current_date_time()
        create_dir(self.experiment_root_directory)
        with open(tsf, "w") as f:
            json.dump({"project_timestamp": ts}, f)
        return ts

    @property
    def data_path(self) -> str:
        return os.path.join(self.experiment_root_directory, self.experiment_name, self.timestamp, self.feature_level)

    @property
    def data_dir(self) -> str:
        return os.path.join(self.data_path, "data")

    @property
    def trained_model_dir(self) -> str:
        return os.path.join(self.data_path, "model")

    @property
    def pickle_files_dir(self) -> str:
        return os.path.join(self.data_path, "pickled_files")

    @property
    def vectors_directory(self) -> str:
        return os.path.join(self.experiment_root_directory, "vectors")

    @property
    def word_vectors_file(self) -> str:
        name = "vectors_wholecorpus100.txt" if self.word_vectors == "word2vec" else "fast_model_ns.vec"
        return os.path.join(self.vectors_directory, name)

    @property
    def input_dataset(self) -> str:
        return os.path.join(self.data_dir, "input_dataset_new.txt")

    @property
    def model_training_data(self) -> str:
        return os.path.join(self.data_dir, "model_training_data_new.txt")

    @property
    def model_validation_data(self) -> str:
        return os.path.join(self.data_dir, "model_validation_data_new.txt")

    @property
    def input_file_list(self) -> List[str]:
        return [self.model_training_data, self.model_validation_data]

    # pickles of the reference become JSON (vocab) / safetensors (weights)
    @property
    def vocab_set_file(self) -> str:
        return os.path.join(self.pickle_files_dir, "vocab_set_{}.json")

    @property
    def vocab_index_file(self) -> str:
        return os.path.join(self.pickle_files_dir, "vocab_index_dict_{}.json")

    @property
    def embedding_weights_file_tpl(self) -> str:
        return os.path.join(self.pickle_files_dir, "we_embedding_weights_compact_{}.safetensors")

    @property
    def masking_value(self) -> str:
        return "masked" if self.embedding_weights_masking else "non_masked"

    # ---- serialization / overrides -------------------------------------------
    def to_dict(self) -> Dict[str, Any]:
        d = dataclasses.asdict(self)
        for k, v in d.items():
            if isinstance(v, tuple):
                d[k] = list(v)
        return d

    @classmethod
    def from_dict(cls, d: Dict[str, Any]) -> "Configuration":
        names = {f.name for f in fields(cls)}
        unknown = set(d) - names
        if unknown:
            raise KeyError(f"unknown configuration keys: {sorted(unknown)}")
        return cls(**d)

    @classmethod
    def from_yaml(cls, path: str) -> "Configuration":
        import yaml

        with open(path) as f:
            d = yaml.safe_load(f) or {}
        preset = d.pop("preset", None)
        base = preset_config(preset) if preset else cls()
        return base.replace(**d)

    def replace(self, **kw: Any) -> "Configuration":
        d = self.to_dict()
        # lengths follow feature_level unless explicitly given
        if "feature_level" in kw and kw["feature_level"] != self.feature_level:
            d["query_length"] = None
            d["document_length"] = None
        d.update(kw)
        return Configuration.from_dict(d)

    def override(self, assignments: Sequence[str]) -> "Configuration":
        """Apply ``key=value`` strings (CLI ``--set``); values parsed as YAML scalars."""
        import yaml

        kw: Dict[str, Any] = {}
        types = {f.name: f for f in fields(self)}
        for a in assignments:
            if "=" not in a:
                raise ValueError(f"override must be key=value, got {a!r}")
            k, v = a.split("=", 1)
            k = k.strip()
            if k not in types:
                raise KeyError(f"unknown configuration key {k!r}")
            val = yaml.safe_load(v)
            cur = getattr(self, k)
            # YAML 1.1 reads "2e-3" (no dot) as a string: coerce to the field's current type
            if isinstance(val, (str, int)) and not isinstance(val, bool) and isinstance(cur, float):
                val = float(val)
            elif isinstance(val, str) and isinstance(cur, int) and not isinstance(cur, bool):
                val = int(val)
            if isinstance(cur, tuple) and not isinstance(val, (list, tuple)):
                val = [val]
            kw[k] = val
        return self.replace(**kw)

    def save_json(self, path: str) -> None:
        with open(path, "w") as f:
            json.dump(self.to_dict(), f, indent=2, sort_keys=True)

    @classmethod
    def load_json(cls, path: str) -> "Configuration":
        with open(path) as f:
            d = json.load(f)
        if "config_version" not in d:  # version 1: saved before the version field existed
            if d.get("dtype") == "fp32":
                # a version-1 file cannot tell the old no-op fp32 default (before 066a651) from an
                # explicit choice of reference precision made later: keep what the file says
                logging.getLogger(__name__).warning(
                    "%s: version-1 config with dtype='fp32' loads as reference precision (fp32 "
                    "kernels); configs saved before 066a651 meant the bf16 HIP path by it — set "
                    "dtype='bf16' for that", path)
            d["config_version"] = 2
        return cls.from_dict(d)


# ---- presets: the reference run + the five BASELINE.json configs -------------
def preset_config(name: str) -> Configuration:
    name = name.lower()
    if name in ("reference", "reference_char", "cdssm_v2"):
        # exact dssm_cnn_v2/cnn_dssm_th.py run configuration, in its fp32 precision
        return Configuration(dtype="fp32")
    if name in ("reference_v1", "cdssm_v1"):
        return Configuration(feature_level="word", batch_size=1024, nb_epoch=3,
                             share_doc_tower=False, final_dropout=True, dtype="fp32")
    if name in ("tiny_dssm_cpu", "config1"):
        # Tiny 3-layer DSSM, 1k tri-gram hash, batch 32 on CPU
        return Configuration(model="mlp", feature_level="ngram", vocab_hash_size=1024,
                             embedding_dim=300, mlp_dims=(300, 300, 128), batch_size=32,
                             query_length=45, document_length=256, nb_epoch=1, loss_mode="in_batch",
                             cos_clip=False, lr=3e-3, J=0, num_train_samples=1024, num_validation_samples=256)
    if name in ("cdssm_ngram_bf16", "config2"):
        # CDSSM 1D-conv 300d, 30k hashed tri-grams, bf16, batch 4096 on 1 MI355X
        # inbatch_gamma 40: the reference's GAMMA = 10 is the scale of its 4-way head; over 16k
        # in-batch negatives it caps Recall@10 near 0.15 (profiles/quality_r2_final.md:
        # 2000 steps, gamma 10 / 20 / 40 / 80 -> Recall@10 0.15 / 0.29 / 0.35 / 0.37)
        return Configuration(model="cdssm", feature_level="ngram", vocab_hash_size=30000,
                             batch_size=4096, dtype="bf16", loss_mode="cross_gpu", inbatch_gamma=40.0)
    if name in ("mlp_xgpu", "config3"):
        # Two-tower MLP 512-512-128, cross-GPU in-batch negatives via all-gather
        return Configuration(model="mlp", feature_level="ngram", vocab_hash_size=30000,
                             embedding_dim=512, mlp_dims=(512, 512, 128), batch_size=4096,
                             dtype="bf16", loss_mode="cross_gpu", J=0, cos_clip=False, lr=3e-3)
    if name in ("bert_dp8", "config4"):
        # recipe (round-5 sweeps, profiles/r5_bert/ + r5_bq2/, Recall@10 after the 200-step
        # bench protocol): lr 2e-5 with the reference's softmax scale 10 and [0, 1] cosine clip
        # 0.25; scale 20 without the clip: lr 2e-5 0.25-0.38 (five runs), 3e-5 0.42 / 0.42,
        # 5e-5 (20 warmup steps) 0.19 / 0.09, 1e-4 collapses (loss stays ln B); scale 30 0.31,
        # 40 0.06.  The fp32 parity arm at full depth (12 layers, B 64) agrees with the HIP step
        # (tail loss 0.2 %, Recall@10 0.002 apart: tools/bert_parity.py)
        return Configuration(model="bert", feature_level="word", vocab_hash_size=30522,
                             query_length=32, document_length=256, batch_size=256,
                             dtype="bf16", loss_mode="cross_gpu", J=0, lr=3e-5,
                             inbatch_gamma=20.0, cos_clip=False)
    if name in ("longpage_fp8", "config5"):
        return Configuration(model="chunked", feature_level="ngram", vocab_hash_size=30000,
                             embedding_dim=512, mlp_dims=(512, 512, 128), chunk_len=512,
                             num_chunks=8, query_length=45, document_length=4096,
                             batch_size=512, dtype="bf16", use_fp8=True, loss_mode="cross_gpu", J=0,
                             # the MLP tower's in-batch training setting (mlp_xgpu): with the
                             # reference's [0, 1] cosine clip a fresh batch whose cosines all sit
                             # <= 0 has zero gradient (loss stuck at ln B, measured round 3)
                             cos_clip=False, lr=3e-3)
    if name in ("longpage_cdssm", "config5_cdssm"):
        # config 5 with the reference's conv tower as the chunk encoder (8 x 512-trigram chunks
        # through the fused conv kernel, chunk vectors mean-pooled).  Recipe (round-4 sweeps,
        # profiles/r4_quality/README.md, Recall@10 after the 500-step protocol): the reference's
        # ReLU Dense head + cosine clip made every chunk vector non-negative, and their mean
        # washed out a query's chunk (0.15 at lr 1e-3, 0.22-0.25 at 3e-3); a tanh head without
        # the clip (like the MLP chunk encoder) 0.35, and embedding dropout 0.1 instead of 0.25
        # 0.39-0.42; 0.125 = 2/16 keeps the one-hash-per-8-columns mask path (0.1 does not)
        return Configuration(model="chunked", chunk_encoder="cdssm", feature_level="ngram",
                             vocab_hash_size=30000, chunk_len=512, num_chunks=8, query_length=45,
                             document_length=4096, batch_size=512, dtype="bf16", loss_mode="cross_gpu",
                             J=0, inbatch_gamma=40.0, lr=3e-3, cdssm_act="tanh", cos_clip=False,
                             dropout_prob=(0.125, 0.5))
    if name in ("lstm", "legacy_lstm"):
        return Configuration(model="lstm", feature_level="word", batch_size=64, nb_epoch=2)
    raise KeyError(f"unknown preset {name!r}")


PRESETS = ["reference_char", "reference_v1", "tiny_dssm_cpu", "cdssm_ngram_bf16",
           "mlp_xgpu", "bert_dp8", "longpage_fp8", "longpage_cdssm", "lstm"]
