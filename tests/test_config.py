import os

import pytest

from dnn_page_vectors_amd.config import FEATURE_LEVEL_LENGTHS, PRESETS, Configuration, preset_config


def test_reference_defaults():
    c = Configuration()
    assert (c.feature_level, c.query_length, c.document_length) == ("char", 250, 5000)
    assert c.num_negative_examples == 3 and c.train_validation_split == 0.2
    assert (c.embedding_dim, c.batch_size, c.nb_epoch, c.filter_sizes, c.num_filters, c.hidden_dims, c.J,
            c.GAMMA) == (100, 128, 5, (3, 4), 150, 150, 3, 10.0)
    assert c.timestamp == "2016-09-16T23-04-38"
    assert c.data_path.endswith(os.path.join("dssm_cnn_v2", "2016-09-16T23-04-38", "char"))
    assert c.trained_model_dir.endswith("model") and c.pickle_files_dir.endswith("pickled_files")
    assert c.input_file_list == [c.model_training_data, c.model_validation_data]


@pytest.mark.parametrize("lvl", list(FEATURE_LEVEL_LENGTHS))
def test_lengths_follow_feature_level(lvl):
    c = Configuration().replace(feature_level=lvl)
    assert (c.query_length, c.document_length) == FEATURE_LEVEL_LENGTHS[lvl]


def test_override_and_yaml(tmp_path):
    c = Configuration().override(["batch_size=4096", "feature_level=ngram", "filter_sizes=[3,4,5]"])
    assert c.batch_size == 4096 and c.document_length == 2000 and c.filter_sizes == (3, 4, 5)
    y = tmp_path / "c.yaml"
    y.write_text("preset: cdssm_ngram_bf16\nbatch_size: 8\n")
    c2 = Configuration.from_yaml(str(y))
    assert c2.vocab_hash_size == 30000 and c2.batch_size == 8
    with pytest.raises(KeyError):
        Configuration().override(["nope=1"])


def test_presets_construct():
    for p in PRESETS:
        c = preset_config(p)
        assert c.query_length > 0 and c.document_length > 0


def test_timestamp_file(tmp_path):
    c = Configuration(experiment_root_directory=str(tmp_path), reuse_experiment_timestamp=False)
    ts = c.timestamp
    assert os.path.exists(tmp_path / "_TIMESTAMP")
    assert c.timestamp == ts


def test_json_roundtrip(tmp_path):
    c = preset_config("mlp_xgpu")
    p = tmp_path / "c.json"
    c.save_json(str(p))
    assert Configuration.load_json(str(p)) == c


def test_config_validation_and_precision_scope():
    from dnn_page_vectors_amd.ops._common import get_backend, precision_scope

    with pytest.raises(ValueError):
        Configuration(dtype="fp16")
    with pytest.raises(ValueError):
        Configuration(dtype="fp32", use_fp8=True)
    with pytest.raises(ValueError):
        Configuration(chunk_encoder="bert")
    with pytest.raises(ValueError):
        Configuration(num_workers=-1)
    assert preset_config("reference_char").dtype == "fp32"      # the reference trains in fp32
    assert preset_config("cdssm_ngram_bf16").dtype == "bf16"
    before = get_backend()
    with precision_scope(Configuration(dtype="fp32")):
        assert get_backend() == "torch"                         # no bf16 HIP kernel inside
    assert get_backend() == before
    with precision_scope(Configuration(dtype="bf16")):
        assert get_backend() == before


def test_override_coerces_yaml_strings_to_the_field_type():
    """`--set lr=2e-3`: YAML 1.1 parses exponent floats without a dot as strings."""
    from dnn_page_vectors_amd.config import Configuration

    c = Configuration().override(["lr=2e-3", "inbatch_gamma=60", "batch_size=64"])
    assert c.lr == 2e-3 and isinstance(c.lr, float)
    assert c.inbatch_gamma == 60.0 and isinstance(c.inbatch_gamma, float)
    assert c.batch_size == 64
