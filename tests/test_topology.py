"""xGMI message-class policy (parallel/topology.py)."""
import os

from dnn_page_vectors_amd.parallel import topology


def test_message_classes_and_buckets():
    assert topology.message_class(12.6) == "latency"      # CDSSM-ngram gradient
    assert topology.message_class(126.0) == "bandwidth"   # MLP 512-512-128
    assert topology.message_class(440.0) == "bandwidth"   # BERT-base
    # latency class: one bucket per tower cut (bigger than the whole gradient)
    assert topology.bucket_mb(12.6, 32.0) > 12.6
    assert topology.bucket_mb(440.0, 32.0) == topology.BANDWIDTH_BUCKET_MB
    assert topology.bucket_mb(440.0, 8.0) == 8.0  # an explicit grad_bucket_mb wins


def test_channel_floor_only_for_bandwidth_class_and_never_overrides(monkeypatch):
    monkeypatch.delenv("NCCL_MIN_NCHANNELS", raising=False)
    topology._APPLIED.clear()
    assert topology.apply_env(12.6, 8) == {} and "NCCL_MIN_NCHANNELS" not in os.environ
    assert topology.apply_env(440.0, 1) == {}  # single process: nothing to tune
    got = topology.apply_env(440.0, 8)
    assert got == {"NCCL_MIN_NCHANNELS": str(topology.BANDWIDTH_MIN_CHANNELS)}
    monkeypatch.setenv("NCCL_MIN_NCHANNELS", "4")
    topology._APPLIED.clear()
    assert topology.apply_env(440.0, 8) == {} and os.environ["NCCL_MIN_NCHANNELS"] == "4"
    topology._APPLIED.clear()
