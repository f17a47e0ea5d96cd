"""Pretrained word-vector ingestion (reference data_helpers.py:17-74 semantics) and the
LOG_CFG logging mechanism (reference log/setup_log.py:9-25)."""
import logging

import numpy as np
import torch

from dnn_page_vectors_amd.data.text import Vocab
from dnn_page_vectors_amd.io.vectors import init_embedding_, load_word_vectors
from dnn_page_vectors_amd.log import setup_log


def test_load_word_vectors_rules(tmp_path):
    p = tmp_path / "v.vec"
    p.write_text("4 3\n"                      # fastText header: skipped (too short)
                 "statue 0.1 0.2 0.3\n"
                 "liberty 1 2 3 4 5\n"          # extra columns: first dim kept
                 "short 1\n"                    # short line: skipped
                 "unknownword 9 9 9\n"          # not in vocab
                 "of x y z\n",                  # garbled floats: skipped
                 encoding="utf-8")
    voc = Vocab(["statue", "liberty", "of", "new"])
    W, found = load_word_vectors(str(p), voc, 3, seed=1)
    assert W.shape == (len(voc), 3) and W.dtype == np.float32
    assert found == 2
    np.testing.assert_allclose(W[voc.stoi["statue"]], [0.1, 0.2, 0.3], rtol=1e-6)
    np.testing.assert_allclose(W[voc.stoi["liberty"]], [1, 2, 3])
    assert np.all(W[voc.pad_id] == 0)
    rest = W[[voc.stoi["of"], voc.stoi["new"], 1, 2]]
    assert np.all(np.abs(rest) <= 0.25) and np.any(rest != 0)  # U(-0.25, 0.25) init
    emb = torch.nn.Parameter(torch.zeros(len(voc), 3))
    init_embedding_(emb, W)
    torch.testing.assert_close(emb.detach(), torch.from_numpy(W))


def test_setup_logging_log_cfg(tmp_path, monkeypatch):
    cfg = tmp_path / "log.yaml"
    logfile = tmp_path / "sub" / "x.log"
    cfg.write_text(f"""
version: 1
disable_existing_loggers: false
handlers:
  f:
    class: logging.FileHandler
    filename: {logfile}
    level: INFO
loggers:
  pagevec_test:
    level: INFO
    handlers: [f]
""")
    monkeypatch.setenv("LOG_CFG", str(cfg))
    setup_log.setup_logging()
    logging.getLogger("pagevec_test").info("hello from LOG_CFG")
    for h in logging.getLogger("pagevec_test").handlers:
        h.flush()
    assert "hello from LOG_CFG" in logfile.read_text()
    # missing file -> basicConfig fallback, no exception
    monkeypatch.setenv("LOG_CFG", str(tmp_path / "missing.yaml"))
    setup_log.setup_logging(default_path=str(tmp_path / "missing.yaml"))
