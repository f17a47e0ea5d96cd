"""YAML ``dictConfig`` logging, overridable through ``LOG_CFG``.

Same mechanism as the reference ``log/setup_log.py:9-25``: load the YAML at
``$LOG_CFG`` (or the packaged default); otherwise ``basicConfig(level)``.
Unlike the reference it is *not* installed as an import side effect
(``utils/gen_utils.py:12-13``); call it from entry points.
"""
from __future__ import annotations

import logging
import logging.config
import os

_DEFAULT = os.path.join(os.path.dirname(os.path.realpath(__file__)), "logging.yaml")


def setup_logging(default_path: str = _DEFAULT, default_level: int = logging.INFO,
                  env_key: str = "LOG_CFG") -> None:
    path = os.getenv(env_key, None) or default_path
    if os.path.exists(path):
        import yaml

        with open(path, "rt") as f:
            config = yaml.safe_load(f.read())
        # file handlers: make sure their directories exist
        for h in (config.get("handlers") or {}).values():
            fn = h.get("filename")
            if fn:
                os.makedirs(os.path.dirname(os.path.abspath(fn)), exist_ok=True)
        logging.config.dictConfig(config)
    else:
        logging.basicConfig(level=default_level)
