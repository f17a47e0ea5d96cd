"""Logging setup with the reference's ``LOG_CFG`` semantics (log/setup_log.py:9-25)."""
from .setup_log import setup_logging  # noqa: F401
