"""Logging with the reference's levels (``log4j.properties:1-17``).

Root at WARN, the application loggers (``com.giorgioinf``) at DEBUG, pattern
``yy/MM/dd HH:mm:ss LEVEL logger: message`` on stderr.  ``TWTML_LOG_LEVEL``
overrides the application level.
"""
from __future__ import annotations

import logging
import os
import sys

__all__ = ["setup_logging"]


def setup_logging(app_level: str | None = None, root_level: str = "WARNING") -> None:
    level = (app_level or os.environ.get("TWTML_LOG_LEVEL") or "DEBUG").upper()
    root = logging.getLogger()
    if not root.handlers:
        h = logging.StreamHandler(sys.stderr)
        h.setFormatter(logging.Formatter("%(asctime)s %(levelname)s %(name)s: %(message)s",
                                         datefmt="%y/%m/%d %H:%M:%S"))
        root.addHandler(h)
    root.setLevel(root_level)
    for name in ("com.giorgioinf", "twtml"):
        logging.getLogger(name).setLevel(level)
    for name in ("org.apache.spark", "org.apache.spark.mllib"):
        logging.getLogger(name).setLevel("INFO" if level == "DEBUG" else level)
