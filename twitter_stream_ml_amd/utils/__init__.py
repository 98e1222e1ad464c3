"""Utilities: Utils.round, logging setup, metrics JSONL, tracing ranges."""
from ..oracle.mllib import round_half_up
from .logging import setup_logging
from .metrics import MetricsLogger
from .tracing import trace_range

__all__ = ["round_half_up", "setup_logging", "MetricsLogger", "trace_range", "Utils"]


class Utils:
    """``com.giorgioinf.twtml.spark.Utils`` (``Utils.scala:3-7``)."""

    @staticmethod
    def round(number: float) -> float:
        return round_half_up(number)
