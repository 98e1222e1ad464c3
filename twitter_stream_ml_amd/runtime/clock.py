"""Batch clocks for the streaming scheduler (Spark's ``spark.streaming.clock``).

Spark Streaming reads batch times from a pluggable clock: ``SystemClock`` in
production, ``ManualClock`` in its own test suites (upstream
``org.apache.spark.util.ManualClock``; the reference's jobs run on the
default, ``LinearRegression.scala:40-44`` builds the context with
``Seconds(conf.seconds)``).  The batch time matters to the models: the
``age`` feature of every tweet is ``batch time - createdAt``
(``MllibHelper.scala:50``), so two runs agree on every weight only if they
see the same clock.

:class:`ManualClock` starts at ``start_ms`` and moves ``step_ms`` forward
each time a batch is sealed: the k-th batch of any run has time
``start_ms + k * step_ms`` and every poll of the receiver inside it reads the
same time, whatever the wall clock does.  ``TWTML_STREAMING_CLOCK=manual:
<start_ms>:<step_ms>`` selects it for the apps (tests, reproducible replays).
"""
from __future__ import annotations

import os
import threading
import time

__all__ = ["SystemClock", "ManualClock", "streaming_clock"]


class SystemClock:
    def now_ms(self) -> int:
        return int(time.time() * 1000)

    def advance(self) -> None:
        """Called after each sealed batch (a wall clock moves on its own)."""


class ManualClock:
    def __init__(self, start_ms: int, step_ms: int):
        self._t = int(start_ms)
        self.step_ms = int(step_ms)
        self._lock = threading.Lock()

    def now_ms(self) -> int:
        with self._lock:
            return self._t

    def advance(self) -> None:
        with self._lock:
            self._t += self.step_ms


def streaming_clock(spec: str = None):
    """Clock named by ``spec`` (default: ``$TWTML_STREAMING_CLOCK``): ``system``
    or ``manual:<start_ms>:<step_ms>``."""
    spec = (os.environ.get("TWTML_STREAMING_CLOCK", "") if spec is None else spec).strip()
    if not spec or spec == "system":
        return SystemClock()
    kind, _, rest = spec.partition(":")
    if kind == "manual":
        parts = rest.split(":")
        if len(parts) != 2:
            raise ValueError(f"streaming clock {spec!r}: expected manual:<start_ms>:<step_ms>")
        return ManualClock(int(parts[0]), int(parts[1]))
    raise ValueError(f"unknown streaming clock {spec!r} (system | manual:<start_ms>:<step_ms>)")
