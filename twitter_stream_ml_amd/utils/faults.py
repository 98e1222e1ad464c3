"""Failure detection and fault injection (SURVEY §5 "failure detection").

* :class:`Watchdog` -- a per-process timer kicked once per micro-batch.  A
  batch that does not finish within ``timeout_s`` (a peer rank died inside a
  collective, a hung device) aborts the communicator and exits the process
  with :data:`EXIT_HUNG`, so the launcher (``torchrun --max-restarts``) can
  restart the group from the last checkpoint (``--resume auto``).
* :func:`maybe_inject` -- test hook driven by ``TWTML_FAULT``, e.g.
  ``rank=1,batch=4,kind=exit`` (``kind`` = ``exit`` | ``raise`` | ``hang``):
  kills / fails / stalls that rank right before it processes that batch.
"""
from __future__ import annotations

import logging
import os
import threading
import time
from typing import Callable, Optional

__all__ = ["Watchdog", "maybe_inject", "FaultInjected", "EXIT_FAULT", "EXIT_HUNG"]

log = logging.getLogger("twtml.faults")
EXIT_FAULT = 13
EXIT_HUNG = 75


class FaultInjected(RuntimeError):
    pass


def _parse(spec: str) -> dict:
    out = {}
    for part in spec.split(","):
        if "=" in part:
            k, v = part.split("=", 1)
            out[k.strip()] = v.strip()
    return out


def maybe_inject(rank: int, batch: int, spec: Optional[str] = None) -> None:
    """Trigger the fault described by ``TWTML_FAULT`` if it targets (rank, batch)."""
    spec = os.environ.get("TWTML_FAULT", "") if spec is None else spec
    if not spec:
        return
    f = _parse(spec)
    if int(f.get("rank", -1)) not in (-1, rank) or int(f.get("batch", -1)) != batch:
        return
    kind = f.get("kind", "exit")
    log.error("fault injection: rank %d batch %d kind %s", rank, batch, kind)
    if kind == "raise":
        raise FaultInjected(f"injected fault at rank {rank} batch {batch}")
    if kind == "hang":
        while True:
            time.sleep(3600)
    logging.shutdown()
    os._exit(EXIT_FAULT)


class Watchdog:
    """Abort the process if a kicked section does not complete in time."""

    def __init__(self, timeout_s: float, on_timeout: Optional[Callable[[], None]] = None,
                 name: str = "batch"):
        self.timeout_s = float(timeout_s)
        self.on_timeout = on_timeout
        self.name = name
        self._deadline: Optional[float] = None
        self._lock = threading.Lock()
        self._stop = threading.Event()
        self.fired = False
        self._thread: Optional[threading.Thread] = None
        if self.timeout_s > 0:
            self._thread = threading.Thread(target=self._run, name="twtml-watchdog", daemon=True)
            self._thread.start()

    def arm(self) -> None:
        with self._lock:
            self._deadline = time.monotonic() + self.timeout_s

    def disarm(self) -> None:
        with self._lock:
            self._deadline = None

    def __enter__(self) -> "Watchdog":
        self.arm()
        return self

    def __exit__(self, *exc) -> None:
        self.disarm()

    def close(self) -> None:
        self._stop.set()

    def _run(self) -> None:
        while not self._stop.wait(min(1.0, max(0.05, self.timeout_s / 10))):
            with self._lock:
                late = self._deadline is not None and time.monotonic() > self._deadline
            if late:
                self.fired = True
                log.critical("%s exceeded %.1f s: peer failure or hang; aborting", self.name,
                             self.timeout_s)
                try:
                    if self.on_timeout is not None:
                        self.on_timeout()
                finally:
                    if self.on_timeout is None:
                        logging.shutdown()
                        os._exit(EXIT_HUNG)
                return
