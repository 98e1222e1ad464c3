"""Resume / checkpoint / failure-detection plumbing shared by the drivers."""
from __future__ import annotations

import logging
import os
from dataclasses import dataclass
from typing import Callable, Optional

from ..checkpoint import StreamPositions, load_progress, resolve_resume
from ..utils.faults import EXIT_HUNG, Watchdog

__all__ = ["ResumeState", "load_resume_state", "StreamCheckpointer", "make_watchdog"]

log = logging.getLogger("twtml.apps")


@dataclass
class ResumeState:
    path: Optional[str] = None     # model directory to warm start from
    batches: int = 0               # batches already trained into that model
    count: int = 0                 # the driver's "count" accumulator
    records: int = 0               # source records this rank had consumed


def load_resume_state(resume: str, checkpoint: str, rank: int) -> ResumeState:
    """``--resume DIR`` warm-starts (stream restarts at 0, as loading an MLlib
    model would); ``--resume auto`` continues a checkpointed run exactly."""
    path = resolve_resume(resume, checkpoint)
    if path is None:
        return ResumeState()
    if resume != "auto":
        return ResumeState(path)      # warm start: weights only, a fresh stream
    prog = load_progress(path) or {}
    batches = int(prog.get("batches", 0))
    st = ResumeState(path, batches, int(prog.get("count", 0)), 0)
    if batches > 0:
        rec = StreamPositions(path, rank).records_at(batches)
        if rec is None:
            raise RuntimeError(f"checkpoint {path} is at batch {batches} but rank {rank} has no "
                               f"stream position for it (inconsistent checkpoint)")
        st.records = rec
    return st


class StreamCheckpointer:
    """Every ``interval`` batches: each rank records its stream position, a
    barrier, then rank 0 atomically replaces the model directory (with
    ``streaming/progress.json``).  A crash at any point leaves a model whose
    batch count every rank can resume from."""

    def __init__(self, path: str, interval: int, rank: int,
                 save_model: Callable[[str, dict], None], barrier: Callable[[], None]):
        self.path = path
        self.interval = int(interval)
        self.rank = rank
        self.save_model = save_model
        self.barrier = barrier
        self.positions = StreamPositions(path, rank) if path else None

    def after_batch(self, batches: int, records: int, count: int, force: bool = False) -> bool:
        if not self.path:
            return False
        if not force and (self.interval <= 0 or batches % self.interval != 0):
            return False
        self.positions.record(batches, records)
        self.barrier()
        if self.rank == 0:
            self.save_model(self.path, {"batches": int(batches), "count": int(count)})
            log.info("checkpoint written to %s after %d batches", self.path, batches)
        return True


def make_watchdog(timeout_s: float, comm=None) -> Optional[Watchdog]:
    """``--batchTimeout``: abort the RCCL communicator and exit if a batch
    hangs (e.g. a peer died inside a collective)."""
    if not timeout_s or timeout_s <= 0:
        return None

    def on_timeout() -> None:
        try:
            if comm is not None and hasattr(comm, "abort"):
                comm.abort()
        finally:
            logging.shutdown()
            os._exit(EXIT_HUNG)

    return Watchdog(timeout_s, on_timeout, name="micro-batch")
