"""Resume / checkpoint / failure-detection plumbing shared by the drivers."""
from __future__ import annotations

import logging
import os
import threading
from dataclasses import dataclass
from typing import Callable, Optional

from ..checkpoint import StreamPositions, load_progress, resolve_resume
from ..utils.faults import EXIT_HUNG, Watchdog

__all__ = ["ResumeState", "load_resume_state", "StreamCheckpointer", "make_watchdog",
           "exit_on_sigterm"]

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


def background_writer_thread(threads: int = 2) -> None:
    """The calling thread is a background writer (checkpoints): lowest CPU
    priority for it, and at most ``threads`` pyarrow encode threads.  On a
    CPU quota (a GPU box's cgroup: 16 CPUs) a writer that fans out over
    pyarrow's default pool (one thread per machine CPU) throttles the whole
    process, the training thread included."""
    try:
        os.setpriority(os.PRIO_PROCESS, threading.get_native_id(), 19)   # this thread only (Linux)
    except (OSError, AttributeError):
        pass
    try:
        import pyarrow as pa
        if pa.cpu_count() > threads:
            pa.set_cpu_count(threads)
        pa.set_io_thread_count(min(threads, pa.io_thread_count()))
    except Exception:   # noqa: BLE001 -- pyarrow absent: the writer is not ours to tune
        pass


class StreamCheckpointer:
    """Every ``interval`` batches: each rank records its stream position, a
    barrier, then rank 0 takes a snapshot of the model and replaces the model
    directory (with ``streaming/progress.json``) atomically.  A crash at any
    point leaves a model whose batch count every rank can resume from
    (positions keep a history, ``checkpoint/stream_state.py``).

    ``snapshot()`` runs on the training thread between two batches and
    returns ``save(path, progress)``.  With ``asynchronous`` (the default)
    ``save`` runs on a writer thread while the next batches train: for the
    device LR engine the snapshot is a device-side compaction of the non-zero
    weights and ``save`` copies just those pairs to the host (its own stream)
    and writes the parquet file -- nothing of size F touches the training
    thread (an F = 1e8 checkpoint used to copy 800 MB and scan it
    on the host inside the batch).  One write is in flight at most: a
    checkpoint that comes due while the previous one is still being written
    is skipped (positions are still recorded; the next due batch snapshots
    the newest model), so training never waits on the disk -- with
    ``--checkpointInterval 1`` the model on disk is as fresh as the writer
    can keep it.  The final checkpoint (``force``) waits and is synchronous.
    Errors of a background write are raised at the next checkpoint or at
    :meth:`flush`."""

    def __init__(self, path: str, interval: int, rank: int,
                 snapshot: Callable[[], Callable[[str, dict], None]], barrier: Callable[[], None],
                 asynchronous: Optional[bool] = None):
        self.path = path
        self.interval = int(interval)
        self.rank = rank
        self.snapshot = snapshot
        self.barrier = barrier
        if asynchronous is None:
            asynchronous = os.environ.get("TWTML_CHECKPOINT_ASYNC", "1") != "0"
        self.asynchronous = bool(asynchronous)
        self.positions = StreamPositions(path, rank) if path else None
        self._thread: Optional[threading.Thread] = None
        self._error: Optional[BaseException] = None
        self.written = 0          # checkpoints completed (rank 0)
        self.skipped = 0          # due while the previous write was in flight (rank 0)

    def after_batch(self, batches: int, records: int, count: int, force: bool = False) -> bool:
        if not self.path:
            return False
        if not force and (self.interval <= 0 or batches % self.interval != 0):
            return False
        self.positions.record(batches, records)
        self.barrier()
        if self.rank == 0:
            progress = {"batches": int(batches), "count": int(count)}
            if self.asynchronous and not force:
                if self._thread is not None and self._thread.is_alive():
                    self.skipped += 1
                    log.debug("checkpoint after batch %d skipped: the previous write is in flight", batches)
                    return False
                self._wait_writer()
                save = self.snapshot()
                t = threading.Thread(target=self._write, args=(save, progress, batches),
                                     name="twtml-checkpoint", daemon=True)
                self._thread = t
                t.start()
            else:
                self._wait_writer()
                self._write(self.snapshot(), progress, batches)
                self._raise_error()
        return True

    def flush(self) -> None:
        """Wait for a background write (end of run) and raise its error."""
        self._wait_writer()

    def _write(self, save, progress: dict, batches: int) -> None:
        background_writer_thread()
        try:
            save(self.path, progress)
            self.written += 1
            log.info("checkpoint written to %s after %d batches", self.path, batches)
        except BaseException as e:   # surfaced on the training thread
            self._error = e

    def _wait_writer(self) -> None:
        t = self._thread
        if t is not None:
            t.join()
            self._thread = None
        self._raise_error()

    def _raise_error(self) -> None:
        if self._error is not None:
            e, self._error = self._error, None
            raise RuntimeError(f"checkpoint write to {self.path} failed: {e}") from e


def exit_on_sigterm() -> None:
    """Turn SIGTERM into ``SystemExit`` on the main thread, so the drivers'
    ``finally`` blocks run: a launcher that tears the job down after a peer
    rank failed (torchrun, ``torch.multiprocessing``) sends SIGTERM first,
    and an asynchronous checkpoint write still in flight must complete
    (:meth:`StreamCheckpointer.flush`) rather than die with the process --
    otherwise the newest checkpoint on disk can be far older than the last
    batch every rank finished."""
    import signal
    if threading.current_thread() is not threading.main_thread():
        return

    def _term(signum, frame):
        raise SystemExit(128 + signum)

    signal.signal(signal.SIGTERM, _term)


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
