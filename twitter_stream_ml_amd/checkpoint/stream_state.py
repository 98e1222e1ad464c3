"""Per-rank stream positions for exact resume after a failure.

The reference keeps no checkpoint at all (the model lives in
driver memory, ``ssc.checkpoint`` is never called).  Here rank 0 saves the
model every ``--checkpointInterval`` batches with ``streaming/progress.json =
{"batches": t}``, and *every* rank records how many source records it had
consumed after each batch in ``<checkpoint>.stream/rank-<r>.json`` (a short
history, written atomically before the model).  On restart each rank looks up
its position for the model's batch count and resumes its source there, so a
job killed mid-stream and restarted (e.g. ``torchrun --max-restarts``) ends
with the same model as an uninterrupted run.
"""
from __future__ import annotations

import json
import os
import tempfile
from typing import Dict, Optional, Tuple

__all__ = ["StreamPositions", "resolve_resume"]


class StreamPositions:
    """This rank's ``{batches: records consumed}`` history.

    Pruning never drops a position a resume can still ask for: every entry at
    or above the oldest batch count of a model on disk (``<checkpoint>`` and a
    ``<checkpoint>.old`` left by an interrupted replacement) is kept, plus the
    newest ``keep`` entries.  A write still in flight is newer than the models
    on disk, so its position survives too, however many batches the write
    spans (with ``--checkpointInterval 1`` one asynchronous write
    covers dozens of batches)."""

    def __init__(self, checkpoint: str, rank: int, keep: int = 16):
        self.checkpoint = os.path.abspath(checkpoint)
        self.dir = self.checkpoint + ".stream"
        self.path = os.path.join(self.dir, f"rank-{int(rank)}.json")
        self.keep = int(keep)
        self._h: Optional[Dict[int, int]] = None   # this rank's history (it is the only writer)
        self._floor_key = None
        self._floor = 0

    def disk_floor(self) -> int:
        """Oldest batch count of a model on disk (0 if none): positions at or
        above it must be kept.  Cached on the progress files' mtimes, so the
        per-batch cost is two ``stat`` calls."""
        keys, found = [], []
        for d in (self.checkpoint, self.checkpoint + ".old"):
            p = os.path.join(d, "streaming", "progress.json")
            try:
                st = os.stat(p)
            except OSError:
                keys.append(None)
                continue
            keys.append((st.st_mtime_ns, st.st_ino))
            found.append(p)
        key = tuple(keys)
        if key == self._floor_key:
            return self._floor
        vals = []
        for p in found:
            try:
                with open(p) as fh:
                    vals.append(int(json.load(fh).get("batches", 0)))
            except (OSError, ValueError):
                # replaced between the stat and the open: keep everything this time
                return 0
        self._floor_key, self._floor = key, (min(vals) if vals else 0)
        return self._floor

    def history(self) -> Dict[int, int]:
        if self._h is not None:
            return dict(self._h)
        try:
            with open(self.path) as fh:
                return {int(k): int(v) for k, v in json.load(fh).items()}
        except (OSError, ValueError):
            return {}

    def record(self, batches: int, records: int, floor: Optional[int] = None) -> None:
        """Record this rank's position after ``batches``.  ``floor``: the
        oldest batch count a resume may still need (default: from the models
        on disk, :meth:`disk_floor`)."""
        # kept in memory after the first read: with --checkpointInterval 1 this
        # runs on the training thread every batch (one small atomic write, no read)
        h = self.history()
        h[int(batches)] = int(records)
        lo = self.disk_floor() if floor is None else int(floor)
        for k in sorted(h)[:-self.keep]:
            if k < lo:
                del h[k]
        # hard cap: with no model readable on this rank's
        # filesystem the floor stays 0 and nothing above prunes; keep the
        # newest keep * 64 positions even then, so the file (rewritten on the
        # training thread) cannot grow for the whole run
        cap = self.keep * 64
        if len(h) > cap:
            for k in sorted(h)[:-cap]:
                del h[k]
        os.makedirs(self.dir, exist_ok=True)
        fd, tmp = tempfile.mkstemp(prefix=".pos-", dir=self.dir)
        with os.fdopen(fd, "w") as fh:
            json.dump({str(k): v for k, v in sorted(h.items())}, fh)
        os.replace(tmp, self.path)
        self._h = h

    def records_at(self, batches: int) -> Optional[int]:
        return self.history().get(int(batches))


def resolve_resume(resume: str, checkpoint: str) -> Optional[str]:
    """``--resume auto`` -> the checkpoint path if a model exists there."""
    if not resume:
        return None
    if resume == "auto":
        if checkpoint and os.path.isdir(os.path.join(checkpoint, "metadata")):
            return checkpoint
        # a crash between the two renames of a checkpoint replacement leaves
        # the previous model at <checkpoint>.old (saveable._write_dir)
        old = os.path.abspath(checkpoint) + ".old" if checkpoint else ""
        if old and os.path.isdir(os.path.join(old, "metadata")):
            return old
        return None
    return resume


def progress_of(path: str) -> Tuple[int, Optional[dict]]:
    from .saveable import load_progress
    p = load_progress(path)
    return (int(p.get("batches", 0)) if p else 0), p
