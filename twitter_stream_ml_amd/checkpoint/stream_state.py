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
    def __init__(self, checkpoint: str, rank: int, keep: int = 16):
        self.dir = os.path.abspath(checkpoint) + ".stream"
        self.path = os.path.join(self.dir, f"rank-{int(rank)}.json")
        self.keep = int(keep)
        self._h: Optional[Dict[int, int]] = None   # this rank's history (it is the only writer)

    def history(self) -> Dict[int, int]:
        if self._h is not None:
            return dict(self._h)
        try:
            with open(self.path) as fh:
                return {int(k): int(v) for k, v in json.load(fh).items()}
        except (OSError, ValueError):
            return {}

    def record(self, batches: int, records: int) -> None:
        # kept in memory after the first read: with --checkpointInterval 1 this
        # runs on the training thread every batch (one small atomic write, no read)
        h = self.history()
        h[int(batches)] = int(records)
        for k in sorted(h)[:-self.keep]:
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
