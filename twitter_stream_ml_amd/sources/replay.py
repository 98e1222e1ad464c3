"""Replay source: tweets from a JSON-lines file (one Twitter-API status per line).

Stands in for a recorded sample stream (SURVEY §7.1 ``sources/``): each line
is parsed with :func:`status_from_json` (v1.1 field names; ``created_at_ms`` or
``created_at``).  ``rate`` paces the replay (tweets/s, 0 = as fast as asked);
``loop`` restarts at the end of the file.  Data-parallel ranks read disjoint
records (``shard``/``num_shards``: every ``num_shards``-th line), and
``skip`` resumes after records already consumed.
"""
from __future__ import annotations

import json
import time
from typing import List, Optional

from ..records.batch import RawBatch
from ..records.schema import Status, status_from_json

__all__ = ["JsonlReplaySource", "write_jsonl"]


class JsonlReplaySource:
    def __init__(self, path: str, rate: float = 0.0, loop: bool = False, skip: int = 0,
                 shard: int = 0, num_shards: int = 1):
        self.shard, self.num_shards = int(shard), max(1, int(num_shards))
        self._line = 0
        self.path = path
        self.rate = float(rate)
        self.loop = loop
        self._fh = open(path, "r", encoding="utf-8")
        self._t0 = time.monotonic()
        self._emitted = 0
        self.exhausted = False
        for _ in range(int(skip)):          # resume: records already consumed
            if self._next_line() is None:
                break

    def _next_line(self) -> Optional[str]:
        while True:
            line = self._fh.readline()
            if line:
                if line.strip():
                    mine = self._line % self.num_shards == self.shard   # DP: rank r takes every
                    self._line += 1                                     # world-th record
                    if mine:
                        return line
                continue
            if not self.loop:
                self.exhausted = True
                return None
            self._fh.seek(0)
            self._line = 0

    def poll(self, max_n: int, now_ms: Optional[int] = None) -> RawBatch:
        n = int(max_n)
        if self.rate > 0:
            n = min(n, max(0, int((time.monotonic() - self._t0) * self.rate) - self._emitted))
        out: List[Status] = []
        for _ in range(n):
            line = self._next_line()
            if line is None:
                break
            out.append(status_from_json(json.loads(line)))
        self._emitted += len(out)
        return RawBatch.from_statuses(out, batch_time_ms=int(now_ms or time.time() * 1000))

    def close(self) -> None:
        self._fh.close()


def write_jsonl(path: str, statuses) -> None:
    from ..records.schema import status_to_json
    with open(path, "w", encoding="utf-8") as fh:
        for s in statuses:
            fh.write(json.dumps(status_to_json(s), ensure_ascii=False) + "\n")
