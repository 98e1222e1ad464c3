"""Per-batch metrics as JSON lines (SURVEY §5 metrics row).

One record per micro-batch: batch time, tweets seen/trained, GD iterations,
convergence, MSE/stdevs, device prep/train milliseconds, scheduling delay and
end-to-end latency -- what the reference only exposed through the Spark UI.
"""
from __future__ import annotations

import json
import threading
import time
from typing import Any, Dict, Optional

__all__ = ["MetricsLogger"]


class MetricsLogger:
    def __init__(self, path: Optional[str] = None):
        self.path = path
        self._fh = open(path, "a", encoding="utf-8") if path else None
        self._lock = threading.Lock()
        self.records = []

    def log(self, **rec: Any) -> Dict[str, Any]:
        rec.setdefault("ts", time.time())
        self.records.append(rec)
        if self._fh is not None:
            with self._lock:
                self._fh.write(json.dumps(rec, default=float) + "\n")
                self._fh.flush()
        return rec

    def close(self) -> None:
        if self._fh is not None:
            self._fh.close()
            self._fh = None
