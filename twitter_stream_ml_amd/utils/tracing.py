"""Trace ranges: roctx markers (visible in rocprofv3 --marker-trace) + wall timers.

``trace_range("featurize")`` pushes a roctx range through torch's
``torch.cuda.nvtx`` binding (routed to roctx on ROCm) when a GPU runtime is
loaded, and always records host wall time into ``TIMERS``.
"""
from __future__ import annotations

import contextlib
import time
from collections import defaultdict
from typing import Dict, List

__all__ = ["trace_range", "TIMERS", "timer_summary"]

TIMERS: Dict[str, List[float]] = defaultdict(list)


def _nvtx():
    try:
        import torch
        if torch.cuda.is_available():
            return torch.cuda.nvtx
    except Exception:
        return None
    return None


@contextlib.contextmanager
def trace_range(name: str, marker: bool = True):
    nv = _nvtx() if marker else None
    if nv is not None:
        nv.range_push(name)
    t0 = time.perf_counter()
    try:
        yield
    finally:
        TIMERS[name].append((time.perf_counter() - t0) * 1e3)
        if nv is not None:
            nv.range_pop()


def timer_summary() -> Dict[str, Dict[str, float]]:
    out = {}
    for k, v in TIMERS.items():
        s = sorted(v)
        out[k] = {"n": len(s), "p50_ms": s[len(s) // 2], "max_ms": s[-1], "sum_ms": sum(s)}
    return out
