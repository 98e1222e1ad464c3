"""Bound how long a background Python thread can keep the training thread
waiting for the GIL.

The drivers run report / plot / checkpoint / metrics work on Python threads
next to the training thread.  CPython hands the GIL to a waiting thread only
when the holder blocks or after ``sys.getswitchinterval()`` (5 ms by default),
so one CPU-bound slice of a background thread (an HTTP request being built,
a JSON body, a numpy copy) can stall the training thread by a whole interval
between two engine calls.  Measured on MI355X with a live Lightning plot at
1M tweets/batch (``tools/diag/plot_stall.py``): per-batch p99 8.45 ms at the
default 5 ms interval vs 3.89 ms with plotting off, 3.98 ms at 500 us.

The other source of such stalls is the cyclic garbage collector: a full
(generation-2) collection walks every tracked object -- with torch and the
engine loaded, ~10 ms -- holding the GIL in whatever thread tripped it, and
the report threads' allocations trip it mid-stream.  ``quiet_gc`` collects
once before streaming and freezes what is alive then (the modules, the
engine, the configuration), so later collections only walk what the stream
itself allocates.
"""
from __future__ import annotations

import contextlib
import gc
import sys

__all__ = ["short_gil_slices", "quiet_gc", "streaming_latency"]


@contextlib.contextmanager
def short_gil_slices(us: float = 500.0):
    """Within the block the switch interval is at most ``us`` microseconds
    (restored after: the drivers also run in-process under tests)."""
    old = sys.getswitchinterval()
    sys.setswitchinterval(min(old, us * 1e-6))
    try:
        yield
    finally:
        sys.setswitchinterval(old)


@contextlib.contextmanager
def quiet_gc():
    """Collect, then move every live object to the permanent generation for
    the block (unfrozen after)."""
    gc.collect()
    gc.freeze()
    try:
        yield
    finally:
        gc.unfreeze()


@contextlib.contextmanager
def streaming_latency(us: float = 500.0):
    """Both of the above: what the drivers wrap their streaming loop in."""
    with quiet_gc(), short_gil_slices(us):
        yield
