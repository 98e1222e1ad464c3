"""HBM-sized micro-batches (BASELINE config 5: "288 GB HBM micro-batch sizing").

An engine's device footprint is affine in its row capacity: a part that does
not depend on the batch (fp64 master weights, F-sized flag / slot maps, the
LDS-tier and partial-row buffers) plus per-row staging (raw text slots with
their decode tails, the prepared-batch entry streams, tier lists).  Rather
than restating every allocation here, :func:`engine_footprint` builds two
probe engines and reads the bytes they allocate
(``_twtml_hip.device_bytes_allocated``) plus what an LR engine allocates on
its first tiered batch (``lazy_bytes``: the entry-sized far lists and CSC of
both prepared buffers, ~48 B per text unit of capacity), and
:func:`hbm_max_rows` solves for the largest capacity that fits a fraction of
the GPU's free memory.  The remaining headroom covers the buffers that grow
with a batch's active set (compact weights, slot-sized tier arrays: ~100 B
per active feature).
"""
from __future__ import annotations

import gc
from typing import Callable, Tuple

__all__ = ["engine_footprint", "footprint_model", "hbm_max_rows"]


def _allocated() -> int:
    from ._native import hip
    return int(hip().device_bytes_allocated())


def engine_footprint(make_engine: Callable[[int], object], rows: int) -> int:
    """Device bytes one engine of ``rows`` capacity allocates at construction."""
    before = _allocated()
    eng = make_engine(int(rows))
    used = _allocated() - before
    inner = getattr(eng, "_eng", eng)
    used += int(getattr(inner, "lazy_bytes", 0) or 0)   # allocated by the first tiered batch
    del eng
    gc.collect()   # engine wrappers hold reference cycles: free the probe now
    return used


def footprint_model(make_engine: Callable[[int], object], probe: Tuple[int, int] = (65536, 262144)) -> Tuple[float, float]:
    """(fixed bytes, bytes per row) from two probe engines."""
    r1, r2 = int(probe[0]), int(probe[1])
    a1, a2 = engine_footprint(make_engine, r1), engine_footprint(make_engine, r2)
    per_row = max(0.0, (a2 - a1) / float(r2 - r1))
    return float(a1) - per_row * r1, per_row


def hbm_max_rows(make_engine: Callable[[int], object], free_bytes: int, fraction: float = 0.8,
                 probe: Tuple[int, int] = (65536, 262144), quantum: int = 65536) -> int:
    """Largest row capacity (a multiple of ``quantum``) whose engine fits in
    ``fraction`` of ``free_bytes``."""
    fixed, per_row = footprint_model(make_engine, probe)
    if per_row <= 0.0:
        raise RuntimeError("engine footprint does not grow with its row capacity")
    rows = int((float(free_bytes) * float(fraction) - fixed) / per_row)
    return max(quantum, rows // quantum * quantum)
