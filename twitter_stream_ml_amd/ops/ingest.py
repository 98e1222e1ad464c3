"""Ingest || compute pipelining over an engine's device raw slots.

The reference overlaps ingest with compute by running the Twitter receiver on
its own core while the JobScheduler trains the previous batch (SURVEY §2.4,
U13/U14).  Here a sealed micro-batch that is still queued behind the one being
trained is staged into a pinned host buffer (wire format) and its H2D is
enqueued on the engine's copy stream (``RawSlots::submit``), so by the time
the executor reaches it the bytes are already resident.

Slot protocol: a slot is *in flight* from ``submit`` until ``process`` of that
slot returns (``process`` blocks on the compute stream, which waited for the
slot's H2D), or until the engine ``discard``\\ s it.  A slot's pinned staging
buffer is only rewritten when the slot is not in flight, so a host write
never races a DMA read.  At most ``n_slots - 1`` batches are prefetched,
leaving one slot for a batch that arrives without a prefetch.

Matching: a prefetched batch is found again by its *content key* -- seal time,
row count and the addresses of its offset / text buffers -- not by the Python
object: ``RawBatch.with_time`` copies share the arrays, so a driver that
prefetches one copy and trains another still hits.  Batches are trained in
prefetch order; entries prefetched before the batch a ``take`` matches were
skipped and can never be trained in order: they are *orphans*, discarded on
the engine (``LREngine::discard``: out of the prepare-ahead queue, H2D
waited for) and counted, so no slot is ever stranded (round 5: orphans kept
``raw_slots - 1`` slots pinned for the rest of a run).
"""
from __future__ import annotations

from collections import OrderedDict
from typing import Callable, Hashable, List, Optional, Tuple

__all__ = ["SlotPipeline", "batch_key"]


def batch_key(raw) -> Hashable:
    """Content key of a raw batch: equal for ``with_time``-style copies that
    share the arrays and carry the same seal time."""
    offsets = getattr(raw, "offsets", None)
    if offsets is None or not hasattr(offsets, "ctypes"):
        return ("obj", id(raw))
    u8 = getattr(raw, "utf8", None)
    text = u8.data if u8 is not None else getattr(raw, "text", None)
    tptr = int(text.ctypes.data) if text is not None and getattr(text, "size", 0) else 0
    return ("batch", int(getattr(raw, "batch_time_ms", 0)), int(offsets.shape[0]), int(offsets.ctypes.data), tptr)


class SlotPipeline:
    def __init__(self, n_slots: int, stage: Callable[[int, object], object],
                 submit: Callable[[object, int], None], sync: Callable[[], None],
                 discard: Optional[Callable[[int], None]] = None):
        if n_slots < 1:
            raise ValueError("n_slots must be >= 1")
        self.n_slots = int(n_slots)
        self._stage = stage        # (slot, raw) -> HostBatchView holding raw
        self._submit = submit      # (host batch view, slot) -> async H2D
        self._sync = sync          # wait for the engine's copy + compute streams
        self._discard = discard    # slot -> engine forgets a submitted batch (H2D waited for)
        # key -> (raw, slot), in prefetch order (the raw keeps its buffers alive)
        self._inflight: "OrderedDict[Hashable, Tuple[object, int]]" = OrderedDict()
        self._rr = 0
        self.prefetched = 0        # batches whose H2D was issued ahead of time
        self.hits = 0              # ... and later consumed by take()
        self.orphaned = 0          # ... and skipped by the trained sequence (discarded)

    def _free_slot(self) -> int:
        busy = {s for _, s in self._inflight.values()}
        for k in range(self.n_slots):
            s = (self._rr + k) % self.n_slots
            if s not in busy:
                self._rr = (s + 1) % self.n_slots
                return s
        raise RuntimeError("no free raw slot")

    def _release(self, key: Hashable) -> None:
        _, slot = self._inflight.pop(key)
        if self._discard is not None:
            self._discard(slot)
        else:   # no engine hook: wait for every stream before the staging buffer is reused
            self._sync()
        self.orphaned += 1

    def prefetch(self, raw) -> bool:
        """Stage + async H2D of a batch that will be trained later."""
        key = batch_key(raw)
        if key in self._inflight:
            return True
        if len(self._inflight) >= self.n_slots - 1:
            return False
        slot = self._free_slot()
        self._submit(self._stage(slot, raw), slot)
        self._inflight[key] = (raw, slot)
        self.prefetched += 1
        return True

    def take(self, raw) -> int:
        """Slot holding ``raw`` (staged and submitted now if not prefetched).

        The caller must ``process`` the returned slot before the next take."""
        key = batch_key(raw)
        if key in self._inflight:
            for k in list(self._inflight):   # prefetched before raw, never trained: orphans
                if k == key:
                    break
                self._release(k)
            self.hits += 1
            return self._inflight.pop(key)[1]
        if len(self._inflight) >= self.n_slots:   # cannot happen with the prefetch cap
            raise RuntimeError("all raw slots in flight")
        slot = self._free_slot()
        self._submit(self._stage(slot, raw), slot)
        return slot

    def pending(self) -> List[object]:
        return [r for r, _ in self._inflight.values()]

    @property
    def in_flight(self) -> int:
        """Prefetched batches not yet taken (slots they hold)."""
        return len(self._inflight)

    def drop(self) -> None:
        """Forget every prefetched batch (discarded on the engine, so their
        staging buffers can be rewritten)."""
        if self._inflight and self._discard is None:
            self._sync()
            self.orphaned += len(self._inflight)
            self._inflight.clear()
            return
        for k in list(self._inflight):
            self._release(k)
