"""Ingest || compute pipelining over an engine's device raw slots.

The reference overlaps ingest with compute by running the Twitter receiver on
its own core while the JobScheduler trains the previous batch (SURVEY §2.4,
U13/U14).  Here a sealed micro-batch that is still queued behind the one being
trained is staged into a pinned host buffer (wire format) and its H2D is
enqueued on the engine's copy stream (``RawSlots::submit``), so by the time
the executor reaches it the bytes are already resident.

Slot protocol: a slot is *in flight* from ``submit`` until ``process`` of that
slot returns (``process`` blocks on the compute stream, which waited for the
slot's H2D).  A slot's pinned staging buffer is only rewritten when the slot
is not in flight, so a host write never races a DMA read.  At most
``n_slots - 1`` batches are prefetched, leaving one slot for a batch that
arrives without a prefetch.
"""
from __future__ import annotations

from typing import Callable, Dict, List, Tuple

__all__ = ["SlotPipeline"]


class SlotPipeline:
    def __init__(self, n_slots: int, stage: Callable[[int, object], object],
                 submit: Callable[[object, int], None], sync: Callable[[], None]):
        if n_slots < 1:
            raise ValueError("n_slots must be >= 1")
        self.n_slots = int(n_slots)
        self._stage = stage        # (slot, raw) -> HostBatchView holding raw
        self._submit = submit      # (host batch view, slot) -> async H2D
        self._sync = sync          # wait for the engine's copy + compute streams
        self._inflight: Dict[int, Tuple[object, int]] = {}   # id(raw) -> (raw, slot)
        self._rr = 0
        self.prefetched = 0        # batches whose H2D was issued ahead of time
        self.hits = 0              # ... and later consumed by take()

    def _free_slot(self) -> int:
        busy = {s for _, s in self._inflight.values()}
        for k in range(self.n_slots):
            s = (self._rr + k) % self.n_slots
            if s not in busy:
                self._rr = (s + 1) % self.n_slots
                return s
        raise RuntimeError("no free raw slot")

    def prefetch(self, raw) -> bool:
        """Stage + async H2D of a batch that will be trained later."""
        if id(raw) in self._inflight:
            return True
        if len(self._inflight) >= self.n_slots - 1:
            return False
        slot = self._free_slot()
        self._submit(self._stage(slot, raw), slot)
        self._inflight[id(raw)] = (raw, slot)
        self.prefetched += 1
        return True

    def take(self, raw) -> int:
        """Slot holding ``raw`` (staged and submitted now if not prefetched).

        The caller must ``process`` the returned slot before the next take."""
        hit = self._inflight.pop(id(raw), None)
        if hit is not None:
            self.hits += 1
            return hit[1]
        if len(self._inflight) >= self.n_slots:   # cannot happen with the prefetch cap
            raise RuntimeError("all raw slots in flight")
        slot = self._free_slot()
        self._submit(self._stage(slot, raw), slot)
        return slot

    def pending(self) -> List[object]:
        return [r for r, _ in self._inflight.values()]

    def drop(self) -> None:
        """Forget prefetched batches (after their H2Ds finished, so the
        staging buffers can be rewritten)."""
        if self._inflight:
            self._sync()
        self._inflight.clear()
