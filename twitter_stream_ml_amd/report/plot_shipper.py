"""Lightning plot samples to rank 0, off the training thread.

The reference ``collect``s every batch's real and predicted values to the
driver and appends them to the Lightning plot inside output op #1
(``LinearRegression.scala:76-77``, ``SessionStats.scala:22-34``), best
effort.  Here the device samples ``plotPoints`` (pred, real) pairs per batch
(``sgd.hip`` ``k_plot_sample``), and a shipper thread on every rank takes
them from there: with several ranks it gathers the samples to rank 0 over a
gloo process group of its own (so its collectives never interleave with the
training thread's), and rank 0 hands the series to the :class:`SessionStats`
worker, which does the HTTP.  The batch's twtml-web ``Stats`` do not wait for
the gather: rank 0's training thread posts them itself (async, drop-oldest).

Back-pressure never reaches training (``SessionStats.scala:29-33``: best
effort).  :meth:`submit` never blocks: it appends a (sequence number,
sample) entry; when more than ``maxsize`` samples wait, the oldest waiting
sample is dropped but its sequence number stays queued.  The shipper gathers
every sequence number in order on every rank -- a dropped sample travels as
an empty "dropped" record -- so the gathers stay paired across ranks
whatever each rank dropped, and a stalled gather only makes the backlog of
tiny markers grow.  Every gather carries its sequence number and rank 0
checks them: a batch whose sample some rank dropped is not plotted (the same
batch is then missing on every rank's side of the plot, not half of it), and
a sequence mismatch or a gather error stops the shipping for good (pairs
could no longer be trusted) instead of plotting mismatched pairs.
"""
from __future__ import annotations

import collections
import datetime
import logging
import threading
from typing import Optional

import numpy as np

__all__ = ["PlotShipper"]

log = logging.getLogger("twtml.report.plot")


class PlotShipper:
    def __init__(self, session, rank: int = 0, world: int = 1, maxsize: int = 64,
                 gather_timeout_s: float = 60.0, max_bytes: int = 64 << 20):
        self.session = session
        self.rank, self.world = int(rank), int(world)
        self.maxsize = max(1, int(maxsize))
        # the backlog is also bounded in bytes: with --plotPoints 0 a waiting
        # sample holds every kept row (16 B per row as two fp64 series)
        self.max_bytes = max(1, int(max_bytes))
        self._bytes = 0
        self.group = None
        if self.world > 1:
            import torch.distributed as dist
            # collective: every rank creates it; the timeout bounds a gather
            # stuck on a dead peer
            self.group = dist.new_group(backend="gloo",
                                        timeout=datetime.timedelta(seconds=gather_timeout_s))
        self._cv = threading.Condition()
        self._items: "collections.deque" = collections.deque()   # [seq, stats, real, pred] / None
        self._waiting = 0          # entries that still hold their sample
        self._seq = 0
        self._err: Optional[BaseException] = None
        self.shipped = 0           # batches plotted (rank 0) / gathered (other ranks)
        self.dropped = 0           # this rank's samples dropped on a full backlog
        self.skipped = 0           # rank 0: batches not plotted because some rank dropped its sample
        self.stopped = False       # a gather failed or paired different batches: shipping ended
        self._th = threading.Thread(target=self._run, name="plot-shipper", daemon=True)
        self._th.start()

    def submit(self, stats, real, pred) -> None:
        """stats: (count, batch, mse, realStdev, predStdev); real / pred: this
        rank's sampled series (copied: the caller may reuse its arrays).
        Never blocks."""
        with self._cv:
            if self.stopped:
                return
            r, p = np.array(real, np.float64), np.array(pred, np.float64)
            self._items.append([self._seq, tuple(stats), r, p])
            self._seq += 1
            self._waiting += 1
            self._bytes += r.nbytes + p.nbytes
            # drop the oldest waiting samples (keep their markers) beyond either bound;
            # the newest sample always stays
            while self._waiting > 1 and (self._waiting > self.maxsize or self._bytes > self.max_bytes):
                for it in self._items:
                    if it is not None and it[2] is not None:
                        self._bytes -= it[2].nbytes + it[3].nbytes
                        it[2] = it[3] = None
                        self._waiting -= 1
                        self.dropped += 1
                        break
            self._cv.notify()

    def backlog(self) -> int:
        with self._cv:
            return len(self._items)

    def _next(self):
        with self._cv:
            while not self._items:
                self._cv.wait()
            it = self._items.popleft()
            if it is not None and it[2] is not None:
                self._waiting -= 1
                self._bytes -= it[2].nbytes + it[3].nbytes
            return it

    def _stop(self, why: str) -> None:
        with self._cv:
            self.stopped = True
            self._items.clear()
            self._waiting = 0
            self._bytes = 0
        log.warning("plot shipping stopped: %s", why)

    def _run(self) -> None:
        from ..parallel.dist import gather_parts
        while True:
            it = self._next()
            if it is None:
                return
            seq, stats, real, pred = it
            ok = real is not None
            try:
                if self.world > 1:
                    head = np.array([float(seq), 1.0 if ok else 0.0])
                    body = np.stack([real, pred]).T.reshape(-1) if ok else np.zeros(0)
                    parts = gather_parts(np.concatenate([head, body]), group=self.group)
                    if parts is not None:   # rank 0
                        seqs = [int(p[0]) for p in parts]
                        if any(s != seq for s in seqs):
                            self._stop(f"gather paired batches {seqs} (expected {seq})")
                            return
                        ok = all(p[1] == 1.0 for p in parts)
                        if ok:
                            both = np.concatenate([p[2:] for p in parts]).reshape(-1, 2)
                            real, pred = both[:, 0], both[:, 1]
                if self.rank == 0 and self.session is not None:
                    if ok:
                        _, batch, _, real_sd, pred_sd = stats
                        self.session.append_plot(batch, real_sd, pred_sd, real, pred)
                    else:
                        self.skipped += 1
                self.shipped += 1
            except BaseException as e:   # noqa: BLE001 -- best effort, like the reference's Try
                self._err = e
                self._stop(f"gather failed: {e}")
                return

    def close(self, timeout: float = 60.0) -> None:
        if self._th.is_alive():
            with self._cv:
                self._items.append(None)
                self._cv.notify()
            # a shipper that already failed has exited; a healthy one drains
            self._th.join(0.0 if self.stopped else timeout)
