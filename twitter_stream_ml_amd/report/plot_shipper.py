"""Lightning plot samples to rank 0, off the training thread.

The reference ``collect``s every batch's real and predicted values to the
driver and appends them to the Lightning plot inside output op #1
(``LinearRegression.scala:76-77``, ``SessionStats.scala:22-34``), best
effort.  Here the device samples ``plotPoints`` (pred, real) pairs per batch
(``sgd.hip`` ``k_plot_sample``), and a shipper thread on every rank takes
them from there: with several ranks it gathers the samples to rank 0 over a
gloo process group of its own (so its collectives never interleave with the
training thread's), and rank 0 hands stats + series to the
:class:`SessionStats` worker, which does the HTTP.  The training thread only
enqueues.

Every rank must submit the same sequence of batches (each submit is one
gather); the queue is bounded and a full queue blocks the producer instead
of dropping, so the gathers stay paired across ranks.  Rank 0's own HTTP
pushes are drop-oldest in :class:`SessionStats`.
"""
from __future__ import annotations

import logging
import queue
import threading
from typing import Optional

import numpy as np

__all__ = ["PlotShipper"]

log = logging.getLogger("twtml.report.plot")


class PlotShipper:
    def __init__(self, session, rank: int = 0, world: int = 1, maxsize: int = 64):
        self.session = session
        self.rank, self.world = int(rank), int(world)
        self.group = None
        if self.world > 1:
            import torch.distributed as dist
            self.group = dist.new_group(backend="gloo")   # collective: every rank creates it
        self._q: "queue.Queue" = queue.Queue(maxsize=maxsize)
        self._err: Optional[BaseException] = None
        self.shipped = 0
        self._th = threading.Thread(target=self._run, name="plot-shipper", daemon=True)
        self._th.start()

    def submit(self, stats, real, pred) -> None:
        """stats: (count, batch, mse, realStdev, predStdev); real / pred: this
        rank's sampled series (copied: the caller may reuse its arrays)."""
        self._q.put((tuple(stats), np.array(real, np.float64), np.array(pred, np.float64)))

    def _run(self) -> None:
        from ..parallel.dist import gather_to_main
        while True:
            item = self._q.get()
            if item is None:
                return
            stats, real, pred = item
            try:
                if self.world > 1:
                    both = gather_to_main(np.stack([real, pred]).T.reshape(-1), group=self.group)
                    if both is not None:
                        both = both.reshape(-1, 2)
                        real, pred = both[:, 0], both[:, 1]
                if self.rank == 0 and self.session is not None:
                    self.session.update(*stats, real, pred)
                self.shipped += 1
            except BaseException as e:   # noqa: BLE001 -- best effort, like the reference's Try
                self._err = e
                log.warning("plot shipping failed: %s", e)

    def close(self, timeout: float = 60.0) -> None:
        if self._th.is_alive():
            self._q.put(None)
            self._th.join(timeout)
