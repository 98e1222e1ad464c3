"""Per-session reporting to twtml-web and Lightning (``SessionStats.scala``; C5).

``open()`` creates a 4-series Lightning ``line-streaming`` plot (sizes
1,1,2,2; light-blue / light-yellow / blue / yellow, ``SessionStats.scala:
16-20,49-52``), logs the session and pym URLs and posts ``Config(session,
lightningHost, [vizId])`` to twtml-web (``:60``).  ``update()`` posts
``Stats(count, batch, mse, realStdev, predStdev)`` (Longs, ``:29``) and appends
``[real, pred, realStdev x batch, predStdev x batch]`` to the plot
(``:26-27,31-33``).

Differences, by design (SURVEY §5 failure detection): pushes run on a
background thread through a bounded queue, so a slow or dead server never
stalls training (the reference blocks the output op on each HTTP call, then
drops errors with ``Try``); when the queue is full the oldest update is
dropped.  A Lightning server that is down at ``open()`` is logged instead of
aborting the job unless ``strict=True`` (the reference's behaviour).
``plot_points`` caps the points appended per batch (0 = all, the default,
as the reference; at millions of tweets per batch pass ``--plotPoints 10000``).
"""
from __future__ import annotations

import logging
import queue
import threading
from typing import Callable, List, Optional, Sequence

import numpy as np

from .lightning import Lightning, LightningError, Visualization
from .webclient import WebClient

__all__ = ["SessionStats", "REAL_COLOR_DET", "PRED_COLOR_DET", "REAL_COLOR", "PRED_COLOR"]

log = logging.getLogger("com.giorgioinf.twtml.spark.SessionStats")

REAL_COLOR_DET = [173.0, 216.0, 230.0]   # light blue
REAL_COLOR = [30.0, 144.0, 255.0]        # blue
PRED_COLOR_DET = [238.0, 232.0, 170.0]   # light yellow
PRED_COLOR = [255.0, 215.0, 0.0]         # gold


class SessionStats:
    def __init__(self, lightning: str, twtweb: str, plot_points: int = 0, strict: bool = False,
                 async_push: bool = True, queue_size: int = 64, timeout: float = 5.0):
        self.lightning_host = lightning
        self.twtweb = twtweb
        self.plot_points = int(plot_points)
        self.strict = strict
        self.lgn = Lightning(lightning, timeout=timeout)
        self.web = WebClient.apply(twtweb)
        self.web.timeout = timeout
        self.viz: Optional[Visualization] = None
        self.errors = 0
        self.sent = 0
        self._async = async_push
        self._q: "queue.Queue[Optional[Callable[[], None]]]" = queue.Queue(maxsize=queue_size)
        self._worker: Optional[threading.Thread] = None

    @classmethod
    def from_conf(cls, conf, **kw) -> "SessionStats":
        return cls(conf.lightning, conf.twtweb, plot_points=getattr(conf, "plotPoints", 0), **kw)

    # ------------------------------------------------------------------
    def open(self) -> "SessionStats":
        log.info("Initializing plot on lightning server: %s", self.lightning_host)
        try:
            self.viz = self.lgn.line_streaming(series=[[0.0]] * 4, size=[1.0, 1.0, 2.0, 2.0],
                                               color=[REAL_COLOR_DET, PRED_COLOR_DET, REAL_COLOR,
                                                      PRED_COLOR])
            log.info("lightning server session: \n  %s/sessions/%s\n  %s/visualizations/%s/pym",
                     self.lightning_host, self.lgn.session, self.lightning_host, self.viz.id)
        except LightningError as e:
            if self.strict:
                raise
            log.warning("lightning unavailable, plotting disabled: %s", e)
            self.viz = None
        log.info("Initializing config on web server: %s", self.twtweb)
        if self.viz is not None:
            self._try(lambda: self.web.config(self.lgn.session, self.lgn.host, [self.viz.id]))
        if self._async:
            self._worker = threading.Thread(target=self._run, name="session-stats", daemon=True)
            self._worker.start()
        return self

    def update(self, count: int, batch: int, mse: float, realStdev: float, predStdev: float,
               real: Sequence[float], pred: Sequence[float]) -> None:
        stats = (int(count), int(batch), int(mse), int(realStdev), int(predStdev))
        real = np.array(real, dtype=np.float64)   # a copy: the caller may reuse its buffers
        pred = np.array(pred, dtype=np.float64)

        def push() -> None:
            self._try(lambda: self.web.stats(*stats))
            if self.viz is not None:
                # the JSON series are built here, on the worker, not on the caller's thread
                series = self._series(stats[1], float(realStdev), float(predStdev), real, pred)
                self._try(lambda: self.lgn.line_streaming(series=series, viz=self.viz))

        self._enqueue(push)

    def push_stats(self, count: int, batch: int, mse: float, realStdev: float, predStdev: float) -> None:
        """The twtml-web half of :meth:`update` (``SessionStats.scala:29``):
        posted whether or not the batch's plot sample reaches rank 0."""
        stats = (int(count), int(batch), int(mse), int(realStdev), int(predStdev))
        self._enqueue(lambda: self._try(lambda: self.web.stats(*stats)))

    def append_plot(self, batch: int, realStdev: float, predStdev: float,
                    real: Sequence[float], pred: Sequence[float]) -> None:
        """The Lightning half of :meth:`update` (``SessionStats.scala:31-33``)."""
        if self.viz is None:
            return
        real = np.array(real, dtype=np.float64)
        pred = np.array(pred, dtype=np.float64)

        def push() -> None:
            series = self._series(int(batch), float(realStdev), float(predStdev), real, pred)
            self._try(lambda: self.lgn.line_streaming(series=series, viz=self.viz))

        self._enqueue(push)

    def _enqueue(self, push: Callable[[], None]) -> None:
        if not self._async:
            push()
            return
        try:
            self._q.put_nowait(push)
        except queue.Full:
            try:
                self._q.get_nowait()          # drop the oldest pending update
            except queue.Empty:
                pass
            self._q.put_nowait(push)

    def web_stats_only(self, count: int, batch: int) -> None:
        """``Try(web.stats(count))`` of the k-means job (commented out in the
        reference at ``KMeans.scala:116``; enabled with ``--report``)."""
        job = lambda: self._try(lambda: self.web.stats(int(count), int(batch), 0, 0, 0))  # noqa: E731
        if self._async:
            try:
                self._q.put_nowait(job)
            except queue.Full:
                pass
        else:
            job()

    def _series(self, batch: int, real_sd: float, pred_sd: float, real, pred) -> List[np.ndarray]:
        real = np.asarray(real, dtype=np.float64)
        pred = np.asarray(pred, dtype=np.float64)
        if self.plot_points and real.shape[0] > self.plot_points:
            idx = np.linspace(0, real.shape[0] - 1, self.plot_points).astype(np.int64)
            real, pred = real[idx], pred[idx]
        n = real.shape[0]
        # numpy series: the Lightning client encodes them natively (GIL released)
        return [real, pred, np.full(n, real_sd), np.full(n, pred_sd)]

    def _try(self, fn: Callable[[], object]) -> None:
        try:
            fn()
            self.sent += 1
        except Exception as e:  # best effort: Try(...) in the reference
            self.errors += 1
            log.debug("report push failed: %s", e)

    def _run(self) -> None:
        while True:
            job = self._q.get()
            if job is None:
                return
            job()

    def flush(self, timeout: float = 10.0) -> None:
        """Wait until queued pushes are done (tests / shutdown)."""
        if not self._async or self._worker is None:
            return
        done = threading.Event()
        try:
            self._q.put(done.set, timeout=timeout)
        except queue.Full:
            return
        done.wait(timeout)

    def close(self) -> None:
        if self._worker is not None:
            self.flush()
            self._q.put(None)
            self._worker.join(timeout=5.0)
            self._worker = None
