"""Micro-batch streaming runtime (the slice of Spark Streaming the jobs use).

Semantics kept from Spark Streaming 1.6:

* a receiver thread continuously pulls records from the source into a buffer
  (``TwitterInputDStream``; the reference dedicates a core to it);
* a job generator seals the buffer every ``batch_seconds`` (``StreamingContext
  (sc, Seconds(n))``) — or, as an extension, as soon as ``batch_size`` records
  are buffered — into one micro-batch;
* the registered output operations run **sequentially in registration order**
  for each batch (``spark.streaming.concurrentJobs = 1``), so
  ``foreachRDD(predict+stats)`` registered before ``model.trainOn(stream)``
  sees the model of batch t-1 and training then consumes batch t
  (prequential test-then-train, ``LinearRegression.scala:53-86``);
* ingest overlaps compute: before a batch's output ops run, the sealed
  batches queued behind it are handed to the registered prefetch hooks
  (``add_prefetch``; a device engine stages them and starts their H2D on a
  side stream), the receiver-on-its-own-core overlap of the reference;
* batches that take longer than the interval queue up (scheduling delay);
  with ``max_pending`` the receiver stops pulling while that many sealed
  batches wait (backpressure, ``spark.streaming.backpressure.enabled``).

Size-sealed batches (``batch_size > 0``, ``batch_seconds <= 0``) contain
exactly ``batch_size`` records in source order, so a stream position is just
"records consumed" (``records_done``) -- what checkpoints store for an exact
resume after a failure.

``DStream`` transformations (``filter``/``map``/``cache``) are lazy per batch;
an output operation receives an :class:`RDD`.  ``run_batches`` drives the same
pipeline synchronously (tests, benchmarks, replay), without threads.
"""
from __future__ import annotations

import logging
import queue
import threading
import time
from dataclasses import dataclass, field
from typing import Any, Callable, List, Optional

from ..records.batch import RawBatch
from .clock import SystemClock
from .rdd import RDD

__all__ = ["StreamingContext", "DStream", "ReceiverDStream", "Accumulator", "BatchInfo",
           "Seconds"]

log = logging.getLogger("twtml.streaming")


def Seconds(n: float) -> float:  # noqa: N802 (Spark spelling)
    return float(n)


class Accumulator:
    """Driver-side named counter (``sc.accumulator(0L, "count")``)."""

    def __init__(self, value: Any = 0, name: str = ""):
        self.value = value
        self.name = name
        self._lock = threading.Lock()

    def add(self, v: Any) -> None:
        with self._lock:
            self.value += v

    def __iadd__(self, v: Any) -> "Accumulator":
        self.add(v)
        return self


@dataclass
class BatchInfo:
    batch_time_ms: int
    num_records: int
    submission_s: float
    processing_start_s: float = 0.0
    processing_end_s: float = 0.0

    @property
    def scheduling_delay_ms(self) -> float:
        return (self.processing_start_s - self.submission_s) * 1e3

    @property
    def processing_ms(self) -> float:
        return (self.processing_end_s - self.processing_start_s) * 1e3

    @property
    def total_delay_ms(self) -> float:
        return (self.processing_end_s - self.submission_s) * 1e3


class DStream:
    def __init__(self, ssc: "StreamingContext", parent: Optional["DStream"] = None,
                 op: Optional[Callable[[RDD], RDD]] = None):
        self.ssc = ssc
        self.parent = parent
        self._op = op
        self._cached = False
        self._memo: Optional[tuple] = None

    def compute(self, batch: RawBatch) -> RDD:
        if self._memo is not None and self._memo[0] is batch:
            return self._memo[1]
        rdd = self.parent.compute(batch) if self.parent is not None else RDD([], raw=batch)
        if self._op is not None:
            rdd = self._op(rdd)
        if self._cached:
            rdd = rdd.cache()
            self._memo = (batch, rdd)
        return rdd

    # transformations
    def filter(self, f: Callable[[Any], bool]) -> "DStream":
        return DStream(self.ssc, self, lambda r: r.filter(f))

    def map(self, f: Callable[[Any], Any]) -> "DStream":
        return DStream(self.ssc, self, lambda r: r.map(f))

    def flatMap(self, f: Callable[[Any], Any]) -> "DStream":
        return DStream(self.ssc, self, lambda r: r.flatMap(f))

    def transform(self, f: Callable[[RDD], RDD]) -> "DStream":
        return DStream(self.ssc, self, f)

    def cache(self) -> "DStream":
        self._cached = True
        return self

    persist = cache

    # output operations
    def foreachRDD(self, fn: Callable[..., Any]) -> None:
        import inspect
        try:
            two = len(inspect.signature(fn).parameters) >= 2
        except (TypeError, ValueError):
            two = False
        self.ssc._register(self, fn, two)

    def count(self) -> "DStream":
        return DStream(self.ssc, self, lambda r: RDD([r.count()]))

    def print(self, n: int = 10) -> None:  # noqa: A003 (Spark name)
        def show(rdd, t):
            print(f"-------------------------------------------\nTime: {t} ms\n"
                  "-------------------------------------------")
            for x in rdd.take(n):
                print(x)
        self.foreachRDD(show)


class ReceiverDStream(DStream):
    """Input stream of a receiver-based source; batches are :class:`RawBatch`."""

    def __init__(self, ssc: "StreamingContext", source):
        super().__init__(ssc)
        self.source = source

    def compute(self, batch: RawBatch) -> RDD:
        return RDD(lambda: batch.to_statuses(), raw=batch)


class StreamingContext:
    """Micro-batch scheduler (Spark's StreamingContext + JobScheduler).

    ``max_batch_rows`` / ``max_batch_units``: capacity of the engine's
    staging buffers.  A time-sealed batch that would outgrow them is sealed
    early (the rest of the interval's records start the next batch) instead
    of failing the job; Spark has no such limit because its batches live in
    executor memory.
    """

    def __init__(self, batch_seconds: float = 5.0, batch_size: int = 0, num_batches: int = 0,
                 app_name: str = "", poll_chunk: int = 4096, max_pending: int = 8,
                 max_batch_rows: int = 0, max_batch_units: int = 0, clock=None):
        if batch_seconds <= 0 and batch_size <= 0:
            raise ValueError("need batch_seconds > 0 or batch_size > 0")
        self.batch_seconds = float(batch_seconds)
        self.batch_size = int(batch_size)
        self.num_batches = int(num_batches)
        self.app_name = app_name
        self.poll_chunk = poll_chunk
        self.max_pending = int(max_pending)
        self.max_batch_rows = int(max_batch_rows)
        self.max_batch_units = int(max_batch_units)
        self.clock = clock or SystemClock()   # batch times (runtime/clock.py)
        if self.batch_size > 0 and self.max_batch_rows > 0 and self.batch_size > self.max_batch_rows:
            raise ValueError(f"batch_size {self.batch_size} exceeds the engine capacity {self.max_batch_rows}")
        self._buffered_units = 0
        self.capacity_seals = 0          # batches sealed early at the capacity limit
        self.records_done = 0            # records of all processed batches (stream position)
        self._outputs: List[tuple] = []
        self._inputs: List[ReceiverDStream] = []
        self._buffer: List[RawBatch] = []
        self._buffered = 0
        self._lock = threading.Lock()
        self._jobs: "queue.Queue[Optional[tuple]]" = queue.Queue()
        self._stop = threading.Event()
        self._done = threading.Event()
        self._threads: List[threading.Thread] = []
        self.batches_done = 0
        self._sealed = 0
        self.batch_infos: List[BatchInfo] = []
        self.error: Optional[BaseException] = None
        self.on_batch_completed: List[Callable[[BatchInfo], None]] = []
        self._prefetch: List[Callable[[RawBatch], Any]] = []
        self.prefetch_depth = 2

    # ---- graph construction --------------------------------------------------
    def receiverStream(self, source) -> ReceiverDStream:
        s = ReceiverDStream(self, source)
        self._inputs.append(s)
        return s

    twitterStream = receiverStream

    def accumulator(self, value: Any = 0, name: str = "") -> Accumulator:
        return Accumulator(value, name)

    def _register(self, stream: DStream, fn: Callable[..., Any], with_time: bool) -> None:
        self._outputs.append((stream, fn, with_time))

    def add_prefetch(self, fn: Callable[[RawBatch], Any]) -> None:
        """Register ``fn(batch)``, called for sealed batches still queued behind
        the one about to run (at most ``prefetch_depth``, oldest first; a batch
        may be offered more than once, hooks must be idempotent)."""
        self._prefetch.append(fn)

    def _prefetch_upcoming(self) -> None:
        if not self._prefetch or self.prefetch_depth <= 0:
            return
        with self._jobs.mutex:
            upcoming = [it[0] for it in list(self._jobs.queue)[:self.prefetch_depth] if it is not None]
        for b in upcoming:
            for fn in self._prefetch:
                fn(b)

    # ---- execution -----------------------------------------------------------
    def run_batch(self, batch: RawBatch, info: Optional[BatchInfo] = None) -> BatchInfo:
        info = info or BatchInfo(batch.batch_time_ms, batch.n, time.monotonic())
        info.processing_start_s = time.monotonic()
        for stream, fn, with_time in self._outputs:   # registration order, sequential
            rdd = stream.compute(batch)
            fn(rdd, batch.batch_time_ms) if with_time else fn(rdd)
        info.processing_end_s = time.monotonic()
        self.batches_done += 1
        self.records_done += batch.n
        self.batch_infos.append(info)
        for cb in self.on_batch_completed:
            cb(info)
        return info

    def run_batches(self, n: int, now_ms: Optional[Callable[[], int]] = None) -> List[BatchInfo]:
        """Synchronously pull, seal and process ``n`` batches (no threads)."""
        if len(self._inputs) != 1:
            raise RuntimeError("run_batches needs exactly one input stream")
        src = self._inputs[0].source
        out = []
        for _ in range(n):
            t_ms = now_ms() if now_ms else self.clock.now_ms()
            size = self.batch_size if self.batch_size > 0 else self.poll_chunk
            batch = src.poll(size, now_ms=t_ms)
            batch.batch_time_ms = t_ms
            if not now_ms:
                self.clock.advance()
            out.append(self.run_batch(batch))
        return out

    def _receiver_loop(self, stream: ReceiverDStream) -> None:
        src = stream.source
        while not self._stop.is_set():
            if self.num_batches and self._sealed >= self.num_batches:
                self._stop.wait(0.05)           # all requested batches are sealed
                continue
            if self.max_pending > 0 and self._jobs.qsize() >= self.max_pending:
                self._stop.wait(0.005)          # backpressure: executor is behind
                continue
            # a source that delivers whole batches (chunk_rows, e.g. a replay
            # pool) is polled for them: one part per batch, no concatenation
            want = max(self.poll_chunk, int(getattr(src, "chunk_rows", 0) or 0))
            if self.batch_size > 0:             # never overfill: exact-size batches
                with self._lock:
                    want = min(want, self.batch_size - self._buffered)
                if want <= 0:
                    self._seal()
                    continue
            elif self.max_batch_rows > 0:       # time-sealed: stay within capacity
                with self._lock:
                    want = min(want, self.max_batch_rows - self._buffered)
                if want <= 0:
                    self._capacity_seal()
                    continue
            try:
                chunk = src.poll(want, now_ms=self.clock.now_ms())
            except Exception as e:  # receiver restart semantics: log and retry
                log.warning("receiver error, restarting: %s", e)
                time.sleep(0.5)
                continue
            if chunk.n:
                if (self.max_batch_units > 0 and self._buffered
                        and self._buffered_units + chunk.total_units > self.max_batch_units):
                    self._capacity_seal()       # this chunk starts the next batch
                with self._lock:
                    self._buffer.append(chunk)
                    self._buffered += chunk.n
                    self._buffered_units += chunk.total_units
                if self.batch_size > 0 and self._buffered >= self.batch_size:
                    self._seal()
            else:
                time.sleep(0.01)

    def _capacity_seal(self) -> None:
        if self.capacity_seals == 0:
            log.warning("micro-batch reached the engine capacity (%d rows / %d units): sealed early",
                        self.max_batch_rows, self.max_batch_units)
        self.capacity_seals += 1
        self._seal()

    def _seal(self) -> None:
        if self.num_batches and self._sealed >= self.num_batches:
            return                              # never seal past the requested count
        with self._lock:
            parts, self._buffer, self._buffered = self._buffer, [], 0
            self._buffered_units = 0
            self._sealed += 1
            t_ms = self.clock.now_ms()
            self.clock.advance()
        batch = RawBatch.concat(parts, t_ms) if parts else RawBatch.empty(t_ms)
        batch.batch_time_ms = t_ms
        self._jobs.put((batch, BatchInfo(t_ms, batch.n, time.monotonic())))

    def _generator_loop(self) -> None:
        if self.batch_seconds <= 0:
            return
        t_next = time.monotonic() + self.batch_seconds
        while not self._stop.is_set():
            delay = t_next - time.monotonic()
            if delay > 0 and self._stop.wait(delay):
                break
            t_next += self.batch_seconds
            self._seal()

    def _executor_loop(self) -> None:
        try:
            while not self._stop.is_set():
                try:
                    item = self._jobs.get(timeout=0.1)
                except queue.Empty:
                    continue
                if item is None:
                    break
                batch, info = item
                self._prefetch_upcoming()
                self.run_batch(batch, info)
                if self.num_batches and self.batches_done >= self.num_batches:
                    self._stop.set()
        except BaseException as e:  # surfaced by awaitTermination
            self.error = e
            self._stop.set()
        finally:
            self._done.set()

    def start(self) -> None:
        if self._threads:
            raise RuntimeError("StreamingContext already started")
        for s in self._inputs:
            self._threads.append(threading.Thread(target=self._receiver_loop, args=(s,),
                                                  name="receiver", daemon=True))
        self._threads.append(threading.Thread(target=self._generator_loop, name="job-generator",
                                              daemon=True))
        self._threads.append(threading.Thread(target=self._executor_loop, name="job-executor",
                                              daemon=True))
        for t in self._threads:
            t.start()

    def awaitTermination(self, timeout: Optional[float] = None) -> bool:
        finished = self._done.wait(timeout)
        if self.error is not None:
            raise self.error
        return finished

    awaitTerminationOrTimeout = awaitTermination

    def stop(self, stop_gracefully: bool = True) -> None:
        self._stop.set()
        self._jobs.put(None)
        for t in self._threads:
            t.join(timeout=10)
        self._done.set()
