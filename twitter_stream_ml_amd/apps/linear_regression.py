"""twtml-spark LinearRegression driver (``LinearRegression.scala:10-94``).

Flow kept from the reference:

1. parse ``ConfArguments`` (app name ``twitter-stream-ml-linear-regression``);
2. open the report session (Lightning plot + twtml-web Config);
3. ``MllibHelper.reset(conf)``; model with ``numIterations``/``stepSize``/
   ``miniBatchFraction`` and zero initial weights of size ``F + 4``;
4. streaming context with ``seconds`` batches over the tweet source, stream
   ``filter(filtrate).map(featurize).cache()``;
5. per batch, output op #1: prequential predict with the current model,
   ``count``/``batch``/``stdev``/``mse`` (rounded with ``Utils.round``),
   debug logs, ``session.update``; output op #2: ``model.trainOn(stream)``;
6. start and block.

Engines: ``--master local[N]`` runs the fp64 CPU engine; ``--master rocm...``
the MI355X engine, which executes filter, featurize, op #1 and op #2 of a
batch in one fused device pipeline — op #1 still sees the weights of batch
t-1 (the stats come out of GD iteration 1, computed before any update).
Data parallel runs start one process per GPU (``torch.distributed.run``);
every rank reads its own shard of the stream and rank 0 reports.

Extensions (long flags only): ``--source``, ``--batchSize``, ``--numBatches``,
``--hash``, ``--checkpoint``/``--checkpointInterval``, ``--resume``,
``--plotPoints``, ``--metrics FILE`` (via env ``TWTML_METRICS``).
"""
from __future__ import annotations

import logging
import math
import os
import sys
import time
from typing import List, Optional

import numpy as np

from ..config.arguments import ConfArguments
from ..config.hocon import load_java_opts
from ..models.linear_regression import CpuLinearRegression, CpuLRConfig, LinearRegressionModel
from ..models.mllib_helper import MllibHelper
from ..parallel.dist import barrier, broadcast_flag, check_replicas
from ..utils.faults import maybe_inject
from ..checkpoint.saveable import SparseWeights
from ._common import (ResumeState, StreamCheckpointer, exit_on_sigterm, load_resume_state,
                      make_watchdog)
from ..oracle.mllib import round_half_up
from ..utils.gil import streaming_latency
from ..report.session_stats import SessionStats
from ..runtime.streaming import StreamingContext
from ..sources import make_source
from ..utils.logging import setup_logging
from ..utils.metrics import MetricsLogger

__all__ = ["main", "build_engine", "LinearRegressionJob"]

# TWTML_SNAP_REUSE=0 (A/B): a fresh host array per checkpoint
_SNAP_REUSE = os.environ.get("TWTML_SNAP_REUSE", "1") != "0"

log = logging.getLogger("com.giorgioinf.twtml.spark.LinearRegression")
APP_NAME = "twitter-stream-ml-linear-regression"


# The streaming scheduler offers at most this many sealed batches to the
# engine's prefetch (runtime/streaming.py prefetch_depth): one slot trains, one
# is the free slot a batch without a prefetch takes, the rest hold prefetches.
DRIVER_PREFETCH_DEPTH = 2
DRIVER_RAW_SLOTS = DRIVER_PREFETCH_DEPTH + 2


def build_engine(conf: ConfArguments, rank: int, world: int, device: Optional[int] = None,
                 max_rows: int = 0):
    """CPU (local[N]) or MI355X (rocm...) engine for this process."""
    spec = conf.master_spec()
    F = conf.effectiveNumTextFeatures
    if spec.is_gpu:
        from ..ops.lr_engine import DeviceLinearRegression, LRDeviceConfig
        from ..parallel.dist import make_comm
        dev = device if device is not None else (spec.devices[rank] if spec.devices else rank)
        from ..parallel.affinity import bind_local_numa
        bind_local_numa(dev)   # pinned staging buffers on the GPU's NUMA node
        from ..parallel.affinity import share_host_threads
        import torch
        share_host_threads(dev, rank, int(os.environ.get("LOCAL_WORLD_SIZE", world)),
                           max(1, torch.cuda.device_count()))
        cap = os.environ.get("TWTML_BATCH_ROWS", "")

        def lr_cfg(rows: int) -> LRDeviceConfig:
            # ingest "utf8": the receiver's UTF-8 bytes cross PCIe as they are
            # (DMA'd from its page-locked buffer when the source pins them) and
            # the device decodes / lower-cases / narrows -- the path bench.py times.
            # HBM-sized batches keep 4 raw slots: each slot holds a whole batch
            # of text, and the rows are worth more than run-ahead depth there
            return LRDeviceConfig(num_text_features=F, hash=conf.hash, step_size=conf.stepSize,
                                  num_iterations=conf.numIterations, fraction=conf.miniBatchFraction,
                                  begin=conf.numRetweetBegin, end=conf.numRetweetEnd,
                                  max_rows=rows, max_units=rows * 290, ingest="utf8",
                                  # device raw slots (TWTML_RAW_SLOTS overrides): the driver
                                  # prefetches only the batches its scheduler has sealed (at most
                                  # DRIVER_PREFETCH_DEPTH), so it never uses more than that + 2;
                                  # the HBM sizing counts these slots' bytes
                                  raw_slots=int(os.environ.get("TWTML_RAW_SLOTS", "0") or 0) or DRIVER_RAW_SLOTS)

        rows = max_rows or max(65536, int(conf.batchSize or 0))
        if cap.lower() == "hbm":   # the largest micro-batch 80 % of this GPU's free HBM holds
            import torch
            from ..ops.sizing import hbm_max_rows
            rows = max(rows, hbm_max_rows(lambda r: DeviceLinearRegression(lr_cfg(r), device=dev),
                                          torch.cuda.mem_get_info(dev)[0]))
        elif cap:
            rows = max(rows, int(cap))
        cfg = lr_cfg(rows)
        # one RCCL communicator: per GD iteration one int64 all-reduce, per
        # batch one all-gather of the prep packets (overlapped with the
        # previous batch's GD loop) and the stats all-reduce
        comm = make_comm(dev, "rccl") if world > 1 else None
        return DeviceLinearRegression(cfg, device=dev, comm=comm)
    from ..parallel.dist import allreduce_fn
    cfg = CpuLRConfig(num_text_features=F, hash=conf.hash, step_size=conf.stepSize,
                      num_iterations=conf.numIterations, fraction=conf.miniBatchFraction,
                      begin=conf.numRetweetBegin, end=conf.numRetweetEnd)
    return CpuLinearRegression(cfg, allreduce=allreduce_fn(), rank=rank, world=world)


class LinearRegressionJob:
    """The driver's per-batch logic, reusable from tests and the CLI."""

    def __init__(self, conf: ConfArguments, engine, session: Optional[SessionStats] = None,
                 rank: int = 0, metrics: Optional[MetricsLogger] = None,
                 resume: Optional[ResumeState] = None, world: int = 1, plot: Optional[bool] = None):
        self.conf = conf
        self.engine = engine
        self.session = session
        self.rank = rank
        self.world = world
        # plot: rank 0 appends real/pred to a live Lightning plot, so every
        # rank collects its predictions (D2H) and ships a sample; otherwise
        # a batch's report needs only the six fused statistics
        self.plot = (session is not None and getattr(session, "viz", None) is not None) if plot is None else plot
        self.tweets = 0                # trained tweets (all ranks), for the throughput summary
        self.t_first = self.t_last = None
        self.timeline = []             # (end time, trained tweets) per batch
        resume = resume or ResumeState()
        self.count = resume.count      # the "count" accumulator
        self.batches = resume.batches  # stream batches trained into the model
        self.records = resume.records  # source records this rank consumed
        self.metrics = metrics or MetricsLogger(None)
        self.last = None
        self._t0 = 0.0
        self.diverged = 0    # batches on which the model was found diverged (training stopped)
        self.checkpointer = StreamCheckpointer(conf.checkpoint, conf.checkpointInterval, rank,
                                               self._snapshot, barrier)
        # plot samples per rank: the device samples them (0 = every kept row),
        # the shipper thread gathers them to rank 0 and hands them to the
        # session worker -- nothing of the plot runs on the training thread
        pp = int(getattr(conf, "plotPoints", 0) or 0)
        self.plot_points = 0 if pp <= 0 else max(1, -(-pp // max(1, world)))
        self.shipper = None
        if self.plot:
            from ..report.plot_shipper import PlotShipper
            self.shipper = PlotShipper(session if rank == 0 else None, rank, world)
        self.watchdog = make_watchdog(conf.batchTimeout, getattr(engine, "comm", None))

    def on_batch(self, rdd, time_ms: int) -> None:
        raw = rdd.raw
        maybe_inject(self.rank, self.batches + 1)
        if self.watchdog is not None:
            self.watchdog.arm()
        t0 = self._t0 = time.perf_counter()
        res = self.engine.train_batch(raw, want_pred=self.plot, plot_points=self.plot_points)  # op #1, op #2
        t1 = time.perf_counter()
        # the engine call on this thread, and the part of it spent waiting to
        # take the GIL back after the device work (other Python threads)
        self._call_ms = (t1 - t0) * 1e3
        self._gil_ms = (time.monotonic_ns() - res["done_ns"]) / 1e6 if "done_ns" in res else None
        if self.t_first is None:
            self.t_first = t0
        self.t_last = t1
        self.tweets += int(res.get("n_kept_global", 0))
        self.timeline.append((t1, int(res.get("n_kept_global", 0))))
        self.last = res
        if res.get("diverged"):
            # the residual bound / weights left any usable range (sgd.hip
            # sgd_scales): MLlib's fp64 model would go to Inf/NaN here and
            # Utils.round throw; the engine stops training the batch instead
            log.error("batch %d: the model diverged (|residual| bound >= 1e30 or non-finite weights); "
                      "training stopped (stepSize %s too large?)", self.batches + 1, self.conf.stepSize)
            self.diverged += 1
        self.batches += 1
        self.records += raw.n
        try:
            self._report(raw, res, time_ms)
            if self.conf.checkReplicas > 0 and self.batches % self.conf.checkReplicas == 0:
                check_replicas(self.engine.get_weights(), "LR weights")
            self.checkpointer.after_batch(self.batches, self.records, self.count)
        finally:
            if self.watchdog is not None:
                self.watchdog.disarm()

    def _report(self, raw, res, time_ms: int) -> None:
        batch = int(res["n_kept_global"])
        if batch == 0:
            log.debug("batch: 0")
            self.metrics.log(batch_time_ms=time_ms, raw=raw.n, batch=0)
            return
        self.count += batch
        n, sy, sy2, sp, sp2, se2 = res["stats"]
        if n <= 0:   # no prequential pass: the model had diverged before this batch
            log.error("batch %d: model diverged; skipping report", self.batches)
            self.metrics.log(batch_time_ms=time_ms, raw=raw.n, batch=batch, diverged=True)
            return
        my, mp = sy / n, sp / n
        try:
            real_sd = round_half_up(math.sqrt(max(sy2 / n - my * my, 0.0)))
            pred_sd = round_half_up(math.sqrt(max(sp2 / n - mp * mp, 0.0)))
            mse = round_half_up(se2 / n)
        except ValueError as e:  # Utils.round on NaN/Inf: the model diverged
            log.error("batch %d: model diverged (%s); skipping report", self.batches, e)
            self.metrics.log(batch_time_ms=time_ms, raw=raw.n, batch=batch, diverged=True)
            return
        real = pred = np.zeros(0)
        if self.plot:
            # CS7 real.toArray / pred.toArray: this rank's sampled kept rows,
            # labels and predictions straight from the engine (no host mask)
            if res.get("real") is not None:
                real = np.asarray(res["real"], np.float64)
                pred = np.asarray(res["pred"], np.float64)
        if log.isEnabledFor(logging.DEBUG):
            log.debug("count: %d", self.count)
            log.debug("batch: %d,  mse: %d", batch, int(mse))
            log.debug("stdev (real, pred): (%d, %d)", int(real_sd), int(pred_sd))
            log.debug("value (real, pred): %s ...",
                      [(float(a), float(b)) for a, b in zip(real[:10], pred[:10])])
        stats = (self.count, batch, mse, real_sd, pred_sd)
        if self.shipper is not None:   # every rank: its sample goes to rank 0 off this thread
            if self.session is not None and self.rank == 0:
                self.session.push_stats(*stats)   # not held back by the plot gather
            self.shipper.submit(stats, real, pred)
        elif self.session is not None and self.rank == 0:
            self.session.update(*stats, real, pred)
        # step_ms: the batch on the training thread, train + report (the plot included)
        self.metrics.log(batch_time_ms=time_ms, raw=raw.n, batch=batch, count=self.count,
                         mse=mse, realStdev=real_sd, predStdev=pred_sd,
                         iterations=res["iterations"], converged=bool(res["converged"]),
                         diverged=bool(res.get("diverged", False)),
                         prep_ms=res.get("prep_ms", 0.0), train_ms=res.get("train_ms", 0.0),
                         step_ms=round((time.perf_counter() - self._t0) * 1e3, 3),
                         call_ms=round(self._call_ms, 3),
                         wait_ms=round(float(res.get("wait_ms", 0.0)), 3),
                         train_wall_ms=round(float(res.get("train_wall_ms", 0.0)), 3),
                         ahead=bool(res.get("prepared_ahead", False)),
                         phases=[round(float(x), 3) for x in res.get("phases", ())],
                         **({} if self._gil_ms is None else {"gil_wait_ms": round(self._gil_ms, 3)}))

    def summary(self) -> dict:
        """Throughput of the run: trained tweets (all ranks) over the wall
        time from the first batch's start to the last one's end, and the
        steady state after the first quarter of the batches (at most 5, the
        warm-up bench.py does not time either)."""
        secs = (self.t_last - self.t_first) if self.t_first is not None else 0.0
        rec = dict(summary=True, batches=self.batches, tweets=self.tweets, seconds=round(secs, 6),
                   tweets_per_s=(self.tweets / secs) if secs > 0 else 0.0, diverged_batches=self.diverged)
        skip = min(5, len(self.timeline) // 4)
        if len(self.timeline) - skip >= 2:
            t_a = self.timeline[skip - 1][0] if skip else self.t_first
            n = sum(k for _, k in self.timeline[skip:])
            dt = self.timeline[-1][0] - t_a
            rec.update(steady_batches=len(self.timeline) - skip, steady_tweets=n,
                       steady_seconds=round(dt, 6), steady_tweets_per_s=n / dt if dt > 0 else 0.0)
        self.metrics.log(**rec)
        log.info("trained %d tweets in %d batches, %.3f s: %.1f tweets/s", self.tweets, self.batches, secs,
                 rec["tweets_per_s"])
        return rec

    def _snapshot(self):
        """Checkpoint snapshot on the training thread; the returned save runs
        on the checkpoint writer thread.  Device engine: the non-zero weights
        are compacted on the GPU behind the last batch and only they are
        copied (csrc/hip/snapshot.hip); CPU engine: a copy of the weights."""
        eng = self.engine
        if hasattr(eng, "snapshot_begin"):
            eng.snapshot_begin()

            def save(path, prog):
                # views of the engine's own host buffers: one write in flight at
                # a time, so nothing else fetches before this save is done
                size, idx, val = eng.snapshot_fetch(reuse=_SNAP_REUSE)
                LinearRegressionModel.save_sparse(path, SparseWeights(size, idx, val), 0.0, prog)
            return save
        w = np.array(eng.get_weights(), dtype=np.float64, copy=True)
        return lambda path, prog: LinearRegressionModel(w, 0.0).save(path, prog)

    def final_checkpoint(self) -> None:
        self.checkpointer.flush()
        self.checkpointer.after_batch(self.batches, self.records, self.count, force=True)

    def close(self) -> None:
        if self.shipper is not None:
            self.shipper.close()
        try:
            self.checkpointer.flush()   # never leave a checkpoint half-written behind
        except Exception as e:
            log.error("%s", e)
        if self.watchdog is not None:
            self.watchdog.close()


def main(argv: Optional[List[str]] = None) -> int:
    setup_logging()
    exit_on_sigterm()
    from ..runtime.clock import streaming_clock
    args = load_java_opts(list(sys.argv[1:] if argv is None else argv))
    log.info("Parsing applications arguments")
    conf = ConfArguments().setAppName(APP_NAME).parse(args)

    from ..parallel.dist import init_distributed
    spec = conf.master_spec()
    info = init_distributed(backend="nccl" if spec.is_gpu else "gloo")
    rank, world = info.rank, info.world

    session = None
    if rank == 0:
        log.info("Initializing session stats...")
        session = SessionStats.from_conf(conf).open()

    log.info("Initializing Spark Machine Learning Model...")
    MllibHelper.reset(conf)
    engine = build_engine(conf, rank, world)
    w0 = np.zeros(engine.num_weights)                      # Vectors.zeros(numFeatures)
    resume = load_resume_state(conf.resume, conf.checkpoint, rank)
    if resume.path:
        w0 = LinearRegressionModel.load(resume.path).weights
        log.info("resumed %d weights from %s (batch %d, %d records consumed)", w0.shape[0],
                 resume.path, resume.batches, resume.records)
    engine.set_weights(w0)
    remaining = conf.numBatches
    if conf.numBatches and resume.batches:
        remaining = max(0, conf.numBatches - resume.batches)
        if remaining == 0:
            log.info("checkpoint already holds %d batches; nothing to do", resume.batches)
            return 0

    log.info("Initializing Streaming Spark Context... %s sec/batch", conf.seconds)
    cap = getattr(engine, "cfg", None)   # device engines: staging capacity per batch
    ssc = StreamingContext(conf.seconds, batch_size=conf.batchSize, num_batches=remaining,
                           app_name=conf.appName(),
                           max_batch_rows=int(getattr(cap, "max_rows", 0) or 0),
                           max_batch_units=int(getattr(cap, "max_units", 0) or 0),
                           clock=streaming_clock())
    log.info("Initializing Twitter stream...")
    stream = ssc.twitterStream(make_source(conf.source, rate=conf.sourceRate, seed=conf.seed,
                                           shard=rank, num_shards=world,
                                           start=resume.records, batch_size=conf.batchSize)).cache()
    plot = broadcast_flag(session is not None and session.viz is not None)   # the same on every rank
    job = LinearRegressionJob(conf, engine, session, rank,
                              MetricsLogger(os.environ.get("TWTML_METRICS")), resume, world, plot=plot)
    log.info("Initializing prediction model...")
    stream.foreachRDD(job.on_batch)   # op #1 (stats) + op #2 (trainOn), prequential order
    if hasattr(engine, "prefetch"):   # device engine: H2D of queued batches overlaps training
        ssc.add_prefetch(engine.prefetch)
    # from here background threads never hold the training thread up long
    # (GIL slices, a frozen GC heap): entered before the first batch
    latency = streaming_latency()
    latency.__enter__()
    ssc.start()
    log.info("Initialization complete.")
    failed = False
    try:
        ssc.awaitTermination()
    except KeyboardInterrupt:
        pass
    except BaseException:
        failed = True
        raise
    finally:
        ssc.stop()
        latency.__exit__(None, None, None)
        if not failed:
            job.final_checkpoint()
            if rank == 0:
                job.summary()
        job.close()
        if session is not None:
            session.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
