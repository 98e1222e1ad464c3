"""twtml-spark KMeans driver (``KMeans.scala:15-170``).

Reference behaviour: streaming k-means with ``k = 3`` on 2-d points
``[retweetCount, followersCount]`` of every retweet (no range filter),
``setHalfLife(5, "batches")``, ``setRandomCenters(2, 0.0)``, 5 s batches; per
non-empty batch ``count += n``, ``StandardScaler(false, true).fit(rdd)
.transform(rdd)``, ``latestModel.update(scaled, decayFactor, timeUnit)``, then
collect x/y/centers/predictions and debug-log them.  It creates a Lightning
session named ``twitter-stream-ml-kmeans`` but plots nothing (all plotting and
web stats are commented out, ``KMeans.scala:89-131``).

Like the reference it reads ``lightning``/``twtweb`` from ``ConfigFactory.load``
and ignores the LR flags; extension flags select the engine and the k=1024
configuration: ``--master``, ``--k``, ``--textDims`` (hashed bigram dims
appended to the 2 numeric features), ``--seconds``, ``--numBatches``,
``--source``, ``--sourceRate``, ``--batchSize``, ``--checkpoint``, ``--report``
(post Stats/plot like the LR job).
"""
from __future__ import annotations

import argparse
import logging
import os
import sys
from typing import List, Optional

import numpy as np

from ..config.arguments import parse_master
from ..config.hocon import ConfigFactory, load_java_opts
from ..models.kmeans import CpuKMeans, StreamingKMeansModel, kmeans_features
from ..parallel.dist import barrier, check_replicas
from ..runtime.streaming import StreamingContext
from ..sources import make_source
from ..utils.faults import maybe_inject
from ..utils.gil import streaming_latency
from ..utils.logging import setup_logging
from ._common import (ResumeState, StreamCheckpointer, exit_on_sigterm, load_resume_state,
                      make_watchdog)

__all__ = ["main", "KMeansJob", "build_kmeans_engine"]

log = logging.getLogger("com.giorgioinf.twtml.spark.KMeans")
APP_NAME = "twitter-stream-ml-kmeans"


def parse_args(argv: List[str]) -> argparse.Namespace:
    ap = argparse.ArgumentParser(prog="twtml-kmeans")
    ap.add_argument("--master", "-m", default="local[*]")
    ap.add_argument("--k", type=int, default=3)
    ap.add_argument("--textDims", type=int, default=0)
    ap.add_argument("--halfLife", type=float, default=5.0)
    ap.add_argument("--seconds", type=float, default=5.0)
    ap.add_argument("--numBatches", type=int, default=0)
    ap.add_argument("--batchSize", type=int, default=0)
    ap.add_argument("--source", default="synthetic")
    ap.add_argument("--sourceRate", type=float, default=50.0)
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--checkpoint", default="")
    ap.add_argument("--checkpointInterval", type=int, default=10)
    ap.add_argument("--resume", default="", help="model dir (warm start) or 'auto'")
    ap.add_argument("--batchTimeout", type=float, default=0.0)
    ap.add_argument("--checkReplicas", type=int, default=0)
    ap.add_argument("--report", action="store_true")
    return ap.parse_args(argv)


def build_kmeans_engine(args, dim: int, rank: int, world: int):
    spec = parse_master(args.master)
    if spec.is_gpu:
        from ..ops.kmeans_engine import DeviceKMeans, KMDeviceConfig
        from ..parallel.dist import make_rccl_comm
        dev = spec.devices[rank] if spec.devices else rank
        from ..parallel.affinity import bind_local_numa
        bind_local_numa(dev)   # pinned staging buffers on the GPU's NUMA node
        from ..parallel.affinity import share_host_threads
        import torch
        share_host_threads(dev, rank, int(os.environ.get("LOCAL_WORLD_SIZE", world)),
                           max(1, torch.cuda.device_count()))
        rows = max(65536, args.batchSize)
        from .linear_regression import DRIVER_RAW_SLOTS   # sized from the scheduler's prefetch depth
        cfg = KMDeviceConfig(k=args.k, text_dims=args.textDims, half_life=args.halfLife,
                             max_rows=rows, max_units=rows * 290, seed=args.seed,
                             raw_slots=int(os.environ.get("TWTML_RAW_SLOTS", "0") or 0) or DRIVER_RAW_SLOTS)
        return DeviceKMeans(cfg, device=dev, comm=make_rccl_comm(dev) if world > 1 else None)
    from ..parallel.dist import allreduce_fn
    return CpuKMeans(args.k, dim, half_life=args.halfLife, init_weight=0.0, seed=args.seed,
                     allreduce=allreduce_fn())


class KMeansJob:
    def __init__(self, engine, text_dims: int = 0, session=None, rank: int = 0, args=None,
                 resume: Optional[ResumeState] = None):
        self.engine = engine
        self.text_dims = text_dims
        self.session = session
        self.rank = rank
        resume = resume or ResumeState()
        self.count = resume.count
        self.batches = resume.batches      # stream batches seen (incl. empty ones)
        self.records = resume.records
        self.last = None
        ckpt = getattr(args, "checkpoint", "") if args is not None else ""
        interval = getattr(args, "checkpointInterval", 0) if args is not None else 0
        self.check_every = getattr(args, "checkReplicas", 0) if args is not None else 0
        self.checkpointer = StreamCheckpointer(
            ckpt, interval, rank,
            self._snapshot, barrier)
        self.watchdog = make_watchdog(getattr(args, "batchTimeout", 0.0) if args is not None else 0.0,
                                      getattr(engine, "comm", None))

    def on_batch(self, rdd, time_ms: int) -> None:
        raw = rdd.raw
        maybe_inject(self.rank, self.batches + 1)
        if self.watchdog is not None:
            self.watchdog.arm()
        try:
            self._step(raw)
            self.batches += 1
            self.records += raw.n
            if self.check_every > 0 and self.batches % self.check_every == 0:
                check_replicas(np.concatenate([a.ravel() for a in self.engine.get_state()]),
                               "k-means state")
            self.checkpointer.after_batch(self.batches, self.records, self.count)
        finally:
            if self.watchdog is not None:
                self.watchdog.disarm()

    def _snapshot(self):
        """k x d centres + k weights (small): copied on the training thread,
        written on the checkpoint writer thread."""
        model = StreamingKMeansModel(*[np.array(a, copy=True) for a in self.engine.get_state()])
        return model.save

    def final_checkpoint(self) -> None:
        self.checkpointer.flush()
        self.checkpointer.after_batch(self.batches, self.records, self.count, force=True)

    def close(self) -> None:
        try:
            self.checkpointer.flush()   # never leave a checkpoint half-written behind
        except Exception as e:
            log.error("%s", e)
        if self.watchdog is not None:
            self.watchdog.close()

    def _step(self, raw) -> None:
        if hasattr(self.engine, "update_raw"):
            res = self.engine.update_raw(raw)                 # fused device pipeline
        else:
            X, _ = kmeans_features(raw, self.text_dims)
            res = self.engine.update_batch(X)
        self.last = res
        if res["n"] == 0:
            return
        self.count += res["n"]
        centers, weights = self.engine.get_state()
        if log.isEnabledFor(logging.DEBUG):
            scaled = res.get("scaled")
            log.debug("\n\tmodelx: %s\n\tmodely: %s\n\tdatax: %s\n\tdatay: %s\n\tpred: %s",
                      centers[:, 0].tolist(), centers[:, 1].tolist(),
                      [] if scaled is None else scaled[:20, 0].tolist(),
                      [] if scaled is None else scaled[:20, 1].tolist(),
                      np.asarray(res.get("pred", []))[:20].tolist())
        if self.session is not None and self.rank == 0:
            self.session.web_stats_only(self.count, res["n"])


def main(argv: Optional[List[str]] = None) -> int:
    setup_logging()
    exit_on_sigterm()
    from ..runtime.clock import streaming_clock
    rest = load_java_opts(list(sys.argv[1:] if argv is None else argv))
    args = parse_args(rest)
    log.info("Loading application config...")
    conf = ConfigFactory.load()
    lgn_host = conf.getString("lightning")
    web_host = conf.getString("twtweb")
    from ..parallel.dist import init_distributed
    info = init_distributed(backend="nccl" if parse_master(args.master).is_gpu else "gloo")
    dim = 2 + args.textDims
    engine = build_kmeans_engine(args, dim, info.rank, info.world)
    resume = load_resume_state(args.resume, args.checkpoint, info.rank)
    if resume.path:
        model = StreamingKMeansModel.load(resume.path)
        engine.set_state(model.clusterCenters, model.clusterWeights)
        log.info("resumed k-means state from %s (batch %d)", resume.path, resume.batches)
    remaining = args.numBatches
    if args.numBatches and resume.batches:
        remaining = max(0, args.numBatches - resume.batches)
        if remaining == 0:
            return 0
    log.info("Initializing Streaming Spark Context...")
    cap = getattr(engine, "cfg", None)   # device engine: staging capacity per batch
    ssc = StreamingContext(args.seconds, batch_size=args.batchSize, num_batches=remaining,
                           app_name=APP_NAME,
                           max_batch_rows=int(getattr(cap, "max_rows", 0) or 0),
                           max_batch_units=int(getattr(cap, "max_units", 0) or 0),
                           clock=streaming_clock())
    log.info("Initializing Twitter stream...")
    stream = ssc.twitterStream(make_source(args.source, rate=args.sourceRate, seed=args.seed,
                                           shard=info.rank, num_shards=info.world,
                                           start=resume.records, batch_size=args.batchSize))
    session = None
    if info.rank == 0:
        log.info("Initializing Lightning graph session...")
        from ..report.lightning import Lightning, LightningError
        try:
            Lightning(lgn_host).create_session(APP_NAME)
        except LightningError as e:
            log.warning("lightning unavailable: %s", e)
        if args.report:
            from ..report.session_stats import SessionStats
            session = SessionStats(lgn_host, web_host).open()
    job = KMeansJob(engine, args.textDims, session, info.rank, args, resume)
    stream.foreachRDD(job.on_batch)
    if hasattr(engine, "prefetch"):   # device engine: H2D of queued batches overlaps training
        ssc.add_prefetch(engine.prefetch)
    log.info("Initialization complete.")
    # from here background threads never hold the training thread up long
    # (GIL slices, a frozen GC heap): entered before the first batch
    latency = streaming_latency()
    latency.__enter__()
    ssc.start()
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
        job.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
