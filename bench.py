#!/usr/bin/env python3
"""Headline benchmark: tweets/sec trained (whole node) + p50 micro-batch latency.

Config (BASELINE.json config 2/3): online linear regression
(StreamingLinearRegressionWithSGD, stepSize 0.005, numIterations 50,
miniBatchFraction 1.0, convergence tol 1e-3) on 1M-dim hashed character-bigram
features (+4 numeric), synthetic tweet-shaped data, random/zero-init weights
as in the reference (``Vectors.zeros``), data-parallel over N GPUs with the
gradient all-reduced over RCCL every GD iteration.

One *step* = one micro-batch end to end: H2D of the raw tweets (overlapped
with the previous batch), filter, lower-case + bigram hashing, prequential
predict + stats, and up to 50 GD iterations (early exit on convergence, as
MLlib).  Each rank trains ``--batch`` raw tweets per step (weak scaling).

Two ingest modes:

* default (end to end): each timed step also stages a fresh batch on the
  host from the raw records (the pool stands in for the network receiver): a staging
  thread runs ahead of the GPU by up to two batches.  ``--ingest utf8``
  (default) keeps the text as the UTF-8 bytes the network delivers: the
  host stages row words + packed scalars and the text is DMA'd straight from
  the receiver's registered buffer (~152 B per tweet on PCIe; the device
  decodes non-ASCII rows and narrows Latin-1 ones).  ``--ingest utf16`` does
  the same from Java-style UTF-16 records (~300 B per tweet), ``--ingest
  wire`` runs the host packer on every batch.  Lower-casing, incl. the
  special rows, is on the device in every mode.
* ``--prepacked`` (device pipeline only): batches are replayed from a pool
  packed into the wire format once (Latin-1 / cesu rows, row words, 1-4 byte
  scalar columns, ~166 B per tweet); the H2D of every batch is in the timed
  region, the host packing is not.

``--profile wide`` replaces the ~300-word toy vocabulary by a realistic
50K-word multi-script one (~200K active bigrams per batch: the tiered SGD
layout).

Usage:  python bench.py [--gpus N --steps K --warmup W] [--prepacked] [--profile wide]
        (N>1: python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...)
"""
from __future__ import annotations

import argparse
import json
import os
import queue
import sys
import threading
import time

import numpy as np

T_START = time.time()
# The reference publishes no number, so vs_baseline is against
# BASELINE.json config 1 measured here: the reference's own mode, --master
# local[2] (fp64 CPU engine, MLlib semantics) on the same wide synthetic data,
# on a GPU box's host CPU -- profiles/r6/config1_local2.json
# (python bench.py --master 'local[2]' --steps 20 --warmup 5).
BASELINE_TWEETS_PER_SEC = 119353.4


def parse_args(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawTextHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--model", choices=["lr", "kmeans"], default="lr",
                    help="lr: headline config 2/3/5; kmeans: config 4 (StreamingKMeans)")
    ap.add_argument("--k", type=int, default=1024, help="kmeans clusters")
    ap.add_argument("--text-dims", type=int, default=62, help="kmeans hashed bigram dims (+2 numeric)")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", default="1000000",
                    help="raw tweets per GPU per step, or 'hbm': the largest micro-batch whose engine "
                         "fits --hbm-fraction of the GPU's free memory (config 5 sizing), capped by --batch-cap")
    ap.add_argument("--hbm-fraction", type=float, default=0.8, help="--batch hbm: share of free HBM")
    ap.add_argument("--batch-cap", type=int, default=8_000_000, help="--batch hbm: upper bound (host pool size)")
    ap.add_argument("--features", type=int, default=1_000_000, help="numTextFeatures")
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--step-size", type=float, default=0.005)
    ap.add_argument("--pool", type=int, default=0,
                    help="pre-generated batches per rank (0: warmup + steps, i.e. every step trains a batch "
                         "it has never seen; a smaller pool replays batches)")
    ap.add_argument("--hash", default="java")
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--profile", default="wide", choices=["bench", "wide"],
                    help="synthetic data: wide (default: realistic 50K-word multi-script vocabulary, "
                         "~200K active bigrams per batch) or bench (toy ~300-word vocabulary, ~1.4K active "
                         "bigrams)")
    ap.add_argument("--e2e", action="store_true",
                    help="stage every batch on the host inside the timed region (the default)")
    ap.add_argument("--prepacked", action="store_true",
                    help="device pipeline only: replay a pool packed once, host staging not timed")
    ap.add_argument("--ingest", choices=["utf8", "utf16", "wire"], default="",
                    help="host staging of --e2e: utf8 (default) / utf16 (text DMA'd from the receiver "
                         "buffer) or wire (host packer)")
    ap.add_argument("--sgd-grid", type=int, default=0)
    ap.add_argument("--ablate", type=int, default=0, help=argparse.SUPPRESS)
    ap.add_argument("--tol", type=float, default=1e-3, help=argparse.SUPPRESS)
    ap.add_argument("--dedup", type=int, default=0, help="merge repeated bigrams per row (1/0)")
    ap.add_argument("--hybrid", type=int, default=1, help="dense 4-bit counts for hot bigrams (1/0)")
    ap.add_argument("--comm", choices=["rccl", "gloo"], default="rccl",
                    help="DP gradient collectives: RCCL over xGMI, or host-staged torch.distributed "
                         "gloo (lets N ranks share one GPU for testing)")
    ap.add_argument("--force-dp", action="store_true",
                    help="take the engine's DP path at world 1 through a world-1 RCCL communicator (every "
                         "collective issued on the compute stream) and report the per-iteration all-reduce "
                         "time")
    ap.add_argument("--timeout", type=float, default=480.0,
                    help="whole-run watchdog (s, 0 = off): on expiry every rank dumps its Python stacks and "
                         "communicator counters, aborts the communicator and exits non-zero")
    ap.add_argument("--master", default="",
                    help="local[N]: BASELINE config 1 -- the fp64 CPU engine (oracle/mllib.py semantics, "
                         "what the reference's --master local[2] runs) on the same synthetic data, N host "
                         "threads (one stands for the receiver, as in Spark local mode); no GPU is used")
    ap.add_argument("--json-out", default="")
    ap.add_argument("--verbose", action="store_true")
    return ap.parse_args(argv)


class Runner:
    """Continuous stream of batches through an engine's raw slots."""

    def __init__(self, eng, is_km: bool, now_ms: int):
        self.eng, self.is_km, self.now_ms = eng, is_km, now_ms
        self.lat, self.kept, self.iters, self.stage, self.extra = [], [], [], [], []
        self.comm = []            # (gradient all-reduces, their ms) per timed batch
        self.prestaged_at_t0 = 0  # batches of the timed window staged / submitted before t0
        self.steps_done = 0
        self.marks = []           # (sealed, done) host clock per timed batch
        self.phases = []          # the engine's per-batch host / device phase times (LR)
        self.hang_at = 0          # TWTML_BENCH_HANG=<rank>:<step>: that rank hangs before that step

    def process(self, slot: int):
        self.steps_done += 1
        if self.hang_at and self.steps_done == self.hang_at:   # TWTML_BENCH_HANG (tests): never returns
            while True:
                time.sleep(3600)
        if self.is_km:
            return self.eng.process(slot, want_pred=False)
        return self.eng.process(slot, self.now_ms)

    def record(self, res, sealed: float, done: float) -> None:
        self.lat.append((done - sealed) * 1e3)
        self.marks.append((sealed, done))
        if self.is_km:
            self.kept.append(res["n_local"])
            self.stage.append((res["ms"], 0.0))
        else:
            self.kept.append(res["n_kept"])
            self.iters.append(res["iterations"])
            self.stage.append((res["prep_ms"], res["train_ms"]))
            self.extra.append((res.get("tiered", False), res.get("n_unique", 0), res.get("n_near", 0)))
            self.phases.append(list(res.get("phases", [])))
            self.comm.append((res.get("comm_iters", 0), res.get("comm_ms", 0.0), res.get("comm_bytes", 0)))


def run_device_pipeline(r: Runner, pool, warmup: int, steps: int, sync):
    """Pre-packed pool; batch t+depth is submitted (async H2D) before batch t
    is trained, so the copy engine always has the next batch queued.  Every
    timed step trains one batch and submits one."""
    eng = r.eng
    depth = max(1, min(int(os.environ.get("TWTML_BENCH_DEPTH", eng.raw_slots - 1)), eng.raw_slots - 1))
    state = {"next": 0, "cur": 0}
    sealed_at = {}

    def submit_one(limit):
        i = state["next"]
        if i >= limit:   # the timed window's batches are submitted inside it
            return
        sealed_at[i] = time.perf_counter()
        eng.submit(pool[i % len(pool)], i % eng.raw_slots)
        state["next"] = i + 1

    def run(n, record, limit):
        for _ in range(n):
            t = state["cur"]
            submit_one(limit)
            if state["next"] <= t:   # pipeline drained at the window edge: submit this one now
                submit_one(t + 1)
            res = r.process(t % eng.raw_slots)
            done = time.perf_counter()
            state["cur"] = t + 1
            if record:
                r.record(res, sealed_at.pop(t), done)
            else:
                sealed_at.pop(t)

    def timed():
        r.prestaged_at_t0 = max(0, state["next"] - warmup)
        for _ in range(depth - 1):   # prime inside the window
            submit_one(warmup + steps)
        run(steps, True, warmup + steps)

    for _ in range(depth - 1):   # prime: batches 0..depth-2 in flight before step 0
        submit_one(warmup)
    run(warmup, False, warmup)
    t0, t1 = sync(timed)
    return t0, t1


def _h2d_gbps(device: int, mb: int = 256, reps: int = 4) -> float:
    """Pinned host-to-device copy bandwidth of this GPU's link (GB/s)."""
    import torch
    n = mb << 20
    h = torch.empty(n, dtype=torch.uint8).pin_memory()
    d = torch.empty(n, dtype=torch.uint8, device=f"cuda:{device}")
    s = torch.cuda.Stream(device=device)
    with torch.cuda.stream(s):
        d.copy_(h, non_blocking=True)
    torch.cuda.synchronize(device)
    t = time.perf_counter()
    with torch.cuda.stream(s):
        for _ in range(reps):
            d.copy_(h, non_blocking=True)
    torch.cuda.synchronize(device)
    return n * reps / (time.perf_counter() - t) / 1e9


def run_e2e(r: Runner, raws, u8s, views, ingest: str, warmup: int, steps: int, sync):
    """Host staging inside the loop: a staging thread loads raw batch i into
    the staging buffer of a free raw slot (wire pack or UTF-16 row words +
    scalars) and submits its H2D, up to raw_slots - 1 batches ahead of the
    GPU; the main thread trains batches in order."""
    eng = r.eng
    total = warmup + steps
    free: "queue.Queue[int]" = queue.Queue()
    ready: "queue.Queue" = queue.Queue()
    ahead = max(1, min(int(os.environ.get("TWTML_E2E_DEPTH", eng.raw_slots - 1)), eng.raw_slots - 1))
    for s in range(ahead):   # batches staged ahead of the one training
        free.put(s)
    err = []
    # The timed window starts with an empty pipeline: batch `warmup` (the
    # first timed one) is not staged, H2D-submitted or prepared before t0.
    go = threading.Event()
    staged = [0]

    def stager():
        try:
            for i in range(total):
                if i == warmup:
                    go.wait()
                slot = free.get()
                sealed = time.perf_counter()
                raw = raws[i % len(raws)]
                hb = views[slot]
                if ingest == "utf8":
                    hb.load_utf8(raw, u8s[i % len(raws)], copy_text=False)
                elif ingest == "utf16":
                    hb.load_utf16(raw, copy_text=False)
                else:
                    hb.load(raw, "wire")
                eng.submit(hb, slot)
                staged[0] = i + 1
                ready.put((slot, sealed, time.perf_counter() - sealed))
        except BaseException as e:   # surfaced by the main thread
            err.append(e)
            ready.put(None)

    th = threading.Thread(target=stager, name="stager", daemon=True)
    th.start()
    host_ms = []

    def run(n, record):
        for _ in range(n):
            item = ready.get()
            if item is None:
                raise err[0]
            slot, sealed, stage_s = item
            res = r.process(slot)
            done = time.perf_counter()
            free.put(slot)
            if record:
                r.record(res, sealed, done)
                host_ms.append(stage_s * 1e3)

    def timed():
        r.prestaged_at_t0 = max(0, staged[0] - warmup)
        go.set()
        run(steps, True)

    run(warmup, False)
    t0, t1 = sync(timed)
    th.join(timeout=60)
    r.host_stage_ms = float(np.median(host_ms)) if host_ms else 0.0
    return t0, t1


def lr_config(args, rows: int, max_units: int, ingest: str, dp: bool = False, raw_slots: int = 0):
    from twitter_stream_ml_amd.ops.lr_engine import LRDeviceConfig
    return LRDeviceConfig(num_text_features=args.features, hash=args.hash,
                          step_size=args.step_size, num_iterations=args.iters, fraction=1.0,
                          begin=100, end=1000, max_rows=rows, max_units=max_units,
                          sgd_grid=args.sgd_grid, ablate=args.ablate, tol=args.tol, dedup=bool(args.dedup),
                          hybrid=bool(args.hybrid), ingest=ingest if args.e2e else "wire",
                          force_dp=bool(getattr(args, "force_dp", False)),
                          # the per-iteration gradient all-reduce is timed whenever the
                          # engine is in DP (events around it on the compute stream)
                          comm_timing=dp or bool(getattr(args, "force_dp", False)),
                          raw_slots=raw_slots or (4 if str(args.batch).lower() == "hbm" else 0))


def hbm_batch(args, synth, device: int, ingest: str):
    """--batch hbm: micro-batch rows from the engine's measured footprint and
    the GPU's free memory (ops/sizing.py); units per row from a sample."""
    import torch
    from twitter_stream_ml_amd.ops.lr_engine import DeviceLinearRegression
    from twitter_stream_ml_amd.ops.sizing import hbm_max_rows
    from twitter_stream_ml_amd.sources.synthetic import generate_batch
    if args.model != "lr":
        raise SystemExit("--batch hbm sizes the LR engine (config 5)")
    sample = generate_batch(synth, 0, 65536, batch_time_ms=synth.now_ms)
    upr = 1.1 * sample.total_units / max(1, sample.n)   # units per row, 10 % margin

    def make(rows: int):
        return DeviceLinearRegression(lr_config(args, rows, int(rows * upr) + 1024, ingest), device=device)

    free, total = torch.cuda.mem_get_info(device)
    rows = hbm_max_rows(make, free, args.hbm_fraction)
    B = min(rows, args.batch_cap)
    return B, {"rule": f"hbm: {args.hbm_fraction:.2f} x {free / 2**30:.0f} GiB free of {total / 2**30:.0f} GiB",
               "hbm_max_rows": rows, "batch_cap": args.batch_cap}


def final_model(eng, is_km: bool) -> np.ndarray:
    """The replicated model state every DP rank must hold bit for bit."""
    if is_km:
        c, w = eng.get_state()
        return np.concatenate([np.asarray(c, np.float64).ravel(), np.asarray(w, np.float64).ravel()])
    return np.asarray(eng.get_weights())


def rccl_version() -> str:
    try:
        from twitter_stream_ml_amd.ops._native import hip
        return str(hip().rccl_version())
    except Exception as e:   # noqa: BLE001 -- informational
        return f"unknown ({e})"


def start_watchdog(timeout_s: float, comm, rank: int):
    """Whole-run watchdog (--timeout): a rank whose run does not finish in
    time (a peer died inside a collective, a hung device) dumps every
    thread's Python stack and its communicator counters to stderr, aborts
    the communicator (RCCL: ncclCommAbort, so peers blocked in a collective
    error out too) and exits with EXIT_HUNG -- the driver sees a non-zero
    exit long before its own timeout.  No re-exec."""
    if not timeout_s or timeout_s <= 0:
        return None
    import faulthandler
    from twitter_stream_ml_amd.utils.faults import EXIT_HUNG, Watchdog

    def on_timeout() -> None:
        try:
            sys.stderr.write(f"[bench rank {rank}] watchdog: run not finished after {timeout_s:.0f} s; "
                             "Python stacks:\n")
            faulthandler.dump_traceback(file=sys.stderr, all_threads=True)
            if comm is not None:
                sys.stderr.write(f"[bench rank {rank}] comm {comm.kind} world {comm.world} counters "
                                 f"{dict(comm.counters())}\n")
            sys.stderr.flush()
            if comm is not None:
                comm.abort()
        finally:
            os._exit(EXIT_HUNG)

    wd = Watchdog(timeout_s, on_timeout, name="bench run")
    wd.arm()
    return wd


def run_cpu_local(args) -> int:
    """BASELINE config 1: ``--master local[N]`` -- the reference's own mode
    (``ConfArguments.scala:54-56``, README ``local[2]``): the fp64 CPU engine
    (``models/linear_regression.py CpuLinearRegression``, MLlib 1.6.1
    semantics of ``LinearRegression.scala:36-91``) trains the same synthetic
    tweets as the GPU line.  N host threads, one of which stands for Spark's
    receiver (as in local mode), so the featurizer and the GD loop get N - 1.
    A step = one micro-batch: featurize (filter, lower-case, bigram hashing),
    prequential predict + stats, GD to convergence; the latency of a batch is
    its step (the CPU engine has no queue).  The batch is smaller than the
    GPU line's (``--batch``, default 50000 here) and the JSON says so."""
    import re
    m = re.fullmatch(r"local\[(\d+|\*)\]", args.master)
    if not m:
        print(f"--master {args.master}: expected local[N]", file=sys.stderr)
        return 2
    n_thr = os.cpu_count() or 1 if m.group(1) == "*" else int(m.group(1))
    workers = max(1, n_thr - 1)
    os.environ["TWTML_HOST_THREADS"] = str(workers)
    from twitter_stream_ml_amd.models.linear_regression import CpuLinearRegression, CpuLRConfig
    from twitter_stream_ml_amd.sources.synthetic import SynthConfig, generate_batch
    B = 50_000 if str(args.batch) == "1000000" else int(args.batch)
    synth = SynthConfig.profile(args.profile, seed=args.seed)
    n_pool = args.warmup + args.steps
    t_gen = time.time()
    pool = [generate_batch(synth, i * B, B, batch_time_ms=synth.now_ms) for i in range(n_pool)]
    t_gen = time.time() - t_gen
    eng = CpuLinearRegression(CpuLRConfig(num_text_features=args.features, hash=args.hash,
                                          step_size=args.step_size, num_iterations=args.iters, fraction=1.0,
                                          tol=args.tol, begin=100, end=1000))
    lat, kept, iters = [], [], []
    for i, raw in enumerate(pool):
        if i == args.warmup:
            t0 = time.perf_counter()
        s = time.perf_counter()
        res = eng.train_batch(raw, want_pred=False)
        if i >= args.warmup:
            lat.append((time.perf_counter() - s) * 1e3)
            kept.append(res["n_kept"])
            iters.append(res["iterations"])
    t1 = time.perf_counter()
    value = float(sum(kept)) / (t1 - t0)
    out = {
        "metric": "tweets/sec trained (whole node)",
        "value": round(value, 1),
        "unit": "tweets/s",
        "n_gpus": 0,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round((t1 - t0) / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": round(value / BASELINE_TWEETS_PER_SEC, 3),
        "dtype": "fp64",
        "data": (f"synthetic tweet-shaped records (seeded C++ generator, "
                 f"{'realistic 50K-word multi-script' if args.profile == 'wide' else 'toy ~300-word'} vocabulary, "
                 f"{n_pool} distinct batches), zero-init weights"),
        "config": {
            "model": f"StreamingLinearRegressionWithSGD, {args.features}-dim hashed bigrams + 4 numeric",
            "global_batch": B, "seq_len": 280, "parallelism": f"cpu {args.master}",
            "numIterations": args.iters, "stepSize": args.step_size, "miniBatchFraction": 1.0,
            "hash": args.hash, "profile": args.profile,
            "batch_note": f"{B} tweets per micro-batch (the GPU line trains 1M per GPU per step)",
        },
        "baseline_config": "BASELINE.json config 1: --master local[2] CPU, synthetic tweet source",
        "engine": "fp64 CPU engine (MLlib 1.6.1 semantics, oracle/mllib.py run_minibatch_sgd over scipy CSR; "
                  "native C++ featurizer)",
        "host_threads": workers,
        "gd_iterations_mean": float(np.mean(iters)) if iters else 0.0,
        "p50_microbatch_latency_ms": round(float(np.median(lat)), 3),
        "trained_tweets_per_step": round(float(np.mean(kept)), 1),
        "pool_gen_s": round(t_gen, 2),
        "wall_s": round(time.time() - T_START, 1),
    }
    line = json.dumps(out)
    print(line, flush=True)
    if args.json_out:
        with open(args.json_out, "w") as fh:
            fh.write(line + "\n")
    return 0


def main(argv=None) -> int:
    args = parse_args(argv)
    if args.master:   # config 1: the CPU engine (local[N] only)
        return run_cpu_local(args)
    args.e2e = not args.prepacked
    import torch  # noqa: F401  (binds the HIP runtime before the engine loads)
    from twitter_stream_ml_amd.parallel import dist as D
    from twitter_stream_ml_amd.ops.lr_engine import (DeviceLinearRegression, HostBatchView,
                                                     LRDeviceConfig, encode_utf8, register_host)
    from twitter_stream_ml_amd.records.batch import RawBatch
    from twitter_stream_ml_amd.sources.synthetic import SynthConfig, generate_batch

    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    if world_env != args.gpus:
        if args.gpus > 1 and world_env == 1:
            print(f"--gpus {args.gpus} needs torch.distributed.run with {args.gpus} processes",
                  file=sys.stderr)
            return 2
    info = D.init_distributed(backend="gloo" if args.comm == "gloo" else None)
    n_dev = max(1, torch.cuda.device_count())
    device = info.local_rank % n_dev   # gloo comm: several ranks may share a GPU
    torch.cuda.set_device(device)
    from twitter_stream_ml_amd.parallel.affinity import bind_local_numa
    numa_cpus = bind_local_numa(device)   # before the pinned pool is allocated
    from twitter_stream_ml_amd.parallel.affinity import share_host_threads
    host_threads = share_host_threads(device, info.local_rank,
                                      int(os.environ.get("LOCAL_WORLD_SIZE", info.world)), n_dev)
    # one communicator: LR DP issues one int64 all-reduce per GD iteration and
    # one all-gather of the next batch's prep packets per batch
    if args.force_dp and (info.world > 1 or args.comm != "rccl"):
        print("--force-dp is a world-1 RCCL mode", file=sys.stderr)
        return 2
    comm = D.make_comm(device, args.comm, force=args.force_dp)
    watchdog = start_watchdog(args.timeout, comm, info.rank)
    ingest = args.ingest or "utf8"

    synth = SynthConfig.profile(args.profile, seed=args.seed + 7919 * info.rank)
    now_ms = synth.now_ms
    sizing = None
    if str(args.batch).lower() == "hbm":
        B, sizing = hbm_batch(args, synth, device, ingest)
        B = int(D.allreduce_max_scalar(-float(B)) * -1)   # the smallest over ranks
    else:
        B = int(args.batch)
    t_gen = time.time()
    n_pool = args.pool if args.pool > 0 else args.warmup + args.steps
    if args.pool <= 0:   # fresh batches for every step, within a host-memory budget of pooled tweets
        n_pool = max(1, min(n_pool, int(os.environ.get("TWTML_BENCH_POOL_TWEETS", "64000000")) // max(1, B)))
    pool_raw = [generate_batch(synth, i * B, B, batch_time_ms=now_ms) for i in range(n_pool)]
    max_units = max(r.total_units for r in pool_raw) + 1024
    is_km = args.model == "kmeans"
    if is_km:
        from twitter_stream_ml_amd.ops.kmeans_engine import DeviceKMeans, KMDeviceConfig
        kcfg = KMDeviceConfig(k=args.k, text_dims=args.text_dims, half_life=5.0, max_rows=B,
                              max_units=max_units, seed=args.seed, force_dp=args.force_dp)
        eng = DeviceKMeans(kcfg, device=device, comm=comm)
    else:
        eng = DeviceLinearRegression(lr_config(args, B, max_units, ingest, dp=comm is not None), device=device,
                                     comm=comm)
    u8s = []
    pinned = 0   # bytes of page-locked host memory this rank holds (staging views + registered pool)
    if args.e2e:
        # utf8 / utf16 ingest DMAs the text from the receiver's registered
        # buffers: the staging views hold row words and scalars only
        views = [HostBatchView(B, max_units, text=ingest == "wire") for _ in range(eng.raw_slots)]
        pinned += sum(int(v._hb.bytes) for v in views)
        if is_km:
            for v in views:
                v._hb.scalar_cols = 2   # k-means reads retweetCount and followersCount only
        if ingest == "utf8" and is_km and args.text_dims == 0:   # 2 scalar features: no text needed
            from twitter_stream_ml_amd.ops.kmeans_engine import no_text
            u8s = [no_text(r) for r in pool_raw]
        elif ingest == "utf8":   # the receiver's UTF-8 buffers (as the network delivered them)
            u8s = [encode_utf8(r) for r in pool_raw]
            for u in u8s:
                register_host(u.data)
                pinned += int(u.data.nbytes)
            # the UTF-16 copy is not staged in this mode: drop it (the batch
            # carries the receiver's UTF-8 buffer instead)
            pool_raw = [RawBatch(np.zeros(0, np.uint16), r.offsets, r.is_retweet, r.scalars, r.batch_time_ms,
                                 utf8=u) for r, u in zip(pool_raw, u8s)]
        elif ingest == "utf16":
            for r in pool_raw:   # the receiver's buffers: DMA source of the text
                register_host(r.text)
                pinned += int(r.text.nbytes)
        # the receiver records each sealed batch's scalar column bounds (one-pass
        # wire encoding in the staging, every value still checked against them)
        for r in pool_raw:
            r.with_scalar_range()
    else:
        pool = []
        for r in pool_raw:
            v = HostBatchView(B, max_units)
            pinned += int(v._hb.bytes)
            if is_km:
                v._hb.scalar_cols = 2
            pool.append(v.load(r))
        del pool_raw
    t_gen = time.time() - t_gen
    runner = Runner(eng, is_km, now_ms)
    hang = os.environ.get("TWTML_BENCH_HANG", "")
    if hang and int(hang.split(":")[0]) == info.rank:
        runner.hang_at = int(hang.split(":")[1])

    h2d = {}
    # TWTML_H2D_TIMING=1: events on the copy stream at the window's ends (diagnostics)
    wmark = getattr(getattr(eng, "_eng", None), "h2d_window_mark", None) \
        if os.environ.get("TWTML_H2D_TIMING") == "1" else None

    def sync(fn):
        eng.synchronize()
        D.barrier()
        torch.cuda.synchronize()
        h2d["b0"] = eng.h2d_bytes
        if wmark:
            wmark()
        t0 = time.perf_counter()
        fn()
        eng.synchronize()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        if wmark:
            wmark()
        h2d["b1"] = eng.h2d_bytes
        D.barrier()
        return t0, t1

    if args.e2e:
        t0, t1 = run_e2e(runner, pool_raw, u8s, views, ingest, args.warmup, args.steps, sync)
    else:
        t0, t1 = run_device_pipeline(runner, pool, args.warmup, args.steps, sync)
    # DP replicas must be bit-identical after the run (SURVEY §5 race detection)
    replicas = D.replicas_identical(final_model(eng, is_km))
    elapsed = D.allreduce_max_scalar(t1 - t0)
    tweets = D.allreduce_sum_scalar(float(sum(runner.kept)))
    p50 = D.allreduce_max_scalar(float(np.median(runner.lat)))
    value = tweets / elapsed
    ms = elapsed / args.steps * 1e3
    mine = float(sum(runner.kept)) / max(t1 - t0, 1e-12)   # this rank's own tweets/s over its window
    per_rank = D.gather_to_main(np.array([mine]))
    prestaged = int(D.allreduce_max_scalar(float(runner.prestaged_at_t0)))
    # host-link floor: the timed window's H2D bytes (engine counter) over this
    # box's pinned host-to-device bandwidth (measured here, after the window)
    moved = float(h2d.get("b1", 0) - h2d.get("b0", 0))
    gbps = D.allreduce_min_scalar(_h2d_gbps(device))
    import resource
    rss_mb = resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 1024.0
    host = D.gather_to_main(np.array([rss_mb, pinned / 2**20, t_gen]))   # per rank, to rank 0
    stage = runner.stage
    par = f"dp{info.world}" + ("-gloo" if args.comm == "gloo" else "") + ("-forced" if args.force_dp else "")
    data = ("synthetic tweet-shaped records (seeded C++ generator, "
            f"{'realistic 50K-word multi-script' if args.profile == 'wide' else 'toy ~300-word'} vocabulary, "
            + (f"{n_pool} distinct batches per rank: no batch is trained twice)"
               if n_pool >= args.warmup + args.steps else f"{n_pool} batches per rank, replayed)"))
    out = {
        "metric": "tweets/sec trained (whole node)",
        "value": round(value, 1),
        "unit": "tweets/s",
        "n_gpus": info.world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms, 3),
        "higher_is_better": True,
        "scaling": "weak",
        # against config 1 (the LR model on the CPU, local[2]); k-means has no CPU line
        "vs_baseline": (round(value / BASELINE_TWEETS_PER_SEC, 1)
                        if BASELINE_TWEETS_PER_SEC and not is_km else None),
        "dtype": "fp32",
    }
    if is_km:
        out["data"] = data + ", N(0,1) random centres"
        out["config"] = {
            "model": f"StreamingKMeans k={args.k}, d={2 + args.text_dims} "
                     f"([retweetCount, followers] + {args.text_dims} hashed bigram dims), "
                     "halfLife 5 batches, per-batch StandardScaler",
            "global_batch": B * info.world, "seq_len": 280, "parallelism": par,
        }
        out["device_ms_mean"] = float(np.mean([s[0] for s in stage])) if stage else 0.0
    else:
        out["data"] = data + ", zero-init weights"
        out["config"] = {
            "model": f"StreamingLinearRegressionWithSGD, {args.features}-dim hashed bigrams + 4 numeric",
            "global_batch": B * info.world, "seq_len": 280, "parallelism": par,
            "numIterations": args.iters, "stepSize": args.step_size, "miniBatchFraction": 1.0,
            "hash": args.hash, "profile": args.profile,
        }
        if sizing:
            out["config"]["batch_sizing"] = sizing
        out["gd_iterations_mean"] = float(np.mean(runner.iters)) if runner.iters else 0.0
        out["prep_ms_mean"] = float(np.mean([s[0] for s in stage])) if stage else 0.0
        out["train_ms_mean"] = float(np.mean([s[1] for s in stage])) if stage else 0.0
        if runner.extra:
            out["tiered"] = bool(runner.extra[-1][0])
            out["active_features"] = int(np.mean([e[1] for e in runner.extra]))
            out["lds_tier_features"] = int(runner.extra[-1][2])
    out["p50_microbatch_latency_ms"] = round(p50, 3)
    if out["vs_baseline"] is not None:
        out["baseline"] = {"config": "BASELINE.json config 1: --master local[2] CPU (fp64 MLlib-semantics engine), "
                                     "same synthetic data, 50K-tweet batches",
                           "tweets_per_sec": BASELINE_TWEETS_PER_SEC, "source": "profiles/r6/config1_local2.json"}
    out["trained_tweets_per_step"] = round(tweets / args.steps, 1)
    out["ingest"] = (f"e2e-{ingest}: host staging of every batch in the timed region (scalar column bounds "
                     "recorded by the receiver when it sealed the batch)"
                     if args.e2e else "device pipeline: pre-packed wire pool, H2D in the timed region")
    if args.e2e:
        out["host_stage_ms_p50"] = round(getattr(runner, "host_stage_ms", 0.0), 3)
    # the engine communicator's own view: the world it spans and the
    # collectives it carried (so a scaling run shows RCCL saw N ranks)
    out["comm_world"] = int(comm.world) if comm is not None else 1
    out["comm_kind"] = str(comm.kind) if comm is not None else "none"
    if comm is not None:
        out["comm_counters"] = {k: int(v) for k, v in comm.counters().items()}
    if per_rank is not None:
        out["per_rank_value"] = [round(float(v), 1) for v in per_rank]
    out["prestaged_at_t0"] = prestaged
    # device raw-batch slots: the H2D runs up to raw_slots - 1 batches ahead of
    # the batch training (throughput vs queueing latency: TWTML_RAW_SLOTS)
    out["raw_slots"] = int(eng.raw_slots)
    if moved > 0:
        out["h2d_bytes_per_tweet"] = round(moved / (args.steps * B), 1)
        out["h2d_gbps"] = round(gbps, 1)
        out["h2d_floor_ms_per_step"] = round(moved / args.steps / (gbps * 1e9) * 1e3, 3) if gbps > 0 else None
    # TWTML_H2D_TIMING=1 (diagnostics): the copy stream's busy time and gaps
    # over the timed batches (their submits are the last args.steps ones)
    native = getattr(eng, "_eng", None)
    if os.environ.get("TWTML_H2D_TIMING") == "1" and native is not None and hasattr(native, "h2d_timeline"):
        tl = native.h2d_timeline()[-args.steps:]
        win = native.h2d_window()[-2:]
        if tl:
            busy = sum(e - a for _, a, e, _ in tl)
            gaps = [tl[i + 1][1] - tl[i][2] for i in range(len(tl) - 1)]
            out["h2d_timeline"] = {
                "batches": len(tl), "busy_ms": round(busy, 3), "span_ms": round(tl[-1][2] - tl[0][1], 3),
                "gap_ms_total": round(sum(gaps), 3), "gap_ms_max": round(max(gaps), 3) if gaps else 0.0,
                "gbps_while_busy": round(sum(b for _, _, _, b in tl) / (busy * 1e6), 2) if busy > 0 else None,
                "per_batch_ms": [round(e - a, 3) for _, a, e, _ in tl],
                # per gap: the part the copy stream waited for the slot's previous batch
                # (start - queued) and the part no copy was queued yet (host late)
                "gaps_ms": [round(g, 3) for g in gaps],
                "slot_wait_ms": [round(tl[i + 1][1] - max(tl[i + 1][0], tl[i][2]), 3) for i in range(len(tl) - 1)],
                "host_late_ms": [round(max(0.0, tl[i + 1][0] - tl[i][2]), 3) for i in range(len(tl) - 1)]}
            # host clock, ms from t0: a batch's staging start and its process() return
            out["h2d_timeline"]["host_sealed_ms"] = [round((a - t0) * 1e3, 3) for a, _ in runner.marks]
            out["h2d_timeline"]["host_done_ms"] = [round((b - t0) * 1e3, 3) for _, b in runner.marks]
            out["h2d_timeline"]["iterations"] = [int(x) for x in runner.iters]
            out["h2d_timeline"]["prep_ms"] = [round(float(a), 3) for a, _ in runner.stage]
            out["h2d_timeline"]["train_ms"] = [round(float(b), 3) for _, b in runner.stage]
            # engine phases (ms): host pre-GD enqueue, GD loop, post-GD enqueue + sync, result read;
            # device pre-GD kernels, post-GD kernels
            if runner.phases:
                out["h2d_timeline"]["phases_ms"] = [[round(float(x), 3) for x in p[:6]] for p in runner.phases]
            if len(win) == 2:   # the window's ends against the first copy's start / the last copy's end
                out["h2d_timeline"].update(
                    window_ms=round(win[1] - win[0], 3), first_copy_start_ms=round(tl[0][1] - win[0], 3),
                    first_copy_queued_ms=round(tl[0][0] - win[0], 3),
                    after_last_copy_ms=round(win[1] - tl[-1][2], 3))
    if runner.comm and sum(c[0] for c in runner.comm) > 0:
        n_ar = sum(c[0] for c in runner.comm)
        out["grad_allreduce_per_step"] = round(n_ar / len(runner.comm), 2)
        # events around every gradient all-reduce (timed whenever the engine is in DP); the max over ranks
        out["grad_allreduce_us_per_iter"] = round(D.allreduce_max_scalar(
            1e3 * sum(c[1] for c in runner.comm) / n_ar), 2)
        out["allreduce_bytes_per_iter"] = int(round(sum(c[2] for c in runner.comm) / n_ar))
        # gradient all-reduce time per timed step (max over ranks): the DP cost model's check
        out["comm_ms_per_step"] = round(D.allreduce_max_scalar(sum(c[1] for c in runner.comm) / len(runner.comm)), 3)
    out["replicas_identical"] = bool(replicas)
    if comm is not None:
        out["rccl_version"] = rccl_version()
        out["comm_env"] = {k: v for k, v in sorted(os.environ.items())
                           if k.startswith(("NCCL_", "RCCL_", "HSA_ENABLE_IPC"))}
    if host is not None:   # the host budget of every rank (8-rank rehearsal, README)
        h = np.asarray(host).reshape(-1, 3)
        out["per_rank_host"] = [{"peak_rss_mb": round(float(a), 1), "pinned_mb": round(float(b), 1),
                                 "pool_gen_s": round(float(c), 2)} for a, b, c in h]
    out["wall_s"] = round(time.time() - T_START, 1)
    out["pool_gen_s"] = round(t_gen, 2)
    out["pool_batches"] = n_pool
    out["numa_bound_cpus"] = len(numa_cpus) if numa_cpus else None
    out["host_threads"] = host_threads
    if info.is_main:
        line = json.dumps(out)
        print(line, flush=True)
        if args.json_out:
            with open(args.json_out, "w") as fh:
                fh.write(line + "\n")
    if watchdog is not None:
        watchdog.close()
    D.shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
