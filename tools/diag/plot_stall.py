"""Where a live Lightning plot costs the LR driver's training thread.

python tools/diag/plot_stall.py [--batches 40] [--switch-us 0,500]

Runs ``apps/linear_regression.py`` on the GPU engine (1M-tweet wide batches)
with plotting off (unreachable Lightning), then on against a fake Lightning
in a child process, once per GIL switch interval given, and prints the
percentiles of the per-batch metrics: ``step_ms`` (train + report on the
training thread), ``call_ms`` (the engine call) and ``gil_wait_ms`` (the part
of the call after the engine returned, spent taking the GIL back).
"""
import argparse
import functools
import json
import time
import os
import sys
import tempfile

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", type=int, default=40)
    ap.add_argument("--switch-us", default="0")
    ap.add_argument("--fresh-server", action="store_true", help="a new fake Lightning process per plot-on run")
    a = ap.parse_args()
    from fakes import FakeLightningProcess
    from twitter_stream_ml_amd.apps import linear_regression as app
    base = ["--master", "rocm[1]", "--twtweb", "http://127.0.0.1:9", "--source", "replay:synthetic:wide:4",
            "--seconds", "0", "--batchSize", "1000000", "--sourceRate", "0", "--numBatches", str(a.batches),
            "-f", "1000000"]
    default_si = sys.getswitchinterval()

    def cpu_stat():
        try:
            return {k: int(v) for k, v in (l.split() for l in open("/sys/fs/cgroup/cpu.stat"))}
        except OSError:
            return {}
    # timelines: the training thread's batches, the report threads' calls
    from twitter_stream_ml_amd.report import http as rhttp, lightning as lgm, session_stats as ssm
    ev = []

    def wrap(obj, name, tag=None):
        fn = getattr(obj, name)

        @functools.wraps(fn)
        def w(*x, **k):
            t0 = time.perf_counter()
            try:
                return fn(*x, **k)
            finally:
                ev.append((tag or name, t0, time.perf_counter()))
        setattr(obj, name, w)
    wrap(app.LinearRegressionJob, "on_batch", "BATCH")
    win = []   # cgroup cpu.stat at the start of batch 8 and after the last batch
    ob = app.LinearRegressionJob.on_batch

    def on_batch(self, *x, **k):
        if self.batches == 8:
            win.append(cpu_stat())
        try:
            return ob(self, *x, **k)
        finally:
            if self.batches == a.batches:
                win.append(cpu_stat())
    app.LinearRegressionJob.on_batch = on_batch
    import gc
    gc_t0 = {}

    def gc_cb(phase, info):
        if phase == "start":
            gc_t0[info["generation"]] = time.perf_counter()
        elif info["generation"] in gc_t0:
            ev.append((f"gc{info['generation']}", gc_t0.pop(info["generation"]), time.perf_counter()))
    gc.callbacks.append(gc_cb)
    wrap(lgm, "_json_floats")
    wrap(ssm.SessionStats, "_series")
    wrap(rhttp, "post", "http_post")
    # the training thread's own phases, and the receiver's seals
    from twitter_stream_ml_amd.ops import ingest, lr_engine
    from twitter_stream_ml_amd.runtime import streaming
    take0 = ingest.SlotPipeline.take

    def take(self, raw):
        hit = id(raw) in self._inflight
        t0 = time.perf_counter()
        try:
            return take0(self, raw)
        finally:
            ev.append(("take_hit" if hit else "take_MISS", t0, time.perf_counter()))
    ingest.SlotPipeline.take = take
    wrap(ingest.SlotPipeline, "prefetch")
    wrap(lr_engine.DeviceLinearRegression, "process")
    wrap(streaming.StreamingContext, "_seal")
    lgm.http_post = rhttp.post
    from twitter_stream_ml_amd.report import webclient as wcm
    wcm.http_post = rhttp.post

    def run(tag, lightning, si_us):
        sys.setswitchinterval(si_us / 1e6 if si_us > 0 else default_si)
        ev.clear()
        win.clear()
        import resource
        st0, ru0, w0 = cpu_stat(), resource.getrusage(resource.RUSAGE_SELF), time.perf_counter()
        path = os.path.join(tempfile.mkdtemp(), "m.jsonl")
        os.environ["TWTML_METRICS"] = path
        assert app.main(base + ["--lightning", lightning]) == 0
        st1, ru1, w1 = cpu_stat(), resource.getrusage(resource.RUSAGE_SELF), time.perf_counter()
        cpu = {k: st1[k] - st0.get(k, 0) for k in st1 if k in ("nr_periods", "nr_throttled", "throttled_usec", "usage_usec")}
        cpu["proc_cpu_s"] = round(ru1.ru_utime + ru1.ru_stime - ru0.ru_utime - ru0.ru_stime, 3)
        cpu["wall_s"] = round(w1 - w0, 3)
        if len(win) == 2:   # the streaming window (batches 8..end)
            cpu["window"] = {k: win[1][k] - win[0].get(k, 0) for k in win[1]
                             if k in ("nr_periods", "nr_throttled", "throttled_usec", "usage_usec")}
        recs = [json.loads(l) for l in open(path)]
        recs = [r for r in recs if "step_ms" in r]
        allrecs = recs
        recs = recs[8:]
        out = {"run": tag, "switch_us": si_us or default_si * 1e6, "cgroup_cpu": cpu}
        for k in ("step_ms", "call_ms", "gil_wait_ms", "train_ms"):
            v = np.array([r.get(k, np.nan) for r in recs], float)
            out[k] = {"p50": round(float(np.nanpercentile(v, 50)), 3), "p90": round(float(np.nanpercentile(v, 90)), 3),
                      "p99": round(float(np.nanpercentile(v, 99)), 3), "max": round(float(np.nanmax(v)), 3)}
        gcs = [(n, (y - x) * 1e3) for n, x, y in ev if n.startswith("gc")]
        out["gc"] = {g: [sum(1 for n, _ in gcs if n == g), round(max([d for n, d in gcs if n == g] or [0]), 3)]
                     for g in ("gc0", "gc1", "gc2")}
        print(json.dumps(out), flush=True)
        # the slow batches after warm-up, with the report calls overlapping them
        bt = [e for e in ev if e[0] == "BATCH"]
        med = float(np.median([b - a for _, a, b in bt[8:]]))
        for i, (_, a, b) in enumerate(bt):
            if i >= 8 and b - a > 1.5 * med:
                n_app = sum(1 for n, x, y in ev if n == "http_post" and y < a)
                print(f"  batch {i}: {n_app} posts done before it; metrics {allrecs[i] if i < len(allrecs) else None}")
                ov = [(n, round((x - a) * 1e3, 2), round((y - x) * 1e3, 2)) for n, x, y in ev
                      if n != "BATCH" and x < b and y > a]
                print(f"  slow batch {(b - a) * 1e3:.2f} ms (median {med * 1e3:.2f}): {ov}", flush=True)

    sis = [int(x) for x in a.switch_us.split(",")]
    run("off", "http://127.0.0.1:9", sis[0])
    lgn = FakeLightningProcess().start()
    try:
        for si in sis:
            if a.fresh_server:
                lgn.stop()
                lgn = FakeLightningProcess().start()
            run("on", lgn.url, si)
        print(json.dumps({"lightning": lgn.summary()}), flush=True)
    finally:
        lgn.stop()


if __name__ == "__main__":
    main()
