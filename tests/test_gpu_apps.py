"""End-to-end drivers on the MI355X engine (``--master rocm[1]``).

The same CLI run on the CPU engine (``local[1]``) and on the GPU engine must
produce the same model.  Both runs read batch times from a manual streaming
clock (``runtime/clock.py``, Spark's ManualClock), so every tweet's ``age``
feature is the same in both and ALL F+4 LR weights are compared; k-means
centres and weights agree to the rounding of the fp64 CPU sums (the GPU's
are exact integer sums).
"""
import numpy as np
import pytest

from twitter_stream_ml_amd.checkpoint import load_kmeans, load_linear_regression, load_progress

pytestmark = pytest.mark.gpu


def _lr_args(master, ck):
    return ["--master", master, "--lightning", "http://127.0.0.1:9", "--twtweb", "http://127.0.0.1:9",
            "--seconds", "0", "--batchSize", "3000", "--sourceRate", "0", "--numBatches", "4",
            "-f", "2048", "-i", "20", "--checkpoint", str(ck), "--checkpointInterval", "2"]


CLOCK = "manual:1700000000000:5000"


def _metrics(path):
    import json
    return [r for r in (json.loads(l) for l in open(path)) if not r.get("summary")]


def test_lr_driver_gpu_matches_cpu(hip_module, tmp_path, monkeypatch):
    """The fp64 CPU engine (MLlib semantics) and the fixed-point GPU engine
    run the same GD: per batch the same iteration count (early stop included),
    the same kept rows, and weights within 1e-6 of |w| (the bound of
    ``test_gpu_lr_engine.py`` for equal iteration counts)."""
    from twitter_stream_ml_amd.apps import linear_regression as app
    monkeypatch.setenv("TWTML_STREAMING_CLOCK", CLOCK)
    monkeypatch.setenv("TWTML_METRICS", str(tmp_path / "cpu.jsonl"))
    assert app.main(_lr_args("local[1]", tmp_path / "cpu")) == 0
    monkeypatch.setenv("TWTML_METRICS", str(tmp_path / "gpu.jsonl"))
    assert app.main(_lr_args("rocm[1]", tmp_path / "gpu")) == 0
    mc, mg = _metrics(tmp_path / "cpu.jsonl"), _metrics(tmp_path / "gpu.jsonl")
    assert len(mc) == len(mg) == 4
    for a, b in zip(mc, mg):
        assert (a["batch"], a["iterations"]) == (b["batch"], b["iterations"]), (a, b)
    w_cpu, _ = load_linear_regression(str(tmp_path / "cpu"))
    w_gpu, _ = load_linear_regression(str(tmp_path / "gpu"))
    assert load_progress(str(tmp_path / "gpu"))["batches"] == 4
    assert np.linalg.norm(w_gpu - w_cpu) <= 1e-6 * np.linalg.norm(w_cpu), \
        np.linalg.norm(w_gpu - w_cpu) / np.linalg.norm(w_cpu)   # age weight included


def test_lr_driver_gpu_resume_auto(hip_module, tmp_path):
    from twitter_stream_ml_amd.apps import linear_regression as app
    ck = tmp_path / "ck"
    args = _lr_args("rocm[1]", ck)
    args[args.index("--numBatches") + 1] = "2"
    assert app.main(args) == 0
    assert load_progress(str(ck))["batches"] == 2
    args[args.index("--numBatches") + 1] = "4"
    assert app.main(args + ["--resume", "auto"]) == 0
    assert load_progress(str(ck))["batches"] == 4


def test_kmeans_driver_gpu_matches_cpu(hip_module, tmp_path, monkeypatch):
    from twitter_stream_ml_amd.apps import kmeans as app
    monkeypatch.setenv("TWTML_STREAMING_CLOCK", CLOCK)
    base = ["--seconds", "0", "--batchSize", "2500", "--sourceRate", "0", "--numBatches", "3",
            "--k", "3", "--checkpointInterval", "1"]
    assert app.main(base + ["--master", "local[1]", "--checkpoint", str(tmp_path / "cpu")]) == 0
    assert app.main(base + ["--master", "rocm[1]", "--checkpoint", str(tmp_path / "gpu")]) == 0
    c_cpu, w_cpu = load_kmeans(str(tmp_path / "cpu"))
    c_gpu, w_gpu = load_kmeans(str(tmp_path / "gpu"))
    np.testing.assert_allclose(w_gpu, w_cpu, rtol=1e-12)              # same assignments
    np.testing.assert_allclose(c_gpu, c_cpu, rtol=1e-9, atol=1e-9 * np.abs(c_cpu).max())


def test_lr_driver_divergence_reported(hip_module, tmp_path, monkeypatch, caplog):
    """A step size far beyond stability (``-p 1e4``): MLlib's fp64 model goes
    to Inf/NaN and ``Utils.round`` throws (``Utils.scala:3-7``, called at
    ``LinearRegression.scala:63-65``).  The device engine stops training when
    its fixed-point scales leave the usable range; the driver must log it,
    mark the batches diverged in the metrics and never report them as a
    normal mse/stdev."""
    import json
    import logging
    from twitter_stream_ml_amd.apps import linear_regression as app
    metrics = tmp_path / "m.jsonl"
    monkeypatch.setenv("TWTML_METRICS", str(metrics))
    monkeypatch.setenv("TWTML_STREAMING_CLOCK", CLOCK)
    args = _lr_args("rocm[1]", tmp_path / "ck")
    args += ["-p", "10000"]
    caplog.set_level(logging.ERROR)
    assert app.main(args) == 0
    recs = [json.loads(l) for l in open(metrics)]
    batches = [r for r in recs if not r.get("summary")]
    summ = [r for r in recs if r.get("summary")]
    assert len(batches) == 4
    assert all(r.get("diverged") for r in batches), batches
    # the first batch's prequential pass ran on the zero model (MLlib would
    # report it: Utils.round of finite stats); later ones are never reported
    assert all("mse" not in r for r in batches[1:]), batches
    assert summ and summ[0]["diverged_batches"] == 4
    assert any("diverged" in m for m in caplog.messages), caplog.messages


def test_lr_driver_plot_does_not_stall_training(hip_module, tmp_path, monkeypatch, timing_margin):
    """with a live Lightning plot at 1M tweets per batch the
    training thread only enqueues a device-sampled series (plotPoints pairs,
    ``k_plot_sample``); the gather and the HTTP run on the plot shipper /
    session threads.  Per-batch p99 (train + report on the training thread)
    stays within 5 % of the plot-off run on the same data."""
    import json
    from fakes import FakeLightningProcess
    # 300 batches (292 measured): a p99 over 32 samples is nearly their
    # maximum, so one scheduler hiccup decided it (round 6, 92 samples:
    # margins -3.7 .. +5.9 % between attempts of the same tree)
    nb = 300
    base = ["--master", "rocm[1]", "--twtweb", "http://127.0.0.1:9", "--source", "replay:synthetic:wide:4",
            "--seconds", "0", "--batchSize", "1000000", "--sourceRate", "0", "--numBatches", str(nb),
            "-f", "1000000", "--plotPoints", "10000"]

    def p99(path, lightning):
        # each run in a fresh interpreter, as the driver runs: in one process
        # the second and third of the four runs each met one ~3.5-ms stall,
        # which set a 32-sample p99 whichever of off / on it landed in
        import os
        import subprocess
        import sys
        env = dict(os.environ, TWTML_METRICS=str(path))
        out = subprocess.run([sys.executable, "-m", "twitter_stream_ml_amd", *base, "--lightning", lightning],
                             env=env, capture_output=True, text=True, timeout=240)
        assert out.returncode == 0, (out.returncode, out.stderr[-4000:])
        recs = [r for r in (json.loads(l) for l in open(path)) if "step_ms" in r]
        assert len(recs) == nb
        for k in ("step_ms", "call_ms", "gil_wait_ms"):
            v = [r[k] for r in recs[8:]]
            print(f"{lightning} {k}: p50 {np.percentile(v, 50):.3f} p99 {np.percentile(v, 99):.3f} max {max(v):.3f}")
        return float(np.percentile([r["step_ms"] for r in recs[8:]], 99))   # after warm-up

    # A shared box's noise can move a p99 by more than the 5 %
    # bound (one suite run: both p50 and p99 of the plot-on run 13 % up);
    # a miss is measured once more, off and on, and the second pair decides.
    for attempt in (1, 2):
        off = p99(tmp_path / f"off{attempt}.jsonl", "http://127.0.0.1:9")   # unreachable: plotting disabled
        lgn = FakeLightningProcess().start()   # its JSON parsing off this process's GIL
        try:
            on = p99(tmp_path / f"on{attempt}.jsonl", lgn.url)
            summ = lgn.summary()
        finally:
            lgn.stop()
        assert summ["appends"] >= nb - 10 and summ["last_series_lens"] == [10000] * 4, summ
        print(f"step p99 (attempt {attempt}): plot off {off:.3f} ms, plot on {on:.3f} ms")
        timing_margin(f"plot-on step p99, attempt {attempt} (1.05 x plot-off + 0.05 ms)", on, 1.05 * off + 0.05)
        if on <= 1.05 * off + 0.05:
            break
    assert on <= 1.05 * off + 0.05, (on, off)
