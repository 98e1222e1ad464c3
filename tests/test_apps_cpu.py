"""End-to-end driver runs on the CPU engine (local[N]) with real report sinks.

The reference has no driver tests; these run the LinearRegression
and KMeans jobs for a few micro-batches against the in-process twtml-web
server and a fake Lightning server, and check what reaches both.
"""
import json
import os

import numpy as np
import pytest

from twitter_stream_ml_amd.apps import kmeans as km_app
from twitter_stream_ml_amd.apps import linear_regression as lr_app
from twitter_stream_ml_amd.checkpoint import load_kmeans, load_linear_regression
from twitter_stream_ml_amd.report.api_types import Stats
from twitter_stream_ml_amd.report.webclient import WebClient
from twitter_stream_ml_amd.web.main import build_server

from fakes import FakeLightning


@pytest.fixture()
def sinks(tmp_path):
    lgn = FakeLightning().start()
    web = build_server(["-nocache"], port=0, host="127.0.0.1",
                       backup_file=str(tmp_path / "w.json")).start()
    yield lgn, web
    web.stop()
    lgn.stop()


def test_linear_regression_driver_cpu(sinks, tmp_path, monkeypatch):
    lgn, web = sinks
    metrics = tmp_path / "m.jsonl"
    monkeypatch.setenv("TWTML_METRICS", str(metrics))
    ck = tmp_path / "model"
    rc = lr_app.main(["--master", "local[2]", "--lightning", lgn.url, "--twtweb", web.url,
                      "--seconds", "0.3", "--sourceRate", "4000", "--numBatches", "3",
                      "-f", "1000", "--checkpoint", str(ck), "--checkpointInterval", "2"])
    assert rc == 0
    recs = [json.loads(l) for l in open(metrics)]
    summ = [r for r in recs if r.get("summary")]
    recs = [r for r in recs if not r.get("summary")]
    assert len(recs) == 3 and all(r["batch"] > 0 for r in recs)
    # the end-of-run throughput summary (rank 0)
    assert len(summ) == 1 and summ[0]["batches"] == 3 and summ[0]["tweets"] == sum(r["batch"] for r in recs)
    assert summ[0]["tweets_per_s"] > 0
    assert recs[-1]["count"] == sum(r["batch"] for r in recs)
    # twtml-web got Config (viz from Lightning) and the last batch's Stats
    cfg = WebClient(web.url).config()
    assert cfg.host == lgn.url and len(cfg.viz) == 1
    st = WebClient(web.url).stats()
    assert st.count == recs[-1]["count"] and st.batch == recs[-1]["batch"]
    assert st.mse == int(recs[-1]["mse"])
    # Lightning: session + viz creation + one append per batch (4 series)
    appends = lgn.appends()
    assert len(appends) == 3 and len(appends[0]["data"]["series"]) == 4
    w, b = load_linear_regression(str(ck))
    assert w.shape == (1004,) and b == 0.0 and np.abs(w).max() > 0


def test_linear_regression_driver_resume_and_dead_sinks(tmp_path, monkeypatch):
    metrics = tmp_path / "m.jsonl"
    monkeypatch.setenv("TWTML_METRICS", str(metrics))
    ck = tmp_path / "model"
    args = ["--master", "local[1]", "--lightning", "http://127.0.0.1:9",
            "--twtweb", "http://127.0.0.1:9", "--seconds", "0.2", "--sourceRate", "3000",
            "--numBatches", "2", "--checkpoint", str(ck)]
    assert lr_app.main(args) == 0            # unreachable report servers never stop training
    w1, _ = load_linear_regression(str(ck))
    assert lr_app.main(args + ["--resume", str(ck)]) == 0
    w2, _ = load_linear_regression(str(ck))
    assert not np.array_equal(w1, w2)


def test_kmeans_driver_cpu(sinks, tmp_path, monkeypatch):
    lgn, web = sinks
    (tmp_path / "application.conf").write_text(
        f'lightning="{lgn.url}"\ntwtweb="{web.url}"\n')
    monkeypatch.setenv("TWTML_CONFIG_PATH", str(tmp_path))
    ck = tmp_path / "km"
    rc = km_app.main(["--seconds", "0.3", "--sourceRate", "3000", "--numBatches", "3",
                      "--checkpoint", str(ck), "--report"])
    assert rc == 0
    c, w = load_kmeans(str(ck))
    assert c.shape == (3, 2) and w is not None and w.sum() > 0
    assert any(p == "/sessions/" for (_, p, _) in lgn.calls)
    assert WebClient(web.url).stats().count > 0


def test_cpu_drivers_on_replayed_utf8_batches(tmp_path, monkeypatch):
    """``replay:synthetic`` batches carry only their UTF-8
    bytes (empty UTF-16 text); the CPU engines must decode them, not read
    past a zero-length text array."""
    metrics = tmp_path / "m.jsonl"
    monkeypatch.setenv("TWTML_METRICS", str(metrics))
    args = ["--master", "local[1]", "--lightning", "http://127.0.0.1:9", "--twtweb", "http://127.0.0.1:9",
            "--source", "replay:synthetic:bench:2", "--batchSize", "600", "--seconds", "0",
            "--sourceRate", "0", "--numBatches", "2", "-f", "1000"]
    assert lr_app.main(args) == 0
    recs = [json.loads(l) for l in open(metrics) if '"summary"' not in l]
    assert len(recs) == 2 and all(r["batch"] > 0 for r in recs)
    monkeypatch.setenv("TWTML_METRICS", str(tmp_path / "k.jsonl"))
    assert km_app.main(["--master", "local[1]", "--source", "replay:synthetic:bench:2", "--batchSize", "600",
                        "--seconds", "0", "--sourceRate", "0", "--numBatches", "2", "--textDims", "6"]) == 0


def test_featurize_rows_rejects_offsets_beyond_text():
    from twitter_stream_ml_amd.ops._native import host
    with pytest.raises(ValueError, match="exceed"):
        host().featurize_rows(np.zeros(0, np.uint16), np.array([0, 5, 9], np.int64),
                              np.array([0, 1], np.int64), 1000, "java", 0)


def test_lightning_numpy_append_matches_list_payload():
    """The pre-encoded append (``_twtml_host.json_floats``, GIL released) posts
    the same JSON as the list path: shortest round-trip floats, NaN -> null,
    the optional keys after the series."""
    from twitter_stream_ml_amd.report.lightning import Lightning, _json_floats
    x = np.array([0.0, -0.0, 0.1, 1 / 3, 1e-310, 1.7976931348623157e308, 123456789012345.0, np.nan, np.inf])
    assert json.loads(_json_floats(x)) == [v if np.isfinite(v) else None for v in x.tolist()]
    r = np.random.default_rng(0).standard_normal(5000) * 1e3
    assert json.loads(_json_floats(r)) == r.tolist()
    lgn = FakeLightning().start()
    try:
        cli = Lightning(lgn.url)
        viz = cli.line_streaming(series=[[0.0]] * 2)
        series = [r[:100], np.full(100, 2.5)]
        cli.line_streaming(series=series, viz=viz)                             # numpy: pre-encoded
        cli.line_streaming(series=[s.tolist() for s in series], viz=viz)      # lists: json=
        cli.line_streaming(series=series, size=[1.0, 2.0], xaxis="t", viz=viz)
        a = lgn.appends()
    finally:
        lgn.stop()
    assert a[0] == a[1] and a[0]["data"]["series"][0] == r[:100].tolist()
    assert a[2]["data"]["size"] == [1.0, 2.0] and a[2]["data"]["xaxis"] == "t"
