"""MLlib Saveable checkpoints at the wide config (F = 1e8 weights)."""
import json
import os
import time

import numpy as np
import pyarrow.parquet as pq

from twitter_stream_ml_amd.checkpoint.saveable import (load_kmeans, load_linear_regression, save_kmeans,
                                                       save_linear_regression)
from twitter_stream_ml_amd.checkpoint.stream_state import resolve_resume


def test_lr_checkpoint_1e8_sparse_roundtrip(tmp_path):
    """1e8 + 4 weights with 300K non-zeros (a hashed-text model: only touched
    bigrams move) -> sparse VectorUDT; save + load well under 20 s and
    without materialising Python floats."""
    F = 100_000_000
    rng = np.random.default_rng(0)
    w = np.zeros(F + 4)
    idx = np.unique(rng.integers(0, F + 4, 300_000))
    w[idx] = rng.standard_normal(idx.shape[0])
    path = str(tmp_path / "lr")
    t0 = time.time()
    save_linear_regression(path, w, 0.0, {"batches": 3})
    t1 = time.time()
    w2, b = load_linear_regression(path)
    t2 = time.time()
    assert t1 - t0 < 20 and t2 - t1 < 20, (t1 - t0, t2 - t1)
    assert b == 0.0 and w2.shape == w.shape and np.array_equal(w2, w)
    size = os.path.getsize(os.path.join(path, "data", "part-00000.parquet"))
    assert size < 16 * idx.shape[0] + (1 << 20)   # sparse on disk, not 800 MB
    t = pq.read_table(os.path.join(path, "data", "part-00000.parquet"))
    row = t.column("weights")[0].as_py() if idx.shape[0] < 10 else None
    assert t.column("weights").chunk(0).field("type")[0].as_py() == 0
    meta = json.loads(t.schema.metadata[b"org.apache.spark.sql.parquet.row.metadata"])
    assert meta["fields"][0]["type"]["class"] == "org.apache.spark.mllib.linalg.VectorUDT"
    assert row is None


def test_dense_vectors_and_kmeans_roundtrip(tmp_path):
    rng = np.random.default_rng(1)
    w = rng.standard_normal(1004)
    save_linear_regression(str(tmp_path / "d"), w, 0.5)
    w2, b = load_linear_regression(str(tmp_path / "d"))
    assert b == 0.5 and np.array_equal(w, w2)
    t = pq.read_table(str(tmp_path / "d" / "data" / "part-00000.parquet"))
    assert t.column("weights").chunk(0).field("type")[0].as_py() == 1
    c = rng.standard_normal((1024, 64))
    c[3] = 0.0   # an all-zero centre stays a dense point (Spark writes centres dense)
    wt = rng.random(1024)
    save_kmeans(str(tmp_path / "k"), c, wt, {"batches": 2})
    c2, wt2 = load_kmeans(str(tmp_path / "k"))
    assert np.array_equal(c, c2) and np.array_equal(wt, wt2)


def test_resume_auto_falls_back_to_old_after_interrupted_replace(tmp_path):
    """A crash between the renames of a checkpoint replacement leaves only
    <path>.old: --resume auto must pick it up instead of retraining."""
    path = str(tmp_path / "ck")
    save_linear_regression(path, np.ones(8), 0.0, {"batches": 1})
    os.replace(path, path + ".old")           # state right after the first rename
    assert resolve_resume("auto", path) == path + ".old"
    w, _ = load_linear_regression(resolve_resume("auto", path))
    assert np.array_equal(w, np.ones(8))
    assert resolve_resume("auto", str(tmp_path / "none")) is None
