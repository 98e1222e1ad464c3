"""Non-blocking checkpoints (apps/_common.py StreamCheckpointer) and the sparse
weight path of the Saveable writer (checkpoint/saveable.py SparseWeights).

The reference never checkpoints; the format is MLlib's
``GLMRegressionModel.SaveLoadV1_0`` layout, tested in test_checkpoint*.py.
"""
import threading
import time

import numpy as np
import pytest

from twitter_stream_ml_amd.apps._common import StreamCheckpointer
from twitter_stream_ml_amd.checkpoint import (SparseWeights, load_linear_regression, load_progress,
                                              save_linear_regression)


def test_sparse_weights_round_trip(tmp_path):
    rng = np.random.default_rng(0)
    size = 1_000_004
    idx = np.sort(rng.choice(size, 5000, replace=False)).astype(np.int32)
    val = rng.normal(size=5000)
    save_linear_regression(str(tmp_path / "m"), SparseWeights(size, idx, val), 0.0, {"batches": 3})
    w, b = load_linear_regression(str(tmp_path / "m"))
    dense = np.zeros(size)
    dense[idx] = val
    np.testing.assert_array_equal(w, dense)
    assert b == 0.0 and load_progress(str(tmp_path / "m"))["batches"] == 3
    # the same file as the dense writer produces
    save_linear_regression(str(tmp_path / "d"), dense, 0.0, {"batches": 3})
    import pyarrow.parquet as pq
    ts = pq.read_table(str(tmp_path / "m" / "data" / "part-00000.parquet"))
    td = pq.read_table(str(tmp_path / "d" / "data" / "part-00000.parquet"))
    assert ts.equals(td) and ts.schema.metadata == td.schema.metadata


def test_sparse_weights_dense_fallback(tmp_path):
    """Over 25 % non-zeros: written as a dense VectorUDT, like MLlib would."""
    w = np.arange(1, 101, dtype=np.float64)
    w[::10] = 0.0
    nz = np.flatnonzero(w).astype(np.int32)
    save_linear_regression(str(tmp_path / "m"), SparseWeights(100, nz, w[nz]))
    got, _ = load_linear_regression(str(tmp_path / "m"))
    np.testing.assert_array_equal(got, w)
    import pyarrow.parquet as pq
    t = pq.read_table(str(tmp_path / "m" / "data" / "part-00000.parquet"))
    assert t.column("weights")[0].as_py()["type"] == 1


class _SlowModel:
    def __init__(self, delay, log):
        self.delay, self.log = delay, log
        self.gate = threading.Event()

    def snapshot(self):
        v = len(self.log)
        self.log.append(("snap", v))

        def save(path, prog):
            self.gate.wait(self.delay)
            save_linear_regression(path, np.full(8, float(v)), 0.0, prog)
            self.log.append(("saved", v))
        return save


def test_checkpoint_write_does_not_block_training(tmp_path):
    log = []
    m = _SlowModel(10.0, log)
    ck = StreamCheckpointer(str(tmp_path / "ck"), 1, 0, m.snapshot, lambda: None, asynchronous=True)
    t0 = time.perf_counter()
    assert ck.after_batch(1, 100, 100)
    # due while write 1 is in flight: skipped, not waited for
    assert ck.after_batch(2, 200, 200) is False
    assert time.perf_counter() - t0 < 1.0          # the write runs on the writer thread
    assert log == [("snap", 0)] and ck.skipped == 1
    m.gate.set()                                   # let the write finish
    ck.flush()
    assert load_progress(str(tmp_path / "ck"))["batches"] == 1
    assert ck.after_batch(3, 300, 300)             # the next due batch snapshots the newest model
    ck.flush()
    assert load_progress(str(tmp_path / "ck"))["batches"] == 3
    w, _ = load_linear_regression(str(tmp_path / "ck"))
    assert (w == log[-1][1]).all() and log[-1] == ("saved", 2)
    assert ck.written == 2
    # the final checkpoint waits and writes synchronously
    assert ck.after_batch(4, 400, 400, force=True)
    assert load_progress(str(tmp_path / "ck"))["batches"] == 4


def test_checkpoint_writer_error_surfaces(tmp_path):
    def snapshot():
        def save(path, prog):
            raise OSError("disk full")
        return save
    ck = StreamCheckpointer(str(tmp_path / "ck"), 1, 0, snapshot, lambda: None, asynchronous=True)
    ck.after_batch(1, 10, 10)
    with pytest.raises(RuntimeError, match="disk full"):
        ck.flush()


def test_checkpoint_positions_recorded_before_model(tmp_path):
    """Every rank records its position for batch t before rank 0's snapshot;
    the history keeps older positions so a model still being written (or
    the previous one) stays resumable."""
    from twitter_stream_ml_amd.checkpoint import StreamPositions
    log = []
    m = _SlowModel(0.0, log)
    m.gate.set()
    ck = StreamCheckpointer(str(tmp_path / "ck"), 2, 0, m.snapshot, lambda: None, asynchronous=False)
    for t in range(1, 7):
        ck.after_batch(t, 100 * t, 100 * t)
    ck.flush()
    pos = StreamPositions(str(tmp_path / "ck"), 0).history()
    assert pos == {2: 200, 4: 400, 6: 600}
    assert load_progress(str(tmp_path / "ck"))["batches"] == 6


def test_positions_survive_a_slow_writer(tmp_path):
    """with --checkpointInterval 1 an asynchronous write
    spans many batches; every position a resume could need -- the model on
    disk (and a .old copy) and the write in flight -- must survive pruning
    at every point of a long run."""
    from twitter_stream_ml_amd.apps._common import load_resume_state
    from twitter_stream_ml_amd.checkpoint import StreamPositions
    log = []
    m = _SlowModel(30.0, log)
    path = str(tmp_path / "ck")
    ck = StreamCheckpointer(path, 1, 0, m.snapshot, lambda: None, asynchronous=True)
    other = StreamPositions(path, 1)   # a second rank records its own positions
    inflight = None
    for t in range(1, 61):
        started = ck.after_batch(t, 10 * t, 10 * t)
        other.record(t, 7 * t)
        if started:
            inflight = t
        if t % 25 == 0:   # let the write in flight land now and then
            m.gate.set()
            ck._thread.join()
            m.gate.clear()
        prog = load_progress(path)
        if prog is not None:
            b = prog["batches"]
            assert StreamPositions(path, 0).records_at(b) == 10 * b
            assert StreamPositions(path, 1).records_at(b) == 7 * b
            st = load_resume_state("auto", path, 1)
            assert (st.batches, st.records) == (b, 7 * b)
        # the batch of the write in flight stays recorded on every rank
        th = ck._thread
        if th is not None and th.is_alive():
            assert StreamPositions(path, 0).records_at(inflight) == 10 * inflight
            assert StreamPositions(path, 1).records_at(inflight) == 7 * inflight
    m.gate.set()
    ck.flush()
    # bounded history: once the newest model landed, old positions go
    ck.after_batch(61, 610, 610, force=True)
    other.record(61, 427)
    assert len(StreamPositions(path, 0).history()) <= 16 + 1


def test_positions_history_is_bounded_without_a_model(tmp_path):
    """with no model readable on this rank's filesystem (every
    write failing, or a rank that cannot see rank 0's directory) the floor
    is 0; the history must still stay bounded (keep * 64 entries)."""
    from twitter_stream_ml_amd.checkpoint.stream_state import StreamPositions
    sp = StreamPositions(str(tmp_path / "ckpt"), rank=1, keep=4)
    for b in range(1, 1001):
        sp.record(b, 10 * b)
    h = sp.history()
    assert len(h) == 4 * 64 and max(h) == 1000 and h[1000] == 10000
