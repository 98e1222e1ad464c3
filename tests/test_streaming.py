"""Streaming runtime (U13/U14 semantics): sealing, ordering, backpressure, DStream ops."""
import threading
import time

import numpy as np
import pytest

from twitter_stream_ml_amd.records.batch import RawBatch
from twitter_stream_ml_amd.runtime.streaming import StreamingContext
from twitter_stream_ml_amd.sources.synthetic import SynthConfig, SyntheticTweetSource, generate_batch


def test_size_sealed_batches_are_exact_and_in_source_order():
    src = SyntheticTweetSource(SynthConfig(seed=3), rate=0.0)
    ssc = StreamingContext(0, batch_size=1000, num_batches=4, poll_chunk=300)
    seen = []
    ssc.receiverStream(src).foreachRDD(lambda rdd: seen.append(rdd.raw))
    ssc.start()
    assert ssc.awaitTermination(30)
    ssc.stop()
    assert [b.n for b in seen] == [1000] * 4
    assert ssc.records_done == 4000 and ssc.batches_done == 4
    full = generate_batch(SynthConfig(seed=3), 0, 4000)
    got = RawBatch.concat(seen)
    np.testing.assert_array_equal(got.text, full.text)
    np.testing.assert_array_equal(got.scalars[:4], full.scalars[:4])   # createdAt follows the clock


def test_output_ops_run_sequentially_in_registration_order():
    src = SyntheticTweetSource(SynthConfig(seed=1), rate=0.0)
    ssc = StreamingContext(0, batch_size=200, num_batches=3)
    log = []
    stream = ssc.receiverStream(src).cache()
    stream.foreachRDD(lambda rdd, t: log.append(("stats", rdd.count())))
    stream.foreachRDD(lambda rdd: log.append(("train", rdd.count())))
    ssc.start()
    ssc.awaitTermination(30)
    ssc.stop()
    assert log == [("stats", 200), ("train", 200)] * 3


def test_backpressure_bounds_pending_batches():
    src = SyntheticTweetSource(SynthConfig(seed=2), rate=0.0)
    ssc = StreamingContext(0, batch_size=100, num_batches=12, max_pending=2)
    gate = threading.Event()
    max_q = []

    def slow(rdd):
        max_q.append(ssc._jobs.qsize())
        gate.wait(0.05)

    ssc.receiverStream(src).foreachRDD(slow)
    ssc.start()
    ssc.awaitTermination(30)
    ssc.stop()
    assert ssc.batches_done == 12
    assert max(max_q) <= 2


def test_interval_sealing_and_scheduling_delay():
    src = SyntheticTweetSource(SynthConfig(seed=4), rate=2000.0)
    ssc = StreamingContext(0.2, num_batches=3)
    sizes = []
    ssc.receiverStream(src).foreachRDD(lambda rdd: sizes.append(rdd.raw.n))
    t0 = time.time()
    ssc.start()
    ssc.awaitTermination(30)
    ssc.stop()
    assert len(sizes) == 3 and time.time() - t0 >= 0.55
    assert all(150 <= s <= 700 for s in sizes[1:]), sizes       # ~400 records per 0.2 s
    assert all(i.scheduling_delay_ms >= 0 for i in ssc.batch_infos)


def test_dstream_transformations_are_lazy_per_batch():
    ssc = StreamingContext(1.0)
    raw = generate_batch(SynthConfig(seed=5), 0, 500)

    class Src:
        def poll(self, n, now_ms=None):
            return raw

    stream = ssc.receiverStream(Src())
    counted = []
    retweets = stream.filter(lambda s: s.isRetweet())
    retweets.map(lambda s: s.getRetweetCount()).foreachRDD(lambda rdd: counted.append(rdd.count()))
    ssc.run_batches(2)
    assert counted == [int(raw.is_retweet.sum())] * 2


def test_time_sealed_batches_respect_engine_capacity():
    """A time-sealed batch never exceeds the engine's staging capacity: the
    receiver seals early at max_batch_rows / max_batch_units (ADVICE r1:
    a 5 s batch with more rows than the buffers used to kill the job)."""
    import time as _t
    from twitter_stream_ml_amd.runtime.streaming import StreamingContext
    from twitter_stream_ml_amd.sources.synthetic import SynthConfig, SyntheticTweetSource
    ssc = StreamingContext(batch_seconds=30.0, num_batches=4, max_batch_rows=5000,
                           max_batch_units=5000 * 120, poll_chunk=1500)
    sizes = []
    ssc.twitterStream(SyntheticTweetSource(SynthConfig(seed=2))).foreachRDD(
        lambda rdd: sizes.append((rdd.raw.n, rdd.raw.total_units)))
    ssc.start()
    t0 = _t.time()
    assert ssc.awaitTermination(60)
    ssc.stop()
    assert len(sizes) == 4 and _t.time() - t0 < 30   # sealed by capacity, not the 30 s timer
    assert all(0 < n <= 5000 and u <= 5000 * 120 for n, u in sizes), sizes
    assert ssc.capacity_seals >= 4


def test_manual_clock_batch_times():
    """spark.streaming.clock=ManualClock analogue: batch k has time
    start + k * step whatever the wall clock does, and every poll inside it
    reads that time (the age feature's reference point)."""
    from twitter_stream_ml_amd.runtime.clock import ManualClock, SystemClock, streaming_clock
    seen = []

    class Src:
        def poll(self, n, now_ms=None):
            seen.append(now_ms)
            return generate_batch(SynthConfig(seed=1), 0, n, batch_time_ms=now_ms)

    ssc = StreamingContext(0, batch_size=500, num_batches=3, poll_chunk=200, clock=ManualClock(1000, 5000))
    times = []
    ssc.twitterStream(Src()).foreachRDD(lambda rdd, t: times.append(t))
    ssc.start()
    ssc.awaitTermination()
    ssc.stop()
    assert times == [1000, 6000, 11000]
    assert seen[:3] == [1000, 1000, 1000] and seen[3] == 6000   # 200 + 200 + 100 rows, then the next batch
    assert isinstance(streaming_clock(""), SystemClock)
    c = streaming_clock("manual:7:3")
    c.advance()
    assert c.now_ms() == 10
    with pytest.raises(ValueError):
        streaming_clock("manual:1")
