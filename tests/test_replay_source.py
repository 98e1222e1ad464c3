"""``replay:synthetic`` source and receiver-held UTF-8 batches (CPU).

The pooled replay source stands in for the network receiver when the driver
is measured (``python -m twitter_stream_ml_amd --source replay:synthetic:wide:30
--batchSize 1000000 --seconds 0``): whole pre-generated batches, their text as
UTF-8 bytes (``RawBatch.utf8``) that the device engines DMA without a host
copy.  Reference: the Twitter receiver, ``LinearRegression.scala:44``.
"""
import numpy as np

from twitter_stream_ml_amd.records.batch import RawBatch
from twitter_stream_ml_amd.runtime.streaming import StreamingContext
from twitter_stream_ml_amd.sources import SyntheticReplaySource, SynthConfig, generate_batch, make_source


def test_replay_pool_cycles_whole_batches():
    src = make_source("replay:synthetic:bench:3", seed=5, batch_size=500)
    assert isinstance(src, SyntheticReplaySource) and src.chunk_rows == 500
    got = [src.poll(500, now_ms=1000 + i) for i in range(5)]
    assert [b.n for b in got] == [500] * 5
    assert got[3].utf8 is got[0].utf8 and got[4].utf8 is got[1].utf8   # the pool, cycled
    assert got[3] is not got[0] and got[3].batch_time_ms == 1003       # shallow copies, own time
    assert got[0].text.shape[0] == 0 and got[0].total_units > 0          # UTF-16 not kept


def test_replay_utf8_decodes_to_the_generator_text():
    cfg = SynthConfig.profile("wide", seed=9)
    src = SyntheticReplaySource(cfg, 2, 300, pin=False)
    ref = [generate_batch(cfg, i * 300, 300) for i in range(2)]
    for want in ref:
        b = src.poll(300)
        np.testing.assert_array_equal(b.offsets, want.offsets)
        np.testing.assert_array_equal(b.scalars, want.scalars)
        np.testing.assert_array_equal(b.ensure_text().text, want.text)
        assert b.text_of(7) == want.text_of(7)


def test_shards_draw_disjoint_streams():
    a = make_source("replay:synthetic:bench:1", seed=5, batch_size=200, shard=0, num_shards=2).poll(200)
    b = make_source("replay:synthetic:bench:1", seed=5, batch_size=200, shard=1, num_shards=2).poll(200)
    assert not np.array_equal(a.scalars, b.scalars)


def test_exact_size_seal_keeps_the_receiver_buffer():
    src = make_source("replay:synthetic:bench:2", seed=3, batch_size=400)
    ssc = StreamingContext(0, batch_size=400, num_batches=3)
    seen = []
    ssc.receiverStream(src).foreachRDD(lambda rdd: seen.append(rdd.raw))
    ssc.start()
    ssc.awaitTermination(30)
    ssc.stop()
    assert len(seen) == 3 and all(b.n == 400 for b in seen)
    assert seen[0].utf8 is src.pool[0].utf8 and seen[1].utf8 is src.pool[1].utf8   # no concat copy


def test_partial_polls_decode_slices():
    src = make_source("replay:synthetic:bench:1", seed=3, batch_size=400)
    parts = [src.poll(150), src.poll(150), src.poll(100)]
    whole = RawBatch.concat(parts)
    ref = generate_batch(src.cfg, 0, 400)
    np.testing.assert_array_equal(whole.text, ref.text)
    np.testing.assert_array_equal(whole.scalars, ref.scalars)
