"""Host staging with the receiver's scalar column bounds (one-pass wire
encoding, csrc/hip/engine.cpp HostBatch::pack_scalars).

The packed scalar columns must be byte-identical with and without the hint;
a hint that does not hold (a value outside it) falls back to the exact
two-pass encoding; a batch staged with the hint trains exactly as one
without it.  The HostBatch buffers are page-locked, hence a GPU test.
"""
import numpy as np
import pytest

from twitter_stream_ml_amd.sources.synthetic import SynthConfig, generate_batch

pytestmark = pytest.mark.gpu
NOW = 1_700_000_000_000


def _spack(hb):
    w = hb._hb.scalar_wire
    n = int(w["offsets"][-1])
    return np.array(hb._hb.spack_bytes[:n]), w


def test_range_hint_gives_the_same_wire_columns(hip_module):
    from twitter_stream_ml_amd.ops.lr_engine import HostBatchView, encode_utf8
    raw = generate_batch(SynthConfig.profile("wide", seed=31), 0, 50_000, batch_time_ms=NOW)
    u8 = encode_utf8(raw)
    a = HostBatchView(raw.n, raw.total_units + 1024, text=False)
    b = HostBatchView(raw.n, raw.total_units + 1024, text=False)
    a.load_utf8(raw, u8, copy_text=False)                       # two passes (no hint)
    raw.with_scalar_range()
    b.load_utf8(raw, u8, copy_text=False)                       # one pass
    assert (b._hb.range_hits, b._hb.range_misses) == (1, 0)
    pa, wa = _spack(a)
    pb, wb = _spack(b)
    assert wa == wb and np.array_equal(pa, pb)
    # a hint that does not hold: the min of column 1 is overstated (the true
    # min lies below the encoding's base; an understated max that still fits
    # the same bit width is a valid encoding and packs in one pass)
    bad = raw.scalar_range.copy()
    bad[0, 1] = raw.scalars[1].min() + 1
    raw.scalar_range = bad
    b.load_utf8(raw, u8, copy_text=False)
    assert (b._hb.range_hits, b._hb.range_misses) == (1, 1)
    pc, wc = _spack(b)
    assert wc == wa and np.array_equal(pc, pa)
    # a wider (but valid) hint is a valid, possibly wider encoding
    wide = raw.scalar_range.copy()
    wide[0] -= 5
    wide[1] += 5
    wide[1, 1] = raw.scalars[1].max() + 5
    raw.scalar_range = wide
    b.load_utf8(raw, u8, copy_text=False)
    assert b._hb.range_misses == 1 and b._hb.range_hits == 2


def test_training_with_and_without_hint_is_identical(hip_module):
    from twitter_stream_ml_amd.ops.lr_engine import DeviceLinearRegression, LRDeviceConfig
    cfg = SynthConfig.profile("wide", seed=32)
    batches = [generate_batch(cfg, i * 20_000, 20_000, batch_time_ms=NOW + i) for i in range(3)]
    mk = lambda: DeviceLinearRegression(LRDeviceConfig(num_text_features=1 << 20, max_rows=20_000,
                                                       max_units=20_000 * 300, ingest="utf8"), device=0)
    from twitter_stream_ml_amd.ops.lr_engine import encode_utf8
    from twitter_stream_ml_amd.records.batch import RawBatch
    e1, e2 = mk(), mk()
    for b in batches:
        e1.train_batch(b, want_pred=False)
    for b in batches:
        h = RawBatch(b.text, b.offsets, b.is_retweet, b.scalars, b.batch_time_ms, utf8=encode_utf8(b))
        e2.train_batch(h.with_scalar_range(), want_pred=False)
    assert e2.staging(0)._hb.range_hits >= 1
    np.testing.assert_array_equal(e1.get_weights(), e2.get_weights())
