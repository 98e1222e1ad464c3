"""TWTML_H2D_TIMING=1 copy-stream timeline (the bench's window diagnostics).

Every submit records (queued, start, end, bytes) on the copy stream
(``csrc/hip/raw_slots.cpp``); the bench turns them into the window's copy
busy time, gaps, slot waits and host-late gaps (README "What bounds the
window").  Checked here: one record per submitted batch, in stream order,
each mark after the one before it, the bytes adding up to the engine's H2D
counter, and the window marks placed in the same time base.
"""
import numpy as np
import pytest

from twitter_stream_ml_amd.sources.synthetic import SynthConfig, generate_batch

pytestmark = pytest.mark.gpu
NOW = 1_700_000_000_000


def test_h2d_timeline_marks(hip_module, monkeypatch):
    from twitter_stream_ml_amd.ops.lr_engine import DeviceLinearRegression, LRDeviceConfig
    monkeypatch.setenv("TWTML_H2D_TIMING", "1")
    rows = 20_000
    eng = DeviceLinearRegression(LRDeviceConfig(num_text_features=1 << 20, max_rows=rows,
                                                max_units=rows * 300), device=0)
    synth = SynthConfig.profile("wide", seed=31)
    nb = 5
    eng.synchronize()
    eng._eng.h2d_window_mark()
    for t in range(nb):
        eng.train_batch(generate_batch(synth, t * rows, rows, batch_time_ms=NOW + t * 1000), want_pred=False)
    eng.synchronize()
    eng._eng.h2d_window_mark()
    tl = np.asarray(eng._eng.h2d_timeline())
    win = eng._eng.h2d_window()
    assert tl.shape == (nb, 4), tl.shape
    q, a, b, nbytes = tl.T
    assert q[0] == 0.0                                   # the time base: the first submit's queued mark
    assert np.all(q <= a + 1e-3) and np.all(a <= b + 1e-3), tl
    assert np.all(a[1:] >= b[:-1] - 1e-3), tl            # one copy stream: copies in submit order
    assert int(nbytes.sum()) == eng.h2d_bytes             # every byte the engine counted
    assert np.all(nbytes > rows)                          # each batch's text and row words
    assert len(win) == 2 and win[0] <= a[0] + 1e-3 and win[1] >= b[-1] - 1e-3, (win, tl)
