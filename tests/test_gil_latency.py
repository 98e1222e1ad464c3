"""utils/gil.py: the drivers' streaming settings are scoped -- a short GIL
switch interval and a frozen GC heap inside the block, the interpreter's
own settings restored after it (the drivers also run in-process in tests)."""
import gc
import sys

from twitter_stream_ml_amd.utils.gil import quiet_gc, short_gil_slices, streaming_latency


def test_short_gil_slices_scoped():
    old = sys.getswitchinterval()
    with short_gil_slices(250):
        assert abs(sys.getswitchinterval() - 250e-6) < 2e-6
    assert sys.getswitchinterval() == old
    sys.setswitchinterval(1e-4)            # never lengthened
    short = sys.getswitchinterval()
    try:
        with short_gil_slices(500):
            assert abs(sys.getswitchinterval() - short) < 2e-6
    finally:
        sys.setswitchinterval(old)


def test_quiet_gc_freezes_then_unfreezes():
    base = gc.get_freeze_count()
    with quiet_gc():
        assert gc.get_freeze_count() > base
        junk = [[i] for i in range(1000)]   # new objects stay collectable
        del junk
    assert gc.get_freeze_count() == base


def test_streaming_latency_restores_on_error():
    old = sys.getswitchinterval()
    base = gc.get_freeze_count()
    try:
        with streaming_latency():
            raise RuntimeError("batch failed")
    except RuntimeError:
        pass
    assert sys.getswitchinterval() == old and gc.get_freeze_count() == base
