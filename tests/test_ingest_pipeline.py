"""Ingest || compute pipelining: slot protocol and the streaming prefetch hook.

SURVEY §2.4 "Ingest || compute pipelining" (receiver on its own core while the
JobScheduler trains, U13/U14).  CPU-only: the engine is faked, the slot
protocol and the runtime's prefetch ordering are what is checked.
"""
from __future__ import annotations

import threading

import pytest

from twitter_stream_ml_amd.ops.ingest import SlotPipeline
from twitter_stream_ml_amd.runtime.streaming import StreamingContext
from twitter_stream_ml_amd.sources import make_source


class FakeEngine:
    """Records staging writes / H2D submits / processes per slot and checks
    that a staging buffer is never rewritten while its slot is in flight."""

    def __init__(self, n_slots=3):
        self.inflight = set()
        self.log = []
        self.syncs = 0
        self.pipe = SlotPipeline(n_slots, self.stage, self.submit, self.sync)

    def stage(self, slot, raw):
        assert slot not in self.inflight, "staging buffer rewritten during its H2D"
        self.log.append(("stage", slot, raw))
        return (slot, raw)

    def submit(self, hb, slot):
        assert hb[0] == slot
        self.inflight.add(slot)
        self.log.append(("submit", slot, hb[1]))

    def sync(self):
        self.syncs += 1
        self.inflight.clear()

    def process(self, slot, raw):
        assert slot in self.inflight
        staged = [e for e in self.log if e[0] == "stage" and e[1] == slot][-1]
        assert staged[2] is raw, "slot holds a different batch"
        self.inflight.discard(slot)
        self.log.append(("process", slot, raw))

    def train(self, raw):
        self.process(self.pipe.take(raw), raw)


def test_take_without_prefetch_uses_free_slots():
    e = FakeEngine()
    batches = [object() for _ in range(7)]
    for b in batches:
        e.train(b)
    assert e.pipe.hits == 0 and e.pipe.prefetched == 0
    assert [x[1] for x in e.log if x[0] == "process"] == [0, 1, 2, 0, 1, 2, 0]


def test_prefetch_cap_and_hits():
    e = FakeEngine(3)
    b = [object() for _ in range(6)]
    assert e.pipe.prefetch(b[1]) and e.pipe.prefetch(b[2])
    assert not e.pipe.prefetch(b[3])          # cap n_slots - 1: one slot kept free
    assert e.pipe.prefetch(b[1])              # idempotent
    e.train(b[0])                              # not prefetched: the free slot
    e.train(b[1])
    e.train(b[2])
    assert e.pipe.hits == 2 and e.pipe.prefetched == 2
    # steady state: prefetch next two, train current, never overwrite in flight
    for t in range(3, 6):
        for u in b[t + 1:t + 3]:
            e.pipe.prefetch(u)
        e.train(b[t])
    assert e.pipe.pending() == []


def test_drop_syncs_before_forgetting():
    e = FakeEngine(3)
    b = [object() for _ in range(3)]
    e.pipe.prefetch(b[1])
    e.pipe.drop()
    assert e.syncs == 1 and e.pipe.pending() == []
    e.train(b[0])
    e.train(b[1])                              # restaged, not a stale hit
    assert e.pipe.hits == 0


class DiscardEngine(FakeEngine):
    """FakeEngine with the engine's discard hook (LREngine::discard)."""

    def __init__(self, n_slots=4):
        super().__init__(n_slots)
        self.discarded = []
        self.pipe = SlotPipeline(n_slots, self.stage, self.submit, self.sync, discard=self.discard)

    def discard(self, slot):
        assert slot in self.inflight, "discard of a slot that holds no batch"
        self.inflight.discard(slot)
        self.discarded.append(slot)


def _batch(t, n=8):
    import numpy as np
    from twitter_stream_ml_amd.records.batch import RawBatch
    return RawBatch(np.zeros(n * 3, np.uint16), np.arange(n + 1, dtype=np.int64) * 3, np.ones(n, np.uint8),
                    np.zeros((5, n), np.int64), t)


def test_prefetch_matches_copies_that_share_the_arrays():
    """Round-5 verdict: a driver that prefetches pool[i].with_time(t) and
    trains another with_time(t) copy of it must hit (the key is the batch's
    content -- seal time, buffers -- not the Python object)."""
    e = DiscardEngine(4)
    pool = [_batch(0), _batch(0)]
    nxt = pool[1].with_time(5000)
    assert e.pipe.prefetch(nxt)
    e.process(e.pipe.take(pool[1].with_time(5000)), nxt)
    assert (e.pipe.hits, e.pipe.orphaned, e.pipe.in_flight) == (1, 0, 0)
    # another seal time or other buffers are other batches
    assert e.pipe.prefetch(pool[1].with_time(6000))
    slot = e.pipe.take(pool[0].with_time(6000))
    assert e.pipe.hits == 1 and e.pipe.in_flight == 1 and slot not in [s for _, s in e.pipe._inflight.values()]


def test_skipped_prefetches_are_discarded_not_stranded():
    """Entries prefetched before the batch a take matches can never be
    trained in order: they go back to the engine (discard) and their slots
    are reused; with the old id() keys they stayed pinned for the run."""
    e = DiscardEngine(4)
    b = [_batch(t * 1000) for t in range(12)]
    assert e.pipe.prefetch(b[1]) and e.pipe.prefetch(b[2]) and e.pipe.prefetch(b[3])
    e.train(b[0])                                   # not prefetched: the free slot
    e.train(b[3])                                   # skips b[1], b[2]: orphans
    assert e.pipe.orphaned == 2 and len(e.discarded) == 2
    assert e.pipe.in_flight == 0
    # every slot is usable again: three more prefetches fit
    for u in b[4:7]:
        assert e.pipe.prefetch(u)
    for u in b[4:7]:
        e.train(u)
    assert e.pipe.prefetched == e.pipe.hits + e.pipe.orphaned + e.pipe.in_flight == 6


def test_single_slot_pipeline_never_prefetches():
    e = FakeEngine(1)
    b = [object() for _ in range(3)]
    assert not e.pipe.prefetch(b[1])
    for x in b:
        e.train(x)


def test_streaming_prefetch_hook_sees_queued_batches_in_order():
    """Sealed batches queued behind the running one are offered to the hook
    before that batch's output ops run; every batch runs exactly once, in order."""
    ssc = StreamingContext(0, batch_size=64, num_batches=6, max_pending=4)
    stream = ssc.twitterStream(make_source("synthetic", rate=0, seed=3))
    gate = threading.Event()
    ran, offered = [], []

    def on_batch(rdd):
        if not ran:
            gate.wait(5)      # hold the first batch so later ones queue up
        ran.append(rdd.raw)

    def hook(b):
        assert all(b is not r for r in ran), "prefetch offered a batch that already ran"
        offered.append(b)

    stream.foreachRDD(on_batch)
    ssc.add_prefetch(hook)
    ssc.start()
    import time
    deadline = time.time() + 5
    while ssc._jobs.qsize() < 2 and time.time() < deadline:
        time.sleep(0.01)
    gate.set()
    assert ssc.awaitTermination(20)
    ssc.stop()
    assert len(ran) == 6
    assert len({id(r) for r in ran}) == 6
    assert offered, "no batch was offered for prefetch"
    ids = [id(r) for r in ran]
    # every offered batch ran later
    for b in offered:
        assert id(b) in ids


@pytest.mark.gpu
def test_gpu_prefetched_training_matches_synchronous():
    """Prefetched (overlapped H2D) training gives the synchronous path's weights.

    Not bitwise: rows land in chunks in atomic (run-dependent) order, so the
    fp32 per-lane hot-gradient sums differ in the last bits between any two
    runs; two synchronous engines are compared with the same tolerance."""
    import numpy as np
    import torch
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from twitter_stream_ml_amd.ops.lr_engine import DeviceLinearRegression, LRDeviceConfig
    from twitter_stream_ml_amd.sources.synthetic import SynthConfig, generate_batch
    cfg = SynthConfig.profile("twitter", seed=11)
    batches = [generate_batch(cfg, i * 4096, 4096, batch_time_ms=1_700_000_000_000 + i)
               for i in range(5)]
    mk = lambda: DeviceLinearRegression(LRDeviceConfig(num_text_features=1 << 20, max_rows=4096,
                                                       max_units=4096 * 300), device=0)
    a, b, c = mk(), mk(), mk()
    for x in batches:
        a.train_batch(x)
    for x in batches:
        c.train_batch(x)
    wa, wc = a.get_weights(), c.get_weights()
    np.testing.assert_allclose(wc, wa, rtol=1e-4, atol=1e-10, err_msg="sync vs sync")
    for t, x in enumerate(batches):
        for u in batches[t + 1:t + 3]:
            b.prefetch(u)
        b.train_batch(x)
    assert b._pipe.hits == 4
    np.testing.assert_allclose(b.get_weights(), wa, rtol=1e-4, atol=1e-10)
    assert np.count_nonzero(b.get_weights()) == np.count_nonzero(wa)


@pytest.mark.gpu
def test_prepare_ahead_out_of_order_and_toggle(hip_module):
    """Prepare-ahead (batch t+1 prepared on the prep stream while t trains)
    against the in-line engine: same model; prefetched batches trained out of
    submission order (the engine evicts a batch it prepared ahead and
    prepares it again when it is due) still give the in-order result of that
    order."""
    import numpy as np
    from twitter_stream_ml_amd.ops.lr_engine import DeviceLinearRegression, LRDeviceConfig
    from twitter_stream_ml_amd.sources.synthetic import SynthConfig, generate_batch
    cfg = SynthConfig.profile("wide", seed=12)
    batches = [generate_batch(cfg, i * 4096, 4096, batch_time_ms=1_700_000_000_000 + i) for i in range(5)]
    mk = lambda ov: DeviceLinearRegression(LRDeviceConfig(num_text_features=1 << 20, max_rows=4096,
                                                          max_units=4096 * 300, overlap=ov), device=0)
    ref, ahead, ooo = mk(False), mk(True), mk(True)
    order = [0, 2, 1, 4, 3]
    for i in order:
        ref.train_batch(batches[i])
    for i in order[:3]:
        assert ahead.prefetch(batches[i])
    for t, i in enumerate(order):
        if t + 3 < len(order):
            ahead.prefetch(batches[order[t + 3]])
        ahead.train_batch(batches[i])
    # equal up to the summation order (rows of equal length are placed by
    # atomics, so two in-line engines differ in the last bits as well)
    w = ref.get_weights()
    tol = dict(rtol=1e-4, atol=1e-6 * np.abs(w).max())
    np.testing.assert_allclose(ahead.get_weights(), w, **tol)
    # 0, 1, 2 submitted; 0 trains, 1 and 2 get prepared ahead; then 3 (not
    # prefetched) must evict one of them
    order2 = [0, 3, 1, 2, 4]
    ref2 = mk(False)
    for i in order2:
        ref2.train_batch(batches[i])
    for i in (0, 1, 2):
        assert ooo.prefetch(batches[i])
    for i in order2:
        ooo.train_batch(batches[i])
    np.testing.assert_allclose(ooo.get_weights(), ref2.get_weights(), **tol)
