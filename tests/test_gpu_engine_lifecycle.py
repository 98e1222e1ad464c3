"""Engines built and destroyed back to back in one process (round-5 faults).

Round 5 saw two faults that depended on what earlier tests of the same
process had done: ``hipMemcpyAsync ... invalid argument`` on a raw slot's
scalar H2D, and an illegal memory access on a later ``hipMemcpy``.  Their
cause (profiles/README.md, round 6): page-locked receiver buffers
(``register_host``) were freed without ``hipHostUnregister``.  The runtime
keeps such a range in its host-pointer map, and a later buffer mapped at an
overlapping address resolves to the stale registration -- the wrong size
(invalid argument) or the wrong GPU mapping (a faulting DMA).

Here: registrations end with the arrays that own them; a registration that
overlaps a live one is refused; three engines with 8 raw slots prefetch deep
into their high slots while an asynchronous checkpoint writer runs, each
built after the previous one and its replay pool were freed; every prefetch
is trained from its slot or discarded as an orphan, and no slot leaks.
"""
import gc
from types import SimpleNamespace

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
NOW = 1_700_000_000_000


def _live(hip_module):
    return {p: n for p, n in hip_module.host_registrations()}


def _who_holds(ptrs, depth=5):
    """Referrer chains of the objects still holding registered arrays
    (diagnostics; ndarrays are not tracked by gc, their holders are)."""
    import types
    names = ("Utf8Text", "RawBatch", "HostBatchView", "DeviceLinearRegression", "SlotPipeline")
    live = [o for o in gc.get_objects() if type(o).__name__ in names]
    roots = [o for o in live if type(o).__name__ != "Utf8Text" or int(o.data.ctypes.data) in ptrs]
    out = [f"live: " + ", ".join(f"{n}={sum(type(o).__name__ == n for o in live)}" for n in names)]
    for a in roots[:2]:
        out.append(f"-- {type(a).__name__}")
        frontier, seen = [a], {id(a), id(roots), id(live)}
        for d in range(depth):
            nxt = []
            for o in frontier:
                for r in gc.get_referrers(o):
                    if id(r) in seen or isinstance(r, types.FrameType) or r is frontier or r is nxt:
                        continue
                    seen.add(id(r))
                    desc = type(r).__name__
                    if isinstance(r, dict):
                        desc += "{" + ",".join(str(k) for k in list(r)[:8]) + "}"
                    elif isinstance(r, types.FunctionType):
                        desc += f" {r.__qualname__}"
                    out.append(f"{'  ' * (d + 1)}{desc}")
                    nxt.append(r)
            frontier = nxt[:12]
    return "\n".join(out[:120])


def test_registration_follows_array_lifetime(hip_module):
    import torch
    from twitter_stream_ml_amd.ops.lr_engine import register_host, unregister_host
    before = _live(hip_module)
    a = np.arange(1 << 22, dtype=np.uint8)          # 4 MB: its own mapping
    pa = int(a.ctypes.data)
    register_host(a)
    assert _live(hip_module)[pa] == a.nbytes
    with pytest.raises(RuntimeError):               # an overlapping range is refused
        hip_module.host_register(pa + 4096, 4096)
    view = a[1024:]
    del a
    gc.collect()
    assert pa in _live(hip_module)                  # a view keeps the owner (and its registration) alive
    del view
    gc.collect()
    assert pa not in _live(hip_module)              # unregistered before the memory was freed
    # the same size again (often the same address): registers cleanly and DMAs the new bytes
    b = (np.arange(1 << 22, dtype=np.int64) % 251).astype(np.uint8)
    register_host(b)
    d = torch.empty(b.shape[0], dtype=torch.uint8, device="cuda:0")
    d.copy_(torch.from_numpy(b), non_blocking=True)
    torch.cuda.synchronize()
    assert np.array_equal(d.cpu().numpy(), b)
    unregister_host(b)
    assert int(b.ctypes.data) not in _live(hip_module)
    del b
    gc.collect()
    assert _live(hip_module) == before


def test_back_to_back_engines_deep_prefetch_async_checkpoint(hip_module, tmp_path, monkeypatch):
    from twitter_stream_ml_amd.apps.linear_regression import LinearRegressionJob, build_engine
    from twitter_stream_ml_amd.config.arguments import ConfArguments
    from twitter_stream_ml_amd.sources.synthetic import SynthConfig, SyntheticReplaySource
    monkeypatch.setenv("TWTML_RAW_SLOTS", "8")
    rows, n = 100_000, 24
    base_regs = _live(hip_module)
    weights = []
    for r in range(3):
        src = SyntheticReplaySource(SynthConfig.profile("wide", seed=60 + r), batches=6, batch_rows=rows)
        assert len(_live(hip_module)) == len(base_regs) + 6
        ck = str(tmp_path / f"ck{r}")
        conf = ConfArguments().parse(["--master", "rocm[1]", "-f", "1000000", "--checkpoint", ck,
                                      "--checkpointInterval", "1", "--batchSize", str(rows)])
        eng = build_engine(conf, rank=0, world=1, max_rows=rows)
        assert eng.raw_slots == 8
        eng.set_weights(np.zeros(eng.num_weights))
        job = LinearRegressionJob(conf, eng, None, 0, plot=False)
        batches = [src.pool[t % 6].with_time(NOW + t * 5000) for t in range(n + 8)]
        stray = src.pool[0].with_time(NOW - 1)          # prefetched, never trained: an orphan
        slots_seen = set()
        for t in range(n):
            for u in batches[t + 1:t + 7]:              # six ahead: slots up to 7
                eng.prefetch(u)
            if t == 5:
                assert eng.prefetch(stray) is False     # cap: raw_slots - 1 in flight
            if t == 6:
                eng._pipe.drop()                        # all seven discarded on the engine...
                assert eng._pipe.in_flight == 0
                for u in batches[t:t + 4]:              # ... and the next ones prefetched again,
                    eng.prefetch(u)
                eng.prefetch(stray)                     # with a stray behind them
            slots_seen.update(s for _, s in eng._pipe._inflight.values())
            job.on_batch(SimpleNamespace(raw=batches[t]), batches[t].batch_time_ms)
        pipe = eng._pipe
        assert max(slots_seen) == 7
        assert pipe.orphaned == 7 + 1, pipe.orphaned     # the drop + the stray (skipped by a later hit)
        assert pipe.prefetched == pipe.hits + pipe.orphaned + pipe.in_flight
        assert pipe.hits == n - 1
        job.final_checkpoint()
        cp = job.checkpointer
        assert cp.written >= 2 and cp.written + cp.skipped == n + 1
        w = eng.get_weights()
        assert np.isfinite(w).all() and np.count_nonzero(w) > 1000
        weights.append(w)
        pipe.drop()
        assert pipe.in_flight == 0
        eng.synchronize()
        job.close()
        # every local that reaches the engine (cp -> job -> engine -> staging views,
        # which hold the DMA'd pool arrays) or a batch (u: the prefetch loop's last)
        del job, eng, src, batches, stray, u, cp, pipe
        gc.collect()
        assert list(hip_module.teardown_errors()) == []
        left = set(_live(hip_module)) - set(base_regs)
        assert not left, _who_holds(left)               # the pool's registrations ended with it
    # three different streams: three different models
    assert not np.array_equal(weights[0], weights[1])
