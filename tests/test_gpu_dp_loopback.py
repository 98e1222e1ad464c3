"""Data-parallel engine path on one GPU via the in-process loopback communicator.

RCCL refuses two ranks on the same device, so the DP orchestration of the
engine (all-gather of the per-rank active id lists, per-rank kept counts
and sampling offsets, per-iteration gradient all-reduce, stats all-reduce,
early exit agreement) is exercised with N engines on N threads of one
process, reducing through host memory.  DP over shards must equal the
single-engine run on the concatenated batch.
"""
import threading

import numpy as np
import pytest

from twitter_stream_ml_amd.sources.synthetic import SynthConfig, generate_batch

pytestmark = pytest.mark.gpu
NOW = 1_700_000_000_000


def _cfg(F, **kw):
    from twitter_stream_ml_amd.ops.lr_engine import LRDeviceConfig
    return LRDeviceConfig(num_text_features=F, max_rows=8192, max_units=8192 * 300, **kw)


def _run_dp(world, batches, cfg, ahead=True):
    from twitter_stream_ml_amd.ops._native import hip
    from twitter_stream_ml_amd.ops.lr_engine import DeviceLinearRegression
    group = hip().LoopbackGroup(world)
    engines = [DeviceLinearRegression(cfg, device=0, comm=group.comm(r)) for r in range(world)]
    results = [[None] * len(batches) for _ in range(world)]
    errors = []

    def worker(r):
        try:
            eng = engines[r]
            shards = [full.shard(r, world) for full in batches]
            # ahead: queue the shards first -- batch t+1's local part is
            # prepared while t trains, its packets all-gathered between two of
            # t's GD iterations; else every batch's all-gather runs in line
            if ahead:
                for sh in shards[:eng.raw_slots - 1]:
                    assert eng.prefetch(sh)
            for t, sh in enumerate(shards):
                results[r][t] = eng.train_batch(sh, want_pred=False)
        except Exception as e:  # pragma: no cover - surfaced below
            errors.append(e)

    th = [threading.Thread(target=worker, args=(r,)) for r in range(world)]
    for x in th:
        x.start()
    for x in th:
        x.join(timeout=300)
    assert not errors, errors
    return engines, results


@pytest.mark.parametrize("world,fraction,ahead", [(2, 1.0, True), (3, 1.0, True), (2, 0.5, True),
                                                 (2, 1.0, False), (3, 0.5, False)])
def test_dp_equals_single_engine(hip_module, world, fraction, ahead):
    """ahead: batch t+1 is prepared while t trains and its prep packets are
    all-gathered mid-loop (the ready words ride in the gradient all-reduce);
    else in line.  Either way DP equals the single engine bit for bit."""
    from twitter_stream_ml_amd.ops.lr_engine import DeviceLinearRegression
    F = 1 << 20
    cfg = _cfg(F, fraction=fraction, num_iterations=20)
    synth = SynthConfig.profile("twitter", seed=33, unicode_fraction=0.2)
    batches = [generate_batch(synth, t * 3000, 3000, batch_time_ms=NOW + t) for t in range(3)]
    engines, res = _run_dp(world, batches, cfg, ahead)
    single = DeviceLinearRegression(cfg, device=0)
    for t, full in enumerate(batches):
        r1 = single.train_batch(full, want_pred=False)
        for r in range(world):
            assert res[r][t]["n_kept_global"] == r1["n_kept"]
            assert res[r][t]["iterations"] == r1["iterations"]
            # exact fixed-point GD (csrc/hip/sgd.hip): stats and loss history
            # are the single engine's bit for bit
            assert list(res[r][t]["stats"]) == list(r1["stats"])
            assert list(res[r][t]["loss_history"]) == list(r1["loss_history"])
    # after the same 3 batches every replica IS the single-engine model
    w1 = single.get_weights()
    for r in range(world):
        np.testing.assert_array_equal(engines[r].get_weights(), w1)


def test_dp_rank_with_no_rows(hip_module):
    """A rank whose shard is entirely filtered out still joins every collective."""
    from twitter_stream_ml_amd.ops.lr_engine import DeviceLinearRegression
    from twitter_stream_ml_amd.records.batch import RawBatch
    F = 1000
    cfg = _cfg(F, num_iterations=10)
    good = generate_batch(SynthConfig.profile("twitter", seed=4), 0, 2000, batch_time_ms=NOW)
    bad = generate_batch(SynthConfig.profile("twitter", seed=5, retweet_fraction=0.0), 0, 2000,
                         batch_time_ms=NOW)
    full = RawBatch.concat([good, bad])  # shard 1 keeps nothing
    engines, res = _run_dp(2, [full], cfg)
    assert res[1][0]["n_kept"] == 0 and res[1][0]["n_kept_global"] == res[0][0]["n_kept"]
    single = DeviceLinearRegression(cfg, device=0)
    r1 = single.train_batch(full)
    assert res[0][0]["iterations"] == r1["iterations"]
    np.testing.assert_array_equal(engines[1].get_weights(), single.get_weights())


@pytest.mark.parametrize("ahead", [True, False], ids=["ahead", "inline"])
def test_dp_prep_failure_raises_on_every_rank(hip_module, monkeypatch, ahead):
    """a rank whose local prep fails must not leave its peers
    blocked in the packet all-gather -- the in-line all-reduce carries every
    rank's prep status, so all ranks raise for that batch."""
    from twitter_stream_ml_amd.ops._native import hip
    from twitter_stream_ml_amd.ops.lr_engine import DeviceLinearRegression
    # rank 1's second local prep fails: prepared ahead by its prep thread
    # while batch 0 trains, or in line
    monkeypatch.setenv("TWTML_INJECT_PREP_FAIL", "1:2")
    cfg = _cfg(1000, num_iterations=5)
    group = hip().LoopbackGroup(2)
    engines = [DeviceLinearRegression(cfg, device=0, comm=group.comm(r)) for r in range(2)]
    synth = SynthConfig.profile("twitter", seed=4)
    batches = [generate_batch(synth, t * 2000, 2000, batch_time_ms=NOW + t) for t in range(2)]
    errors = [None, None]
    done = [0, 0]

    def worker(r):
        shards = [b.shard(r, 2) for b in batches]
        try:
            if ahead:
                for sh in shards:
                    engines[r].prefetch(sh)
            for sh in shards:
                engines[r].train_batch(sh, want_pred=False)
                done[r] += 1
        except Exception as e:  # noqa: BLE001 -- checked below
            errors[r] = e

    th = [threading.Thread(target=worker, args=(r,)) for r in range(2)]
    for x in th:
        x.start()
    for x in th:
        x.join(timeout=120)
    assert not any(x.is_alive() for x in th), "a rank is still blocked in a collective"
    assert done == [1, 1], done
    assert "injected" in str(errors[1]), errors
    assert errors[0] is not None and "peer" in str(errors[0]), errors
