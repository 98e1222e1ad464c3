"""Exact, partition-independent GD arithmetic (``csrc/hip/sgd.hip``).

The engine's forward dot is an int32 fixed-point sum of count * w_fix and
every gradient / loss / numeric-feature sum is an int64 fixed-point sum
(scales chosen per iteration from values every workgroup and rank holds bit
for bit).  A batch's weights therefore must not depend on HOW its entries are
laid out or split:

* the hybrid dense-hot path vs the plain LDS stream (``hybrid=False``);
* the tiered layout with a tiny LDS tier (most slots far) vs the default;
* any iteration grid (rows split over 1..N workgroups).

Bitwise equality here is what makes DP over any sharding bit-identical to
one GPU (``tests/test_gpu_dp_procs.py``).  Reference semantics:
``GradientDescent.runMiniBatchSGD`` [upstream MLlib 1.6.1] via
``LinearRegression.scala:28-32,86``.
"""
import numpy as np
import pytest

from twitter_stream_ml_amd.sources.synthetic import SynthConfig, generate_batch

pytestmark = pytest.mark.gpu
NOW = 1_700_000_000_000


def _run(profile, F, hash, rows, nb, seed, monkeypatch=None, env=None, **kw):
    from twitter_stream_ml_amd.ops.lr_engine import DeviceLinearRegression, LRDeviceConfig
    if monkeypatch is not None:
        for k, v in (env or {}).items():
            monkeypatch.setenv(k, v)
    eng = DeviceLinearRegression(LRDeviceConfig(num_text_features=F, hash=hash, max_rows=rows,
                                                max_units=rows * 300, **kw), device=0)
    if monkeypatch is not None:
        for k in (env or {}):
            monkeypatch.delenv(k)
    synth = SynthConfig.profile(profile, seed=seed)
    meta = []
    for t in range(nb):
        raw = generate_batch(synth, t * rows, rows, batch_time_ms=NOW + t * 5000)
        r = eng.train_batch(raw, want_pred=True)
        assert not r["diverged"]
        meta.append((r["iterations"], bool(r["tiered"]), r["n_near"], list(r["stats"]), list(r["loss_history"]),
                     np.asarray(r["pred"]).copy()))
    w = eng.get_weights()
    del eng
    return w, meta


def _same(a, b):
    wa, ma = a
    wb, mb = b
    for (ia, _, _, sa, la, pa), (ib, _, _, sb, lb, pb) in zip(ma, mb):
        assert ia == ib
        assert sa == sb                     # batch stats: integer-valued fp64 sums
        assert la == lb                     # loss history: int64 fixed-point sums
        np.testing.assert_array_equal(pa, pb)
    np.testing.assert_array_equal(wa, wb)


def test_hybrid_vs_plain_layout_bitwise(hip_module):
    """Toy data: hot-dense + cold stream vs every entry through the LDS stream."""
    a = _run("bench", 1 << 20, "java", 30000, 3, seed=11)
    b = _run("bench", 1 << 20, "java", 30000, 3, seed=11, hybrid=False)
    _same(a, b)


def test_grid_split_bitwise(hip_module):
    """The same batches over 1, 7 and the default number of workgroups."""
    a = _run("wide", 1 << 20, "java", 20000, 2, seed=12)
    for g in (1, 7):
        _same(a, _run("wide", 1 << 20, "java", 20000, 2, seed=12, sgd_grid=g))


def test_near_tier_size_bitwise(hip_module, monkeypatch):
    """Tiered with the default LDS tier vs a 512-slot tier (most entries far:
    int32 LDS row sums forward, CSC segmented int64 sums backward)."""
    a = _run("wide", 1 << 20, "java", 20000, 2, seed=13)
    assert a[1][0][1]                       # tiered
    b = _run("wide", 1 << 20, "java", 20000, 2, seed=13, monkeypatch=monkeypatch,
             env={"TWTML_NEAR_CAP": "512"})
    assert b[1][0][2] == 512
    _same(a, b)


def test_forced_tiered_vs_hybrid_bitwise(hip_module, monkeypatch):
    """Toy data: the hybrid layout vs the tiered one forced with a 256-slot tier."""
    a = _run("bench", 1 << 20, "java", 20000, 2, seed=14)
    b = _run("bench", 1 << 20, "java", 20000, 2, seed=14, monkeypatch=monkeypatch,
             env={"TWTML_FORCE_TIERED": "1", "TWTML_NEAR_CAP": "256"})
    assert b[1][0][1] and not a[1][0][1]
    _same(a, b)


def test_divergence_stops_training(hip_module):
    """A step size far beyond stability: the residual bound leaves the
    fixed-point range within a few iterations -- the engine stops, flags the
    batch diverged and keeps finite weights (MLlib's fp64 model would reach
    Inf/NaN and ``Utils.round`` throw, ``Utils.scala:3-7``)."""
    from twitter_stream_ml_amd.ops.lr_engine import DeviceLinearRegression, LRDeviceConfig
    eng = DeviceLinearRegression(LRDeviceConfig(num_text_features=1 << 20, max_rows=8000, max_units=8000 * 300,
                                                step_size=1e4), device=0)
    synth = SynthConfig.profile("bench", seed=15)
    flags = []
    for t in range(3):
        r = eng.train_batch(generate_batch(synth, t * 8000, 8000, batch_time_ms=NOW + t * 5000))
        flags.append((bool(r["diverged"]), r["iterations"], r["stats"][0]))
    assert flags[0][0] and flags[0][2] > 0, flags   # the first batch's prequential pass ran
    # the model stays diverged (like NaN weights): later batches are not trained
    assert all(f[0] and f[1] == 0 and f[2] == 0 for f in flags[1:]), flags
    w = eng.get_weights()
    assert np.isfinite(w).all()
    eng.set_weights(np.zeros_like(w))       # a new model trains again
    r = eng.train_batch(generate_batch(synth, 99 * 8000, 8000, batch_time_ms=NOW))
    assert r["diverged"] and r["stats"][0] > 0


def test_batch_stats_exact_int64_and_spill(hip_module):
    """the prequential moments are exact integers (k_batch_stats,
    int64 with 32-bit limbs for the squares): n, sum y, sum y^2, sum p, sum p^2
    and sum (y - p)^2 equal Python's exact integer sums of the engine's own
    (label, rounded prediction) pairs, correctly rounded once.  Predictions
    beyond 2^31 go through the counted fp64 spill path."""
    from twitter_stream_ml_amd.ops.lr_engine import DeviceLinearRegression, LRDeviceConfig
    F = 1 << 20
    eng = DeviceLinearRegression(LRDeviceConfig(num_text_features=F, max_rows=8192, max_units=8192 * 300,
                                                num_iterations=3), device=0)
    synth = SynthConfig.profile("twitter", seed=21)

    def exact(res):
        y = [int(v) for v in np.asarray(res["real"], np.float64)]
        p = [int(v) for v in np.asarray(res["pred"], np.float64)]
        return [float(len(y)), float(sum(y)), float(sum(a * a for a in y)), float(sum(p)),
                float(sum(b * b for b in p)), float(sum((a - b) ** 2 for a, b in zip(y, p)))]

    w = np.random.default_rng(3).normal(0.0, 2e5, F + 4)
    w[F:] = 0.0
    # |predictions| ~1e6-1e7 (< 2^31): sum (y - p)^2 ~1e17, beyond fp64's exact
    # integers -- only the int64 limbs give order-free bits
    eng.set_weights(w)
    res = eng.train_batch(generate_batch(synth, 0, 4000, batch_time_ms=NOW), want_pred=True)
    assert res["stats_spill"] == 0
    assert list(res["stats"]) == exact(res)
    eng.set_weights(np.where(np.arange(F + 4) < F, 3e7, 0.0))   # most |predictions| >= 2^31
    res = eng.train_batch(generate_batch(synth, 4000, 4000, batch_time_ms=NOW), want_pred=True)
    big = int(np.sum(np.abs(np.asarray(res["pred"], np.float64)) >= 2.0 ** 31))
    assert res["stats_spill"] == big and big > res["n_kept"] // 2
    np.testing.assert_allclose(res["stats"], exact(res), rtol=1e-12)
