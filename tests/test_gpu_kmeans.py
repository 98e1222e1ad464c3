"""GPU streaming k-means engine vs the fp64 CPU engine / MLlib oracle.

Covers the KMeans driver's per-batch pipeline (``KMeans.scala:77-115``):
isRetweet filter, dense features (+ hashed bigram dims), the per-batch
StandardScaler, MFMA (and scalar) assignment, decayed update with the
dying-cluster split, prediction with the updated model, and the data-parallel
path through the loopback communicator.
"""
import threading

import numpy as np
import pytest

from twitter_stream_ml_amd.models.kmeans import CpuKMeans, kmeans_features
from twitter_stream_ml_amd.oracle.mllib import find_closest
from twitter_stream_ml_amd.sources.synthetic import SynthConfig, generate_batch

pytestmark = pytest.mark.gpu
NOW = 1_700_000_000_000


def _cfg(k, text_dims=0, **kw):
    from twitter_stream_ml_amd.ops.kmeans_engine import KMDeviceConfig
    return KMDeviceConfig(k=k, text_dims=text_dims, max_rows=8192, max_units=8192 * 300, **kw)


def _batches(n=4, rows=4000, seed=21, **kw):
    synth = SynthConfig.profile("twitter", seed=seed, **kw)
    return [generate_batch(synth, t * rows, rows, batch_time_ms=NOW + t) for t in range(n)]


def _well_conditioned(X, centers, rel=1e-9):
    if X.shape[0] * centers.shape[0] > 4_000_000:
        return np.ones(X.shape[0], bool)
    d = ((X[:, None, :] - centers[None]) ** 2).sum(2)
    if centers.shape[0] < 2:
        return np.ones(X.shape[0], bool)
    s = np.sort(d, 1)
    return (s[:, 1] - s[:, 0]) > rel * np.maximum(s[:, 0], 1e-300)


def _check_state(dev, cpu, rtol=2e-5):
    c, w = dev.get_state()
    scale = max(1.0, float(np.abs(cpu.state.centers).max()))
    np.testing.assert_allclose(w, cpu.state.weights, rtol=rtol, atol=1e-9)
    np.testing.assert_allclose(c, cpu.state.centers, rtol=rtol, atol=rtol * scale)


@pytest.mark.parametrize("k,text_dims,mfma,precision", [
    (3, 0, True, "fp32"), (3, 0, False, "fp32"), (5, 8, True, "fp32"), (64, 30, True, "bf16x3"),
    (64, 30, True, "fp32"), (1024, 0, True, "fp32"), (200, 126, True, "bf16x3"),
    (1024, 14, True, "bf16x3"), (1024, 62, True, "bf16x3")])   # the last: bench config 4 (d = 64)
def test_kmeans_matches_cpu(hip_module, k, text_dims, mfma, precision):
    from twitter_stream_ml_amd.ops.kmeans_engine import DeviceKMeans
    dev = DeviceKMeans(_cfg(k, text_dims, mfma=mfma, precision=precision, seed=5), device=0)
    cpu = CpuKMeans(k, 2 + text_dims, seed=5)
    c0, w0 = dev.get_state()
    np.testing.assert_array_equal(c0, cpu.state.centers)
    for raw in _batches(unicode_fraction=0.2):
        c_old = cpu.state.centers.copy()
        r = dev.update_raw(raw)
        X, _ = kmeans_features(raw, text_dims)
        rc = cpu.update_batch(X)
        assert r["n"] == rc["n"] == X.shape[0] == r["n_local"]
        np.testing.assert_allclose(r["std"], rc["std"], rtol=1e-6)
        Xs = rc["scaled"]
        # Points (near-)equidistant from the two halves of a just-split cluster
        # (1e-14 apart) are ill-conditioned: 1e-15 noise in the centres flips
        # them in fp64 too.  (1) The prediction (updated model) must agree
        # with fp64 find_closest against the engine's own updated centres
        # wherever the best/second gap is resolvable.
        c_new = dev.get_state()[0]
        want = find_closest(c_new, Xs)
        pred = np.asarray(r["pred"])
        mismatch = np.count_nonzero((pred != want) & _well_conditioned(Xs, c_new))
        assert mismatch <= 2, mismatch
        # (2) The update: exact unless an update-time assignment (old centres)
        # was ill-conditioned; a flip there moves one point between clusters.
        n_ill = np.count_nonzero(~_well_conditioned(Xs, c_old))
        if n_ill == 0:
            _check_state(dev, cpu)
        else:
            w_dev = dev.get_state()[1]
            np.testing.assert_allclose(w_dev.sum(), cpu.state.weights.sum(), rtol=1e-9)
            assert np.abs(w_dev - cpu.state.weights).sum() <= 2 * n_ill + 1e-6
            cpu.set_state(*dev.get_state())


def test_kmeans_points_unit_and_set_state(hip_module):
    from twitter_stream_ml_amd.ops.kmeans_engine import DeviceKMeans
    dev = DeviceKMeans(_cfg(4, 0, time_unit="points", seed=9), device=0)
    cpu = CpuKMeans(4, 2, time_unit="points", seed=9)
    rng = np.random.default_rng(0)
    c = rng.normal(size=(4, 2))
    w = np.array([3.0, 1.0, 0.5, 2.0])
    dev.set_state(c, w)
    cpu.set_state(c, w)
    for raw in _batches(n=3, seed=4):
        dev.update_raw(raw)
        cpu.update_batch(kmeans_features(raw)[0])
        _check_state(dev, cpu)


def test_kmeans_empty_batch_is_noop(hip_module):
    from twitter_stream_ml_amd.ops.kmeans_engine import DeviceKMeans
    from twitter_stream_ml_amd.records.batch import RawBatch
    dev = DeviceKMeans(_cfg(3, seed=1), device=0)
    c0, w0 = dev.get_state()
    raw = _batches(n=1)[0]
    none_rt = RawBatch(raw.text, raw.offsets, np.zeros_like(raw.is_retweet), raw.scalars, NOW)
    r = dev.update_raw(none_rt)
    assert r["n"] == 0 and r["n_local"] == 0
    c1, w1 = dev.get_state()
    np.testing.assert_array_equal(c0, c1)
    np.testing.assert_array_equal(w0, w1)


@pytest.mark.parametrize("world", [2, 3])
def test_kmeans_dp_loopback(hip_module, world):
    """DP k-means equals the single engine bit for bit, batch after batch:
    a point's label depends only on the point and the (replicated) centres,
    and the scaler moments and per-cluster sums are exact int64 sums
    (``csrc/hip/kmeans.hip`` K11 / K9), equal in any order over any sharding
    (the fp64 sums needed conditioning checks here)."""
    from twitter_stream_ml_amd.ops.kmeans_engine import DeviceKMeans
    cfg = _cfg(6, 4, seed=2)
    group = hip_module.LoopbackGroup(world)
    engines = [DeviceKMeans(cfg, device=0, comm=group.comm(r)) for r in range(world)]
    batches = _batches(n=3, seed=8)
    errors, out = [], [[None] * len(batches) for _ in range(world)]
    states = [[None] * len(batches) for _ in range(world)]

    def worker(r):
        try:
            for t, full in enumerate(batches):
                out[r][t] = engines[r].update_raw(full.shard(r, world))
                states[r][t] = engines[r].get_state()
        except Exception as e:  # pragma: no cover
            errors.append(e)

    th = [threading.Thread(target=worker, args=(r,)) for r in range(world)]
    for x in th:
        x.start()
    for x in th:
        x.join(timeout=300)
    assert not errors, errors
    single = DeviceKMeans(cfg, device=0)
    for t, full in enumerate(batches):
        r1 = single.update_raw(full)
        c1, w1 = single.get_state()
        assert sum(out[r][t]["n_local"] for r in range(world)) == r1["n"]
        # contiguous shards: the ranks' labels concatenate to the single engine's
        pred = np.concatenate([np.asarray(out[r][t]["pred"]) for r in range(world)])
        np.testing.assert_array_equal(pred, np.asarray(r1["pred"]))
        for r in range(world):
            assert out[r][t]["n"] == r1["n"]
            np.testing.assert_array_equal(out[r][t]["std"], r1["std"])
            c, w = states[r][t]
            np.testing.assert_array_equal(c, c1)
            np.testing.assert_array_equal(w, w1)


def test_kmeans_utf8_ingest_equals_wire(hip_module):
    """The end-to-end bench stages k-means batches as raw UTF-8 (device
    decode); per batch it must equal the host-packed wire ingest bit for bit:
    same points, scaler, labels and model (the two paths order rows
    differently, which the exact integer sums do not see)."""
    from twitter_stream_ml_amd.ops.kmeans_engine import DeviceKMeans
    from twitter_stream_ml_amd.ops.lr_engine import encode_utf8
    cfg = _cfg(16, 14, seed=6)
    a, b = DeviceKMeans(cfg, device=0), DeviceKMeans(cfg, device=0)
    for raw in _batches(n=3, seed=31, unicode_fraction=0.3, special_fraction=0.02):
        ra = a.update_raw(raw)
        hb = b.staging(0).load_utf8(raw, encode_utf8(raw), copy_text=True)
        b.submit(hb, 0)
        rb = b.process(0)
        assert ra["n"] == rb["n"]
        np.testing.assert_array_equal(rb["std"], ra["std"])
        np.testing.assert_array_equal(np.asarray(ra["pred"]), np.asarray(rb["pred"]))
        ca, wa = a.get_state()
        cb, wb = b.get_state()
        np.testing.assert_array_equal(cb, ca)
        np.testing.assert_array_equal(wb, wa)


def _split_twins(C, w):
    """Cluster pairs made by a dying-cluster split in the last update: equal
    weights and centres 2e-14 (relative) apart (``kmeans_update``)."""
    order = np.argsort(w, kind="stable")
    ws = w[order]
    out = []
    for i in np.flatnonzero(ws[1:] == ws[:-1]):
        a, b = int(order[i]), int(order[i + 1])
        tol = 1e-12 * max(1.0, float(np.abs(C[a]).max()))
        if ws[i] > 0 and np.abs(C[a] - C[b]).max() <= tol:
            out.append((a, b))
    return out


def _gap_check(X, C, rel=1e-9, chunk=16384):
    """Per point: the two nearest centres (fp64, |x|^2 - 2 x.c + |c|^2 in
    chunks) and whether the best / second gap is resolvable."""
    n = X.shape[0]
    ok = np.empty(n, bool)
    top = np.empty((n, 2), np.int64)
    cn = np.einsum("ij,ij->i", C, C)
    for s in range(0, n, chunk):
        x = X[s:s + chunk]
        xn = np.einsum("ij,ij->i", x, x)
        d = xn[:, None] - 2.0 * (x @ C.T) + cn[None]
        i2 = np.argpartition(d, 1, axis=1)[:, :2]
        d2 = np.take_along_axis(d, i2, 1)
        o = np.argsort(d2, axis=1)
        i2, d2 = np.take_along_axis(i2, o, 1), np.take_along_axis(d2, o, 1)
        top[s:s + chunk] = i2
        # cancellation in the expanded form: resolve against |x|^2 + |c|^2 too
        ok[s:s + chunk] = (d2[:, 1] - d2[:, 0]) > rel * np.maximum(np.abs(d2[:, 0]), 1e-9 * (xn + cn[i2[:, 0]]))
    return ok, top


def test_kmeans_config4_bench_scale_matches_oracle(hip_module):
    """Bench config 4 at scale: k = 1024, d = 64 (2 numeric + 62 hashed bigram
    dims), 262,144 tweets per batch, 3 warm-started batches against the fp64
    oracle (``KMeans.scala:100-113``: StandardScaler, update, predict) WITHOUT
    re-seeding it from the GPU.  Exact (fp64 summation order aside) for every
    cluster whose point set the two engines provably agree on; a cluster is
    set aside ("tainted") once an ill-conditioned point (best / second gap
    below 1e-9, e.g. the twin halves of a dying-cluster split, 1e-14 apart)
    or a point the two models assign differently touched it."""
    from twitter_stream_ml_amd.ops.kmeans_engine import DeviceKMeans, KMDeviceConfig
    k, td, rows = 1024, 62, 262_144
    dev = DeviceKMeans(KMDeviceConfig(k=k, text_dims=td, max_rows=rows, max_units=rows * 300, seed=5), device=0)
    cpu = CpuKMeans(k, 2 + td, seed=5)
    synth = SynthConfig.profile("wide", seed=31)
    tainted = np.zeros(k, bool)
    for t in range(3):
        raw = generate_batch(synth, t * rows, rows, batch_time_ms=NOW + t * 5000)
        c_gpu_old = dev.get_state()[0]
        c_cpu_old = cpu.state.centers.copy()
        r = dev.update_raw(raw)
        X, _ = kmeans_features(raw, td)
        rc = cpu.update_batch(X)
        assert r["n"] == rc["n"] == X.shape[0]
        np.testing.assert_allclose(r["std"], rc["std"], rtol=1e-6)
        Xs = rc["scaled"]
        ok_c, top_c = _gap_check(Xs, c_cpu_old)
        ok_g, top_g = _gap_check(Xs, c_gpu_old)
        bad = ~ok_c | ~ok_g | (top_c[:, 0] != top_g[:, 0])
        tainted[top_c[bad].ravel()] = True
        tainted[top_g[bad].ravel()] = True
        c, w = dev.get_state()
        # a dying-cluster split gives the dying cluster half of the largest
        # one's weight: a tainted largest taints its (point-less) partner
        for cc, ww in ((c, w), (cpu.state.centers, cpu.state.weights)):
            for a, b in _split_twins(cc, ww):
                if tainted[a] or tainted[b]:
                    tainted[a] = tainted[b] = True
        clean = ~tainted
        print(f"batch {t}: ill/disagreeing points {int(bad.sum())}, tainted clusters {int(tainted.sum())}")
        assert tainted.mean() < 0.05, int(tainted.sum())
        np.testing.assert_allclose(w.sum(), cpu.state.weights.sum(), rtol=1e-12)
        np.testing.assert_allclose(w[clean], cpu.state.weights[clean], rtol=1e-9, atol=1e-9)
        scale = max(1.0, float(np.abs(cpu.state.centers).max()))
        np.testing.assert_allclose(c[clean], cpu.state.centers[clean], rtol=2e-5, atol=2e-5 * scale)
        # predictions with the updated model, where both models agree and the
        # point is well conditioned against the GPU's centres
        ok_n, top_n = _gap_check(Xs, c)
        pred = np.asarray(r["pred"])
        sel = ok_n & clean[top_n[:, 0]]
        assert np.count_nonzero(pred[sel] != top_n[sel, 0]) == 0


@pytest.mark.parametrize("text_dims", [1, 8, 14, 62, 64, 65, 126])
def test_kmeans_features_exact(hip_module, text_dims):
    """The device feature rows (before scaling) equal the host featurizer's
    exactly: the lane-private histogram kernel (text_dims <= 64, config 4's
    62) and the shared-histogram kernel above it; padding columns are 0."""
    from twitter_stream_ml_amd.ops.kmeans_engine import DeviceKMeans
    dev = DeviceKMeans(_cfg(16, text_dims, seed=3), device=0)
    for raw in _batches(n=2, rows=6000, seed=33, unicode_fraction=0.4):
        dev.update_raw(raw, want_pred=False)
        got = np.asarray(dev._eng.debug_features())
        want, _ = kmeans_features(raw, text_dims)
        assert got.shape[0] == want.shape[0]
        np.testing.assert_array_equal(got[:, :2 + text_dims], want.astype(np.float32))
        assert not got[:, 2 + text_dims:].any()


_VARIANT_SCRIPT = r"""
import hashlib, sys
import numpy as np
sys.path.insert(0, sys.argv[1])
from twitter_stream_ml_amd.ops.kmeans_engine import DeviceKMeans, KMDeviceConfig
from twitter_stream_ml_amd.sources.synthetic import SynthConfig, generate_batch
h = hashlib.sha256()
for k, td in ((1024, 62), (200, 14), (64, 30), (96, 126)):
    dev = DeviceKMeans(KMDeviceConfig(k=k, text_dims=td, max_rows=8192, max_units=8192 * 300,
                                      precision="bf16x3", seed=3), device=0)
    synth = SynthConfig.profile("twitter", seed=17, unicode_fraction=0.2)
    for t in range(3):
        r = dev.update_raw(generate_batch(synth, t * 6000, 6000, batch_time_ms=1_700_000_000_000 + t))
        h.update(np.asarray(r["pred"]).tobytes())
    c, w = dev.get_state()
    h.update(c.tobytes()); h.update(w.tobytes())
print("DIGEST", h.hexdigest())
"""


def test_kmeans_assign_variants_bitwise(hip_module, tmp_path):
    """The bf16x3 assignment variants (``TWTML_KM_ASSIGN``: pipe, the default
    = epilogue software-pipelined behind the next tile's MFMAs; lds, lds2, reg)
    issue the same MFMAs in the same order, so labels, refine routing and
    the updated model are identical bit for bit (d = 16, 32, 64, 128)."""
    import os
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    script = tmp_path / "km_variant.py"
    script.write_text(_VARIANT_SCRIPT)
    digests = {}
    for v in ("lds", "pipe", "lds2", "reg"):
        env = dict(os.environ, TWTML_KM_ASSIGN=v)
        out = subprocess.run([sys.executable, str(script), repo], env=env, capture_output=True,
                             text=True, timeout=240)
        assert out.returncode == 0, out.stderr[-2000:]
        digests[v] = [ln for ln in out.stdout.splitlines() if ln.startswith("DIGEST")][-1]
    assert len(set(digests.values())) == 1, digests
