"""Diagnose GPU vs CPU k-means label disagreements (batch by batch)."""
import sys
import numpy as np
import torch  # noqa: F401
from twitter_stream_ml_amd.models.kmeans import CpuKMeans, kmeans_features
from twitter_stream_ml_amd.ops.kmeans_engine import DeviceKMeans, KMDeviceConfig
from twitter_stream_ml_amd.sources.synthetic import SynthConfig, generate_batch

k, td = int(sys.argv[1]), int(sys.argv[2])
dev = DeviceKMeans(KMDeviceConfig(k=k, text_dims=td, max_rows=8192, max_units=8192 * 300, seed=5), 0)
cpu = CpuKMeans(k, 2 + td, seed=5)
synth = SynthConfig.profile("twitter", seed=21, unicode_fraction=0.2)
for t in range(4):
    raw = generate_batch(synth, t * 4000, 4000, batch_time_ms=1_700_000_000_000 + t)
    c_before = cpu.state.centers.copy()
    dc, dw = dev.get_state()
    print(f"batch {t}: state diff centres {np.abs(dc - c_before).max():.3e} weights {np.abs(dw - cpu.state.weights).max():.3e}")
    r = dev.update_raw(raw)
    X, _ = kmeans_features(raw, td)
    rc = cpu.update_batch(X)
    Xs = rc["scaled"]
    pred = np.asarray(r["pred"])
    C = cpu.state.centers
    d = ((Xs[:, None, :] - C[None]) ** 2).sum(2)
    bad = np.nonzero(pred != rc["pred"])[0]
    print(f"  n={X.shape[0]} mismatches={bad.size} std maxrel={np.max(np.abs(r['std'] - rc['std']) / np.maximum(rc['std'], 1e-300)):.2e}")
    for i in bad[:8]:
        a, b = rc["pred"][i], pred[i]
        print(f"   pt {i}: cpu {a} d={d[i, a]:.17g} gpu {b} d={d[i, b]:.17g} rel={(d[i, b] - d[i, a]) / d[i, a]:.3e} |x|^2={np.dot(Xs[i], Xs[i]):.4g}")
    cpu.set_state(*dev.get_state())
