"""Config-4 k-means oracle test (tests/test_gpu_kmeans.py::..._bench_scale_...)
diagnostics: replicate its taint logic and print every clean cluster whose
weight differs, with per-engine label counts and split evidence."""
import sys

import numpy as np

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
from test_gpu_kmeans import _gap_check  # noqa: E402
from twitter_stream_ml_amd.models.kmeans import CpuKMeans, kmeans_features  # noqa: E402
from twitter_stream_ml_amd.ops.kmeans_engine import DeviceKMeans, KMDeviceConfig  # noqa: E402
from twitter_stream_ml_amd.sources.synthetic import SynthConfig, generate_batch  # noqa: E402

NOW = 1_700_000_000_000
k, td, rows = 1024, 62, 262_144
dev = DeviceKMeans(KMDeviceConfig(k=k, text_dims=td, max_rows=rows, max_units=rows * 300, seed=5), device=0)
cpu = CpuKMeans(k, 2 + td, seed=5)
synth = SynthConfig.profile("wide", seed=31)
tainted = np.zeros(k, bool)
for t in range(3):
    raw = generate_batch(synth, t * rows, rows, batch_time_ms=NOW + t * 5000)
    cg_old, wg_old = dev.get_state()
    cc_old, wc_old = cpu.state.centers.copy(), cpu.state.weights.copy()
    dev.update_raw(raw, want_pred=False)
    lab_g = dev._eng.debug_labels().astype(np.int64)
    X, _ = kmeans_features(raw, td)
    rc = cpu.update_batch(X)
    Xs = rc["scaled"]
    lab_c = np.asarray(rc["labels"])
    ok_c, top_c = _gap_check(Xs, cc_old)
    ok_g, top_g = _gap_check(Xs, cg_old)
    bad = ~ok_c | ~ok_g | (top_c[:, 0] != top_g[:, 0])
    tainted[top_c[bad].ravel()] = True
    tainted[top_g[bad].ravel()] = True
    cg, wg = dev.get_state()
    wc = cpu.state.weights
    nb_g = np.bincount(lab_g, minlength=k)
    nb_c = np.bincount(lab_c, minlength=k)
    print(f"batch {t}: bad {int(bad.sum())} tainted {int(tainted.sum())} "
          f"argmax w gpu {int(np.argmax(wg))} cpu {int(np.argmax(wc))}  argmin w gpu {int(np.argmin(wg))} "
          f"cpu {int(np.argmin(wc))}  min/max gpu {wg.min() / wg.max():.3e} cpu {wc.min() / wc.max():.3e}")
    # labels that disagree on points NOT flagged bad
    dis = np.flatnonzero((lab_g != lab_c) & ~bad)
    print(f"  label disagreements on not-bad points: {dis.shape[0]}")
    for p in dis[:20]:
        print(f"    p={p} gpu={lab_g[p]} cpu={lab_c[p]} top_c={top_c[p].tolist()} top_g={top_g[p].tolist()}")
    mism = np.flatnonzero(~tainted & ~np.isclose(wg, wc, rtol=1e-9, atol=1e-9))
    for j in mism[:20]:
        print(f"  cluster {j}: w_gpu {wg[j]:.6f} w_cpu {wc[j]:.6f} old gpu {wg_old[j]:.6f} old cpu {wc_old[j]:.6f} "
              f"n_gpu {nb_g[j]} n_cpu {nb_c[j]} |dc| {np.abs(cg[j] - cpu.state.centers[j]).max():.3e}")
