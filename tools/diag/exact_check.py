"""Diagnostic: where does a grid change alter the weights?  Trains one batch
with 1..N GD iterations at different iteration grids and reports mismatches
(numeric slots vs text features, hot ids)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from twitter_stream_ml_amd.ops.lr_engine import DeviceLinearRegression, LRDeviceConfig  # noqa: E402
from twitter_stream_ml_amd.sources.synthetic import SynthConfig, generate_batch  # noqa: E402

prof = sys.argv[1] if len(sys.argv) > 1 else "wide"
rows = int(sys.argv[2]) if len(sys.argv) > 2 else 20000
F = 1 << 20
raw = generate_batch(SynthConfig.profile(prof, seed=12), 0, rows, batch_time_ms=1_700_000_000_000)
for iters in (1, 2, 3, 5):
    ws = {}
    for g in (0, 1, 7):
        eng = DeviceLinearRegression(LRDeviceConfig(num_text_features=F, max_rows=rows, max_units=rows * 300,
                                                    num_iterations=iters, sgd_grid=g, lazy_idx=False), device=0)
        r = eng.train_batch(raw)
        ws[g] = (eng.get_weights(), r["iterations"], list(r["loss_history"]), r["n_near"], r["tiered"])
        if g == 0:
            hy = eng._eng.debug_hybrid()
            dbg = eng._eng.debug_prepared()
        del eng
    w0 = ws[0][0]
    for g in (1, 7):
        w = ws[g][0]
        d = np.flatnonzero(w != w0)
        num = int(np.sum(d >= F))
        print(f"iters {iters} grid {g}: it {ws[g][1]}/{ws[0][1]} loss_eq {ws[g][2] == ws[0][2]} "
              f"mismatch {len(d)} (numeric {num}) maxrel "
              f"{(np.abs(w[d] - w0[d]) / np.maximum(np.abs(w0[d]), 1e-300)).max() if len(d) else 0:.2e} "
              f"tiered {ws[0][4]} n_near {ws[0][3]}")
        if len(d) and iters == 1:
            print("  first diffs:", [(int(i), float(w0[i]), float(w[i])) for i in d[:5]])
