"""Diagnostic: stream occupancy of the hybrid / tiered SGD layout on one
batch (how much of the cold SELL stream is padding, hot-dense coverage).
python tools/diag/wide_layout.py [profile] [rows]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from twitter_stream_ml_amd.ops.lr_engine import DeviceLinearRegression, LRDeviceConfig
from twitter_stream_ml_amd.sources.synthetic import SynthConfig, generate_batch

prof = sys.argv[1] if len(sys.argv) > 1 else "wide"
N = int(sys.argv[2]) if len(sys.argv) > 2 else 1000000
cfg = SynthConfig.profile(prof, seed=1234)
raw = generate_batch(cfg, 0, N, batch_time_ms=cfg.now_ms)
eng = DeviceLinearRegression(LRDeviceConfig(num_text_features=1000000, max_rows=N,
                                            max_units=raw.total_units + 1024, lazy_idx=False), device=0)
res = eng.train_batch(raw)
hy = eng._eng.debug_hybrid()
dbg = eng._eng.debug_prepared()
nU = len(dbg["uniq"])
n_near = int(res.get("n_near", nU))
rows = int(res["n_kept"])
L = np.asarray(hy["clen8c"])
cs = np.asarray(hy["cslot"])
cb = np.asarray(dbg["cbase"])
hd = np.asarray(hy["hot_dense"]).view(np.uint8)
nib = (hd & 15).astype(np.int64).sum() + (hd >> 4).astype(np.int64).sum()
plain = int((L < 0).sum())
real = pad = 0
Lh = L[L >= 0]
for c in np.flatnonzero(L >= 0):
    g0, l4 = int(cb[c]), int(L[c])
    blk = cs[g0 * 512:g0 * 512 + l4 * 256]
    r = (blk >= 4) & (blk < 4 + n_near)
    real += int(r.sum()); pad += int(r.size - r.sum())
ent = int(res["entries"])
print(f"profile {prof} rows {rows} active {nU} near {n_near} tiered {res.get('tiered')} iters {res['iterations']}")
print(f"chunks {len(L)} plain {plain} mean cold groups {Lh.mean():.2f}")
print(f"hot entries {nib} ({nib / rows:.1f}/row)  cold real {real} ({real / rows:.1f}/row) pad {pad} "
      f"occupancy {real / max(1, real + pad):.3f}  cold bytes/row {2 * (real + pad) / rows:.1f}")
