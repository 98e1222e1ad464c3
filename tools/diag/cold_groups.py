"""Diagnostic: cold-group occupancy of the hybrid layout on a bench batch
(how many of the SELL cold slots are padding)."""
import numpy as np

from twitter_stream_ml_amd.ops.lr_engine import DeviceLinearRegression, LRDeviceConfig
from twitter_stream_ml_amd.sources.synthetic import SynthConfig, generate_batch

cfg = SynthConfig.profile("bench", seed=1234)
raw = generate_batch(cfg, 0, 200000, batch_time_ms=cfg.now_ms)
eng = DeviceLinearRegression(LRDeviceConfig(num_text_features=1 << 20, max_rows=200000,
                                            max_units=200000 * 300), device=0)
eng.train_batch(raw)
hy = eng._eng.debug_hybrid()
dbg = eng._eng.debug_prepared()
nU = len(dbg["uniq"])
L = hy["clen8c"]
L = L[L >= 0]
cs = hy["cslot"]
cb = dbg["cbase"]
real = pad = 0
per_lane = []
for c in range(0, len(L), 7):
    g0, l8 = int(cb[c]), int(L[c])
    blk = cs[g0 * 512:g0 * 512 + l8 * 256].reshape(l8, 64, 4) if l8 else np.zeros((0, 64, 4))
    r = (blk >= 4) & (blk < 4 + nU)
    real += int(r.sum()); pad += int(r.size - r.sum())
    per_lane.extend(r.sum(axis=(0, 2)).tolist())
pl = np.array(per_lane)
print(f"chunks {len(L)} mean cold 4-groups {L.mean():.2f} hist {np.bincount(L)[:8].tolist()}")
print(f"cold slots real {real} pad {pad} -> occupancy {real / max(1, real + pad):.2f}")
print(f"cold entries per lane: mean {pl.mean():.2f} p50 {np.median(pl):.0f} p90 {np.percentile(pl, 90):.0f} max {pl.max()}")
for G in (8, 4, 2):
    need = []
    for c0 in range(0, len(pl), 64):
        lane = pl[c0:c0 + 64]
        need.append(int(np.ceil(lane.max() / G)) * G if lane.size else 0)
    print(f"group {G}: slots per lane (chunk max) mean {np.mean(need):.2f}")
