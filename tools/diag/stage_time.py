"""Host staging cost breakdown of one 1M-tweet batch (GPU box): load_utf8 vs
submit, k-means k=3 d=2 (no text) and LR toy (UTF-8 text by DMA)."""
import time

import numpy as np
import torch

from twitter_stream_ml_amd.ops.kmeans_engine import DeviceKMeans, KMDeviceConfig, no_text
from twitter_stream_ml_amd.ops.lr_engine import HostBatchView, encode_utf8, register_host
from twitter_stream_ml_amd.sources.synthetic import SynthConfig, generate_batch

torch.cuda.set_device(0)
B = 1_000_000
s = SynthConfig.profile("bench", seed=1)
raw = generate_batch(s, 0, B, batch_time_ms=s.now_ms)
eng = DeviceKMeans(KMDeviceConfig(k=3, text_dims=0, half_life=5.0, max_rows=B, max_units=raw.total_units + 1024,
                                  seed=1), device=0)
hb = HostBatchView(B, raw.total_units + 1024)
hb._hb.scalar_cols = 2
u8 = no_text(raw)
u8t = encode_utf8(raw)
register_host(u8t.data)
for name, u in (("no_text", u8), ("utf8", u8t)):
    tl, ts = [], []
    for i in range(30):
        t0 = time.perf_counter()
        hb.load_utf8(raw, u, copy_text=False)
        t1 = time.perf_counter()
        if name == "no_text":
            eng.submit(hb, i % eng.raw_slots)
            eng.process(i % eng.raw_slots, want_pred=False)
        t2 = time.perf_counter()
        tl.append(t1 - t0)
        ts.append(t2 - t1)
    print(f"{name}: load p50 {np.median(tl) * 1e3:.3f} ms  submit+process p50 {np.median(ts) * 1e3:.3f} ms", flush=True)
# load_utf8 pieces: scalar packing alone
sc = np.ascontiguousarray(raw.scalars, dtype=np.int64)
tp = []
for i in range(30):
    t0 = time.perf_counter()
    hb._hb.pack_scalars(B)
    tp.append(time.perf_counter() - t0)
print(f"pack_scalars p50 {np.median(tp) * 1e3:.3f} ms", flush=True)
