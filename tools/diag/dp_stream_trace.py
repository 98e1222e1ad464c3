"""DP prepare-ahead evidence: 2 engines on one GPU through
the in-process loopback communicator, wide-vocabulary shards, batches
prefetched as the streaming runtime does.  Run under
`rocprofv3 --kernel-trace --output-format csv`; tools/diag/stream_kernels.py
then lists which kernels ran on each HIP stream (the compute stream must
carry only the GD loop: no decode / featurize / remap / tier kernels)."""
import os
import sys
import threading

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from twitter_stream_ml_amd.ops._native import hip  # noqa: E402
from twitter_stream_ml_amd.ops.lr_engine import DeviceLinearRegression, LRDeviceConfig  # noqa: E402
from twitter_stream_ml_amd.sources.synthetic import SynthConfig, generate_batch  # noqa: E402

WORLD, ROWS, NB = 2, 131072, 6
synth = SynthConfig.profile("wide", seed=11)
batches = [generate_batch(synth, t * ROWS, ROWS, batch_time_ms=synth.now_ms + t) for t in range(NB)]
cfg = LRDeviceConfig(num_text_features=1_000_000, max_rows=ROWS, max_units=ROWS * 300)
group = hip().LoopbackGroup(WORLD)
engines = [DeviceLinearRegression(cfg, device=0, comm=group.comm(r)) for r in range(WORLD)]
out = [[] for _ in range(WORLD)]


def worker(r):
    eng = engines[r]
    shards = [b.shard(r, WORLD) for b in batches]
    nxt = 0   # next shard to prefetch: strictly in order, stop at the first refusal
    for t, sh in enumerate(shards):
        nxt = max(nxt, t + 1)
        while nxt < NB and nxt <= t + eng.raw_slots - 1 and eng.prefetch(shards[nxt]):
            nxt += 1
        res = eng.train_batch(sh, want_pred=False)
        out[r].append((res["iterations"], round(res["prep_ms"], 3), round(res["train_ms"], 3)))


th = [threading.Thread(target=worker, args=(r,)) for r in range(WORLD)]
for x in th:
    x.start()
for x in th:
    x.join(timeout=300)
for r in range(WORLD):
    print(f"rank {r}: (iterations, prep_ms, train_ms) per batch: {out[r]}")
