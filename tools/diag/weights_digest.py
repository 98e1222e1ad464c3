"""Digest of the LR weights after a few wide batches (one GPU): run from two
trees (the main one and a variant built in another directory) to check that
a kernel variant is bit-identical.  python tools/diag/weights_digest.py"""
import hashlib
import os
import sys

sys.path.insert(0, os.getcwd())   # the tree this is run from, not this file's
import numpy as np  # noqa: E402

from twitter_stream_ml_amd.ops.lr_engine import DeviceLinearRegression, LRDeviceConfig  # noqa: E402
from twitter_stream_ml_amd.sources.synthetic import SynthConfig, generate_batch  # noqa: E402

cfg = SynthConfig.profile("wide", seed=77)
eng = DeviceLinearRegression(LRDeviceConfig(num_text_features=1_000_000, max_rows=200_000, max_units=200_000 * 300,
                                            ingest="utf8"), device=0)
its = []
for i in range(6):
    r = eng.train_batch(generate_batch(cfg, i * 200_000, 200_000, batch_time_ms=1_700_000_000_000 + i),
                        want_pred=False)
    its.append(int(r["iterations"]))
    tiered = bool(r["tiered"])
w = eng.get_weights()
print(f"tiered={tiered} iterations={its} nnz={np.count_nonzero(w)} sha={hashlib.sha256(w.tobytes()).hexdigest()[:16]}")
