#!/usr/bin/env python3
"""Probe: can two ranks share one GPU through the engine's RCCL communicator?

If RCCL accepts it, this exercises the data-parallel engine path (flag MAX
all-reduce, per-rank counts, per-iteration gradient all-reduce, stats
all-reduce) on a single-GPU box and checks DP == 1-process on the
concatenated batch.  Launched as:
  python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \
      --master-port 29511 tools/dp_same_gpu_probe.py
"""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from twitter_stream_ml_amd.ops._native import hip  # noqa: E402
from twitter_stream_ml_amd.ops.lr_engine import DeviceLinearRegression, LRDeviceConfig  # noqa: E402
from twitter_stream_ml_amd.records.batch import RawBatch  # noqa: E402
from twitter_stream_ml_amd.sources.synthetic import SynthConfig, generate_batch  # noqa: E402


def main():
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    h = hip()
    obj = [h.rccl_unique_id() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    comm = h.Comm(obj[0], rank, world, 0)
    F = 1 << 20
    cfg = LRDeviceConfig(num_text_features=F, max_rows=8192, max_units=8192 * 300)
    eng = DeviceLinearRegression(cfg, device=0, comm=comm)
    synth = SynthConfig.profile("twitter", seed=21)
    ok = True
    ref = DeviceLinearRegression(cfg, device=0) if rank == 0 else None
    for t in range(3):
        full = generate_batch(synth, t * 4000, 4000, batch_time_ms=1_700_000_000_000)
        shard = full.shard(rank, world)
        res = eng.train_batch(shard)
        if rank == 0:
            r1 = ref.train_batch(full)
            w_dp, w_1 = eng.get_weights(), ref.get_weights()
            err = np.abs(w_dp - w_1).max() / max(np.abs(w_1).max(), 1e-12)
            print(f"batch {t}: dp kept={res['n_kept_global']} 1gpu kept={r1['n_kept']} "
                  f"iters {res['iterations']}/{r1['iterations']} rel_err={err:.2e} "
                  f"stats_n {res['stats'][0]}/{r1['stats'][0]}", flush=True)
            ok &= res["n_kept_global"] == r1["n_kept"] and err < 1e-4
    dist.barrier()
    if rank == 0:
        print("DP_PROBE", "PASS" if ok else "FAIL", flush=True)
    dist.destroy_process_group()
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
