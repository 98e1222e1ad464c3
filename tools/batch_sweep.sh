#!/bin/bash
# Per-iteration SGD cost vs batch size (MALL residency of the slot stream).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for B in 250000 500000 1000000 2000000; do for dd in 0 1; do
  timeout -k 10 300 python bench.py --batch $B --steps 6 --warmup 1 --dedup $dd > gpurun_out/bs_${B}_$dd.log 2>&1 || exit 3
  python -c "import json;d=json.loads(open('gpurun_out/bs_${B}_$dd.log').read().strip().splitlines()[-1]);it=d['gd_iterations_mean'];print('batch $B dedup $dd ms/step', d['ms_per_step'], 'train_ms', round(d['train_ms_mean'],3), 'us/iter', round(1e3*d['train_ms_mean']/it,1), 'prep', round(d['prep_ms_mean'],3))"
done; done
