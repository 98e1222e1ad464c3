#!/bin/bash
# Fused far update: exactness / tiered / DP tests, then wide bench fused vs TWTML_FAR_FUSED=0, kernel table.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TEST_TIMEOUT=900 bash tools/gpu_t.sh tests/test_gpu_exact.py tests/test_gpu_tiered.py tests/test_gpu_dp_loopback.py tests/test_gpu_lr_engine.py tests/test_gpu_dp_procs.py || exit 1
for v in 1 0 1 0; do
  TWTML_FAR_FUSED=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --json-out gpurun_out/b_wide_f$v.json > gpurun_out/b_wide_f$v.log 2>&1 || { tail -20 gpurun_out/b_wide_f$v.log; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/b_wide_f$v.json'));print('fused=$v', round(d['value']/1e6,1), 'M/s', d['ms_per_step'], 'ms train', round(d['train_ms_mean'],3), 'iters', d['gd_iterations_mean'])"
done
TOP=10 bash tools/kprof.sh wide --steps 20 --warmup 5
