#!/bin/bash
# Far backward in the iteration kernel: exactness / DP / tiered tests, then the wide bench + kernel table.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TEST_TIMEOUT=900 bash tools/gpu_t.sh tests/test_gpu_exact.py tests/test_gpu_tiered.py tests/test_gpu_dp_loopback.py tests/test_gpu_lr_engine.py tests/test_gpu_dp_procs.py tests/test_gpu_app_sizing.py || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --json-out gpurun_out/b_wide.json > gpurun_out/b_wide.log 2>&1 || { tail -20 gpurun_out/b_wide.log; exit 1; }
cat gpurun_out/b_wide.json; echo
TOP=12 bash tools/kprof.sh wide --steps 20 --warmup 5
