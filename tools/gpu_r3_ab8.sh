#!/bin/bash
# Remap placement by prefix sums: LR tests on the tree (R1), then R0/R1 kernel tables and bench lines.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q tests/test_gpu_lr_engine.py tests/test_gpu_tiered.py tests/test_gpu_exact.py --timeout 200 --timeout-method thread > gpurun_out/lr_tests.log 2>&1 || { tail -30 gpurun_out/lr_tests.log; exit 1; }
tail -1 gpurun_out/lr_tests.log
VARIANTS="R0 R1" bash tools/kprof_vs.sh "remap|far_csc" 2 --steps 20 --warmup 5
