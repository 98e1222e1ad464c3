#!/bin/bash
# Case tables in LDS for the row normalisation: LR tests on the tree (N1), then N0/N1 kernel tables and bench lines.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q tests/test_gpu_lr_engine.py --timeout 200 --timeout-method thread > gpurun_out/lr_tests.log 2>&1 || { tail -30 gpurun_out/lr_tests.log; exit 1; }
tail -1 gpurun_out/lr_tests.log
VARIANTS="N0 N1" bash tools/kprof_vs.sh "normalize|decode" 2 --steps 20 --warmup 5 || exit 1
VARIANTS="N0 N1" bash tools/kprof_vs.sh "normalize|km_features" 0 --model kmeans --steps 10 --warmup 3
