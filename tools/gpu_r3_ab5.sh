#!/bin/bash
# Pipelined iteration kernel: SGD tests on the tree (P1), then P0/P1 kernel tables (serial) and bench lines.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q tests/test_gpu_exact.py tests/test_gpu_tiered.py tests/test_gpu_lr_engine.py --timeout 200 --timeout-method thread > gpurun_out/sgd_tests.log 2>&1 || { tail -30 gpurun_out/sgd_tests.log; exit 1; }
tail -1 gpurun_out/sgd_tests.log
TWTML_OVERLAP=0 VARIANTS="P0 P1" bash tools/kprof_vs.sh "iter_hyb|far_grad|update" 0 || exit 1
VARIANTS="P0 P1" bash tools/kprof_vs.sh "iter_hyb" 2 --steps 20 --warmup 5
