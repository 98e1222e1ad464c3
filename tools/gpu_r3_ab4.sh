#!/bin/bash
# Paired UTF-8 decode: LR engine tests on the tree (B), then A/B decode kernel times and bench lines.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q tests/test_gpu_lr_engine.py tests/test_gpu_exact.py --timeout 200 --timeout-method thread > gpurun_out/lr_tests.log 2>&1 || { tail -30 gpurun_out/lr_tests.log; exit 1; }
tail -1 gpurun_out/lr_tests.log
VARIANTS="A B" bash tools/kprof_vs.sh "decode|normalize|bounds" 2 --steps 20 --warmup 5
