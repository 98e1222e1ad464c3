#!/bin/bash
# LR engine tests on the working tree, then A/B kernel deltas and default-config bench lines (ab/A.so vs ab/B.so).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q tests/test_gpu_lr_engine.py --timeout 200 --timeout-method thread > gpurun_out/lr_tests.log 2>&1 || { tail -30 gpurun_out/lr_tests.log; exit 1; }
tail -1 gpurun_out/lr_tests.log
bash tools/kprof_ab.sh "decode|normalize|bounds|far_csc" --steps 10 --warmup 3 || exit 1
bash tools/ab.sh 2 --steps 20 --warmup 5
