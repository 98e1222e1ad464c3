#!/bin/bash
# Decode next dword by DPP wave shift: LR + k-means tests with ab/D1.so, then D0/D1 kernel tables and bench lines.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
SO=twitter_stream_ml_amd/_twtml_hip.cpython-310-x86_64-linux-gnu.so
cp $SO ab/orig.so; cp ab/D1.so $SO
timeout -k 10 500 python -u -m pytest -x -q tests/test_gpu_lr_engine.py tests/test_gpu_kmeans.py --timeout 200 --timeout-method thread > gpurun_out/lr_tests.log 2>&1 || { cp ab/orig.so $SO; tail -30 gpurun_out/lr_tests.log; exit 1; }
cp ab/orig.so $SO
tail -1 gpurun_out/lr_tests.log
VARIANTS="D0 D1" bash tools/kprof_vs.sh "decode" 2 --steps 20 --warmup 5
