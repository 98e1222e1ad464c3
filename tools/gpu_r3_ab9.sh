#!/bin/bash
# Specials-only row normalisation (UTF-8 batches): LR tests on the tree (S16), then S0/S8/S16 kernel tables and bench lines.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q tests/test_gpu_lr_engine.py --timeout 200 --timeout-method thread > gpurun_out/lr_tests.log 2>&1 || { tail -30 gpurun_out/lr_tests.log; exit 1; }
tail -1 gpurun_out/lr_tests.log
cp ab/S8.so twitter_stream_ml_amd/_twtml_hip.cpython-310-x86_64-linux-gnu.so
timeout -k 10 400 python -u -m pytest -x -q tests/test_gpu_lr_engine.py -k "special or utf8" --timeout 200 --timeout-method thread > gpurun_out/lr_tests8.log 2>&1 || { cp ab/S16.so twitter_stream_ml_amd/_twtml_hip.cpython-310-x86_64-linux-gnu.so; tail -30 gpurun_out/lr_tests8.log; exit 1; }
tail -1 gpurun_out/lr_tests8.log
cp ab/S16.so twitter_stream_ml_amd/_twtml_hip.cpython-310-x86_64-linux-gnu.so
VARIANTS="S0 S8 S16" bash tools/kprof_vs.sh "normalize" 2 --steps 20 --warmup 5
