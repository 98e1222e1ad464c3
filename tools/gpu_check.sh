#!/bin/bash
# First-pass GPU validation: smoke, GPU tests, small bench.  Stops at the first
# crash/timeout (exit codes >= 124 or signals); test failures (rc=1) continue.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
timeout -k 10 180 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log
ok $rc || exit $rc
timeout -k 10 400 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
ok $rc || exit $rc
timeout -k 10 300 python bench.py --batch ${BENCH_BATCH:-262144} --steps 10 --warmup 2 > gpurun_out/bench_small.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -5 gpurun_out/bench_small.log
exit $rc
