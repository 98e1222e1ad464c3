#!/bin/bash
# Iteration loop on the GPU box: GPU tests, bench, kernel-trace profile.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py ${BENCH_ARGS:---steps 10 --warmup 2} > gpurun_out/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -2 gpurun_out/bench.log
[ $rc -eq 0 ] || exit $rc
if [ -n "$PROFILE" ]; then
  rm -rf gpurun_out/prof
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python bench.py --steps 5 --warmup 1 > gpurun_out/prof.log 2>&1; rc=$?; echo "prof rc=$rc"
  python tools/kstats.py gpurun_out/prof/run_kernel_stats.csv
fi
exit $rc
