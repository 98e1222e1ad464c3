#!/bin/bash
# Quick GPU pass: GPU tests (unless SKIP_TESTS), LR bench, kernel-trace
# profile of the LR bench (top kernels -> gpurun_out/prof_lr_stats.txt).
# Extra args go to both bench runs.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 200 python bench.py --steps 20 --warmup 3 "$@" > gpurun_out/bench.log 2>&1 || exit $?
grep metric gpurun_out/bench.log | cut -c1-200
rm -rf gpurun_out/prof_lr
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_lr -o run -- \
  python bench.py --steps 5 --warmup 1 "$@" > gpurun_out/prof_lr.log 2>&1 || exit $?
python tools/kstats.py gpurun_out/prof_lr/run_kernel_stats.csv > gpurun_out/prof_lr_stats.txt
head -16 gpurun_out/prof_lr_stats.txt
