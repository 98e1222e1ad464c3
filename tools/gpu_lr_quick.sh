#!/bin/bash
# LR iteration work loop on the GPU box: GPU tests, bench, kernel profile.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu ${TESTS:-tests} > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -${TAIL:-6} gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 200 python bench.py --steps 10 --warmup 2 ${BENCH_ARGS} > gpurun_out/bench_lr.log 2>&1 || exit 3
tail -1 gpurun_out/bench_lr.log | python -c "import json,sys;d=json.loads(sys.stdin.read());print('bench', d['value']/1e6, 'M/s', d['ms_per_step'], 'ms', 'prep', round(d['prep_ms_mean'],3), 'train', round(d['train_ms_mean'],3), 'iters', d['gd_iterations_mean'])"
if [ -n "$PROFILE" ]; then
  rm -rf gpurun_out/prof_lr
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_lr -o run -- python bench.py --steps 5 --warmup 1 ${BENCH_ARGS} > gpurun_out/prof_lr.log 2>&1 || exit 4
  python tools/kstats.py gpurun_out/prof_lr/run_kernel_stats.csv > gpurun_out/prof_lr_stats.txt; head -14 gpurun_out/prof_lr_stats.txt
fi
exit 0
