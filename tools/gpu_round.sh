#!/bin/bash
# One GPU-box pass: all GPU tests, then the bench configs (LR 1M, k-means
# k=1024, wide 100M murmur3) and a kernel-trace profile of the k-means bench.
# Every GPU step has its own time limit; a crash/timeout ends the script.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -${TAIL:-3} "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  return 0
}
[ -z "$SKIP_TESTS" ] && TAIL=12 step pytest_gpu 500 python -m pytest tests -q -m gpu
step bench_lr 300 python bench.py --steps 20 --warmup 3
step bench_km 300 python bench.py --model kmeans --steps 20 --warmup 3
step bench_wide 400 python bench.py --features 100000000 --hash murmur3 --steps 20 --warmup 3
if [ -n "$PROFILE" ]; then
  rm -rf gpurun_out/prof_lr
  step prof_lr 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d gpurun_out/prof_lr -o run -- python bench.py --steps 5 --warmup 1
  python tools/kstats.py gpurun_out/prof_lr/run_kernel_stats.csv > gpurun_out/prof_lr_stats.txt; cat gpurun_out/prof_lr_stats.txt
  rm -rf gpurun_out/prof_km
  step prof_km 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_km -o run -- python bench.py --model kmeans --steps 5 --warmup 1
  python tools/kstats.py gpurun_out/prof_km/run_kernel_stats.csv > gpurun_out/prof_km_stats.txt; cat gpurun_out/prof_km_stats.txt
fi
exit 0
