#!/bin/bash
# Round-2 baseline: current engine on the toy (bench) and realistic (wide)
# profiles, plus a kernel-trace of the wide run.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 200 python bench.py --steps 10 --warmup 2 > gpurun_out/b_bench.log 2>&1 || exit $?
grep metric gpurun_out/b_bench.log | cut -c1-300
timeout -k 10 300 python bench.py --profile wide --steps 4 --warmup 1 --pool 2 > gpurun_out/b_wide.log 2>&1 || exit $?
grep metric gpurun_out/b_wide.log | cut -c1-600
timeout -k 10 300 python bench.py --profile wide --features 100000000 --hash murmur3 --steps 4 --warmup 1 --pool 2 > gpurun_out/b_wide100m.log 2>&1 || exit $?
grep metric gpurun_out/b_wide100m.log | cut -c1-600
rm -rf gpurun_out/prof_wide
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_wide -o run -- \
  python bench.py --profile wide --steps 3 --warmup 1 --pool 2 > gpurun_out/prof_wide.log 2>&1 || exit $?
python tools/kstats.py gpurun_out/prof_wide/run_kernel_stats.csv > gpurun_out/prof_wide_stats.txt
head -20 gpurun_out/prof_wide_stats.txt
