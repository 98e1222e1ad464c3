cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; grep -E "^E|FAILED" gpurun_out/pytest_gpu.log | head -10
[ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 2 > gpurun_out/bench_lr.log 2>&1 || exit $?
tail -1 gpurun_out/bench_lr.log | cut -c1-200; python -c "import json; d=json.loads(open('gpurun_out/bench_lr.log').read().strip().splitlines()[-1]); print('ms', d['ms_per_step'], 'train', d['train_ms_mean'], 'prep', d['prep_ms_mean'], 'p50', d['p50_microbatch_latency_ms'])"
rm -rf gpurun_out/prof_lr
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_lr -o run -- python bench.py --steps 5 --warmup 1 > gpurun_out/prof_lr.log 2>&1 || exit $?
python tools/kstats.py gpurun_out/prof_lr/run_kernel_stats.csv 12
