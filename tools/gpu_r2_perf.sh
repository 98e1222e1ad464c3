#!/bin/bash
# Round-2 perf: device pipeline (toy / wide / wide murmur3 1e8), e2e ingest
# (utf16 / wire), kernel trace of the wide run.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
run() { local name=$1; shift; timeout -k 10 300 python bench.py "$@" > gpurun_out/b_$name.log 2>&1 || { echo "FAIL $name"; tail -5 gpurun_out/b_$name.log; exit 1; }; grep metric gpurun_out/b_$name.log > gpurun_out/b_$name.json; python -c "import json;d=json.load(open('gpurun_out/b_$name.json'));print('$name', d['value']/1e6, 'M/s', d['ms_per_step'], 'ms', d.get('gd_iterations_mean'), d.get('prep_ms_mean'), d.get('train_ms_mean'), d.get('host_stage_ms_p50'), d.get('active_features'), d.get('lds_tier_features'))"; }
run bench --steps 20 --warmup 3
run wide --profile wide --steps 10 --warmup 3 --pool 3
run wide100m --profile wide --features 100000000 --hash murmur3 --steps 10 --warmup 3 --pool 3
run e2e_utf16 --e2e --steps 20 --warmup 3
run e2e_wire --e2e --ingest wire --steps 10 --warmup 3
run e2e_wide --e2e --profile wide --steps 10 --warmup 3 --pool 3
rm -rf gpurun_out/prof_wide2
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_wide2 -o run -- \
  python bench.py --profile wide --steps 5 --warmup 2 --pool 3 > gpurun_out/prof_wide2.log 2>&1 || exit $?
python tools/kstats.py gpurun_out/prof_wide2/run_kernel_stats.csv > gpurun_out/prof_wide2_stats.txt
head -24 gpurun_out/prof_wide2_stats.txt
