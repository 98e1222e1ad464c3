cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
bash tools/gpu_tests.sh -k "utf8 or special or featurize_matches" || exit 1
run() { local name=$1; shift; timeout -k 10 300 python bench.py "$@" > gpurun_out/b_$name.log 2>&1 || { echo "FAIL $name"; tail -5 gpurun_out/b_$name.log; exit 1; }; grep metric gpurun_out/b_$name.log > gpurun_out/b_$name.json; python -c "import json;d=json.load(open('gpurun_out/b_$name.json'));print('$name', d['value']/1e6, 'M/s', d['ms_per_step'], 'ms', d.get('gd_iterations_mean'), d.get('prep_ms_mean'), d.get('train_ms_mean'), d.get('host_stage_ms_p50'), d.get('active_features'))"; }
run e2e_utf8 --e2e --steps 20 --warmup 3
run e2e_utf8_wide --e2e --profile wide --steps 10 --warmup 3 --pool 3
run e2e_utf8_wide100m --e2e --profile wide --features 100000000 --hash murmur3 --steps 10 --warmup 3 --pool 3
