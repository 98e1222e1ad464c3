#!/bin/bash
# Round-3 bench lines: every table row of README "Performance" (JSON -> gpurun_out/final_*.json).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
run() {  # name, bench args...
  local n=$1; shift
  timeout -k 10 400 python bench.py "$@" --json-out gpurun_out/final_$n.json > gpurun_out/final_$n.log 2>&1 || { tail -20 gpurun_out/final_$n.log; return 1; }
  python -c "import json;d=json.load(open('gpurun_out/final_$n.json'));print('$n', round(d['value']/1e6,1), 'M/s', d['ms_per_step'], 'ms', 'iters', d.get('gd_iterations_mean'))"
}
run wide --steps 20 --warmup 5 || exit 1
run toy --profile bench --steps 20 --warmup 5 || exit 1
run kmeans --model kmeans --steps 20 --warmup 5 || exit 1
run kmeans_k3 --model kmeans --k 3 --text-dims 0 --steps 20 --warmup 5 || exit 1
run wide100m --features 100000000 --hash murmur3 --steps 20 --warmup 5 || exit 1
run prepacked --prepacked --steps 20 --warmup 5 || exit 1
bash tools/gpu_r3_app.sh
