#!/bin/bash
# Benches (wide default, toy) + the driver on the measured path + wide kernel stats.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
set -o pipefail
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --json-out gpurun_out/b_wide.json > gpurun_out/b_wide.log 2>&1 || { tail -20 gpurun_out/b_wide.log; exit 1; }
cat gpurun_out/b_wide.json
timeout -k 10 300 python bench.py --profile bench --steps 20 --warmup 5 --json-out gpurun_out/b_toy.json > gpurun_out/b_toy.log 2>&1 || { tail -20 gpurun_out/b_toy.log; exit 1; }
cat gpurun_out/b_toy.json
bash tools/gpu_r3_app.sh || exit 1
TOP=24 bash tools/kprof.sh wide --steps 10 --warmup 3
