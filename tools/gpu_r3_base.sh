#!/bin/bash
# Round-3 baseline: fresh-pool benches (wide default, toy), wide layout occupancy, kernel stats.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
set -o pipefail
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --json-out gpurun_out/b_wide.json > gpurun_out/b_wide.log 2>&1 || { tail -20 gpurun_out/b_wide.log; exit 1; }
cat gpurun_out/b_wide.json
timeout -k 10 300 python bench.py --profile bench --steps 20 --warmup 5 --json-out gpurun_out/b_toy.json > gpurun_out/b_toy.log 2>&1 || { tail -20 gpurun_out/b_toy.log; exit 1; }
cat gpurun_out/b_toy.json
timeout -k 10 200 python tools/diag/wide_layout.py wide 1000000 > gpurun_out/wide_layout.txt 2>&1 || { tail -20 gpurun_out/wide_layout.txt; exit 1; }
cat gpurun_out/wide_layout.txt
TOP=24 bash tools/kprof.sh wide --steps 10 --warmup 3
