#!/bin/bash
# Wide LR: default bench (no profiler), then kernel tables overlapped and with TWTML_OVERLAP=0.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --json-out gpurun_out/b_wide.json > gpurun_out/b_wide.log 2>&1 || { tail -20 gpurun_out/b_wide.log; exit 1; }
cat gpurun_out/b_wide.json; echo
TOP=12 bash tools/kprof.sh wide --steps 20 --warmup 5 || exit 1
TWTML_OVERLAP=0 TOP=12 bash tools/kprof.sh wide_serial --steps 20 --warmup 5
