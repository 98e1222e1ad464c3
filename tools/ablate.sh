#!/bin/bash
# SGD iteration ablation at a fixed iteration count (tol 0: no early stop):
# 0 full, 1 no gradient scatter, 2 no gather/scatter.  Extra args go to bench.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for a in ${ABL:-0 1 2}; do
  timeout -k 10 200 python bench.py --steps 5 --warmup 1 --ablate $a --iters 20 --tol 0 "$@" > gpurun_out/abl$a.log 2>&1 || exit 3
  python -c "import json;d=json.loads(open('gpurun_out/abl$a.log').read().strip().splitlines()[-1]);print('ablate $a train_ms', round(d['train_ms_mean'],3), 'iters', d['gd_iterations_mean'], 'per-iter us', round(1e3*d['train_ms_mean']/d['gd_iterations_mean'],1))"
done
