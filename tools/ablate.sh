#!/bin/bash
# SGD iteration ablation (0: full, 1: no gradient scatter, 2: no gather/scatter)
# with and without per-row bigram merging.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for dd in 0 1; do for a in 0 1 2; do
  timeout -k 10 200 python bench.py --steps 5 --warmup 1 --ablate $a --iters 20 --dedup $dd > gpurun_out/abl$dd$a.log 2>&1 || exit 3
  python -c "import json;d=json.loads(open('gpurun_out/abl$dd$a.log').read().strip().splitlines()[-1]);print('dedup $dd ablate $a train_ms', round(d['train_ms_mean'],3), 'iters', d['gd_iterations_mean'], 'prep', round(d['prep_ms_mean'],3))"
done; done
