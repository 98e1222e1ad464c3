#!/bin/bash
# Sweep the LDS gradient replication factor of the SGD iteration kernel.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for R in 1 2 4 8; do
  TWTML_SGD_REP=$R timeout -k 10 200 python bench.py --steps 10 --warmup 2 > gpurun_out/rep$R.log 2>&1; rc=$?
  echo "REP=$R rc=$rc $(python -c "import json,sys; d=json.loads(open('gpurun_out/rep$R.log').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['train_ms_mean'], d['gd_iterations_mean'])")"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
