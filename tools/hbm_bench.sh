#!/bin/bash
# Config 5 with HBM-sized micro-batches vs the 1M-tweet default (same box).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
for b in ${BATCHES:-hbm 1000000}; do
  timeout -k 10 500 python bench.py --profile wide --features 100000000 --hash murmur3 --batch $b --pool ${POOL:-3} \
    --steps ${STEPS:-10} --warmup ${WARM:-5} > gpurun_out/hbm_$b.log 2>&1 || { echo "FAIL $b"; tail -5 gpurun_out/hbm_$b.log; exit 1; }
  grep metric gpurun_out/hbm_$b.log > gpurun_out/hbm_$b.json
  python -c "import json; d=json.load(open('gpurun_out/hbm_$b.json')); print('$b', d['config']['global_batch'], round(d['value']/1e6,1), 'M/s', d['ms_per_step'], 'ms it', d.get('gd_iterations_mean'), 'prep', round(d.get('prep_ms_mean') or 0,2), 'train', round(d.get('train_ms_mean') or 0,2), d['config'].get('batch_sizing'))"
done
