#!/bin/bash
# Quick GPU check: selected tests (-k $1), then bench lines given as
# "name:arg,arg,..." words in $BENCHES (default: toy + wide).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
if [ -n "$1" ]; then bash tools/gpu_tests.sh -k "$1" || exit 1; fi
run() { local name=$1; shift; timeout -k 10 300 python bench.py "$@" > gpurun_out/b_$name.log 2>&1 || { echo "FAIL $name"; tail -5 gpurun_out/b_$name.log; exit 1; }; grep metric gpurun_out/b_$name.log > gpurun_out/b_$name.json; python -c "import json;d=json.load(open('gpurun_out/b_$name.json'));print('$name', round(d['value']/1e6,1), 'M/s', d['ms_per_step'], 'ms it', d.get('gd_iterations_mean'), 'prep', round(d.get('prep_ms_mean') or 0,3), 'train', round(d.get('train_ms_mean') or 0,3), 'stage', d.get('host_stage_ms_p50'))"; }
for b in ${BENCHES:-toy: wide:--profile,wide,--steps,10,--pool,3}; do
  name=${b%%:*}; args=${b#*:}; run $name ${args//,/ } || exit 1
done
