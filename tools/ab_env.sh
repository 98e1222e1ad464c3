#!/bin/bash
# A/B an environment toggle on one box: tools/ab_env.sh VAR "valA valB" <reps> [bench args]
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
var=$1; vals=$2; reps=$3; shift 3
for r in $(seq $reps); do
  for v in $vals; do
    env $var=$v timeout -k 10 200 python bench.py "$@" > gpurun_out/abe_$v.log 2>&1 || { echo "FAIL $v"; tail -3 gpurun_out/abe_$v.log; exit 1; }
    grep metric gpurun_out/abe_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$var=$v', round(d['value']/1e6,1), 'M/s', d['ms_per_step'], 'ms train', round(d.get('train_ms_mean',0),3), 'prep', round(d.get('prep_ms_mean',0),3))"
  done
done
