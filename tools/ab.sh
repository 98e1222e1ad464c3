#!/bin/bash
# A/B(/C...) builds of the HIP extension on the same box, interleaved:
#   tools/ab.sh <reps> [bench args]     (variants: ab/A.so, ab/B.so, ... prepared beforehand;
#                                        AB_VARIANTS="A C" picks a subset; the in-tree .so is restored after)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
SO=twitter_stream_ml_amd/_twtml_hip.cpython-310-x86_64-linux-gnu.so
cp $SO ab/orig.so
reps=$1; shift
vars=${AB_VARIANTS:-$(cd ab && ls [A-Z].so | sed 's/\.so$//' | tr '\n' ' ')}
for r in $(seq $reps); do
  for v in $vars; do
    cp ab/$v.so $SO
    timeout -k 10 200 python bench.py "$@" > gpurun_out/ab_$v.log 2>&1 || { cp ab/orig.so $SO; echo "FAIL $v"; tail -3 gpurun_out/ab_$v.log; exit 1; }
    grep metric gpurun_out/ab_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', round(d['value']/1e6,1), 'M/s', d['ms_per_step'], 'ms train', round(d.get('train_ms_mean',0),3), 'prep', round(d.get('prep_ms_mean',0),3))"
  done
done
cp ab/orig.so $SO
