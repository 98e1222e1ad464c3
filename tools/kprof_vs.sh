#!/bin/bash
# Kernel-trace stats + bench lines of several builds on one box:
# VARIANTS="V0 V1" tools/kprof_vs.sh <kernel regex> <bench reps> [bench args]   (ab/<V>.so each)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
SO=twitter_stream_ml_amd/_twtml_hip.cpython-310-x86_64-linux-gnu.so
re=$1; reps=$2; shift 2
cp $SO ab/orig.so
for v in $VARIANTS; do
  cp ab/$v.so $SO
  rm -rf gpurun_out/kpv_$v
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kpv_$v -o run -- \
    python bench.py --steps 10 --warmup 3 "$@" > gpurun_out/kpv_$v.log 2>&1 || { cp ab/orig.so $SO; echo "FAIL $v"; exit 1; }
  python tools/kstats.py gpurun_out/kpv_$v/run_kernel_stats.csv > gpurun_out/kpv_${v}_stats.txt
  echo "== $v"; grep -E "$re" gpurun_out/kpv_${v}_stats.txt
done
for r in $(seq $reps); do
  for v in $VARIANTS; do
    cp ab/$v.so $SO
    timeout -k 10 200 python bench.py "$@" > gpurun_out/vs_$v.log 2>&1 || { cp ab/orig.so $SO; echo "FAIL $v"; tail -3 gpurun_out/vs_$v.log; exit 1; }
    grep metric gpurun_out/vs_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', round(d['value']/1e6,1), 'M/s', d['ms_per_step'], 'ms train', round(d.get('train_ms_mean',0),3), 'prep', round(d.get('prep_ms_mean',0),3))"
  done
done
cp ab/orig.so $SO
