#!/bin/bash
# Kernel-trace stats of builds (ab/A.so, ab/B.so, ...; AB_VARIANTS="A C" picks some) on one box:
# tools/kprof_ab.sh <kernel regex> [bench args]
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
SO=twitter_stream_ml_amd/_twtml_hip.cpython-310-x86_64-linux-gnu.so
re=$1; shift
cp $SO ab/orig.so
for v in ${AB_VARIANTS:-A B}; do
  cp ab/$v.so $SO
  rm -rf gpurun_out/kpab_$v
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kpab_$v -o run -- \
    python bench.py "$@" > gpurun_out/kpab_$v.log 2>&1 || { cp ab/orig.so $SO; echo "FAIL $v"; exit 1; }
  python tools/kstats.py gpurun_out/kpab_$v/run_kernel_stats.csv > gpurun_out/kpab_${v}_stats.txt
  echo "== $v"; grep -E "$re" gpurun_out/kpab_${v}_stats.txt
done
cp ab/orig.so $SO
