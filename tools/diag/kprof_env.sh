#!/bin/bash
# Kernel-trace rows matching a regex for values of an environment toggle on one box:
# tools/diag/kprof_env.sh VAR "a b c" <kernel regex> [bench args]
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
var=$1; vals=$2; re=$3; shift 3
for v in $vals; do
  rm -rf gpurun_out/kpe_$v
  env $var=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kpe_$v -o run -- \
    python bench.py "$@" > gpurun_out/kpe_$v.log 2>&1 || { echo "FAIL $v"; exit 1; }
  python tools/kstats.py gpurun_out/kpe_$v/run_kernel_stats.csv > gpurun_out/kpe_${v}_stats.txt
  echo "== $var=$v"; grep -E "$re" gpurun_out/kpe_${v}_stats.txt
done
