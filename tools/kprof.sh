#!/bin/bash
# Kernel-trace stats of one bench configuration: tools/kprof.sh <name> [bench args]
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
name=$1; shift
rm -rf gpurun_out/kp_$name
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kp_$name -o run -- \
  python bench.py "$@" > gpurun_out/kp_$name.log 2>&1 || exit $?
python tools/kstats.py gpurun_out/kp_$name/run_kernel_stats.csv > gpurun_out/kp_${name}_stats.txt
grep metric gpurun_out/kp_$name.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$name', round(d['value']/1e6,1), 'M/s', d['ms_per_step'], 'ms')"
head -${TOP:-14} gpurun_out/kp_${name}_stats.txt
