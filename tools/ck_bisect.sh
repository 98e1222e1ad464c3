#!/bin/bash
# Which earlier GPU test module makes the checkpoint p99 gate fail when it runs after it?
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/bis
for pre in test_gpu_app_sizing test_gpu_apps test_gpu_bench; do
  timeout -k 10 400 python -u -m pytest tests/$pre.py tests/test_gpu_checkpoint.py -m gpu -q -s --timeout 300 \
    --timeout-method thread -p no:cacheprovider -k "not snapshot" > gpurun_out/bis/$pre.log 2>&1
  echo "$pre rc=$? $(grep -h "p99_ms_no_ckpt" gpurun_out/bis/$pre.log | python3 -c "
import sys,ast
for l in sys.stdin:
    for x in l.split('{')[1:]:
        d=ast.literal_eval('{'+x.split('}')[0]+'}'); print('%.2f/%.2f=%.3f p50 %.2f/%.2f' % (d['p99_ms_no_ckpt'], d['p99_ms_ckpt1'], d['p99_ms_ckpt1']/d['p99_ms_no_ckpt'], d['p50_ms_no_ckpt'], d['p50_ms_ckpt1']), end='  ')
")"
done
