#!/bin/bash
# Checkpoint p99 gate vs the snapshot's D2H chunk size (TWTML_SNAP_CHUNK_KB), interleaved.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/ckc
for r in $(seq "${1:-2}"); do
  for kb in 256; do for du in 0.05 0.03 0.02; do
    TWTML_SNAP_DUTY=$du TWTML_SNAP_CHUNK_KB=$kb timeout -k 10 250 python -u -m pytest tests/test_gpu_checkpoint.py -k p99 -x -q -s \
      --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/ckc/k${kb}_d${du}_$r.log 2>&1
    echo "chunk ${kb}KB duty $du rep $r rc=$? $(grep -h "p99_ms_no_ckpt" gpurun_out/ckc/k${kb}_d${du}_$r.log | python3 -c "
import sys,ast
for l in sys.stdin:
    for x in l.split('{')[1:]:
        d=ast.literal_eval('{'+x.split('}')[0]+'}'); print('%.2f/%.2f=%.3f w%d' % (d['p99_ms_no_ckpt'], d['p99_ms_ckpt1'], d['p99_ms_ckpt1']/d['p99_ms_no_ckpt'], d['written']), end='  ')
")"
  done; done
done
