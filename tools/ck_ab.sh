#!/bin/bash
# Same-box A/B of the checkpoint p99 gate: main tree vs a variant tree (abvar/), interleaved.
#   tools/ck_ab.sh <reps>
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/ckab
for r in $(seq "${1:-2}"); do
  for which in main var; do
    d=.; [[ $which == var ]] && d=abvar
    (cd $d && timeout -k 10 250 python -u -m pytest tests/test_gpu_checkpoint.py -k p99 -x -q -s --timeout 240 \
      --timeout-method thread -p no:cacheprovider) > gpurun_out/ckab/${which}_$r.log 2>&1
    echo "$which $r rc=$? $(grep -h "p99_ms_no_ckpt" gpurun_out/ckab/${which}_$r.log | tr '\n' ' ' | cut -c1-600)"
  done
done
