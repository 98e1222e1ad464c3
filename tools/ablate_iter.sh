#!/bin/bash
# GD iteration kernel ablations with per-workgroup timing (TWTML_ITER_TIMING):
#   tools/ablate_iter.sh "0 8 7"  -> gpurun_out/$TAG/abl<a>.log
# (ablate 8: no far forward in the iteration kernel; 7: no chunks -- fixed cost;
# results are numerically meaningless, only the timings count)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/${TAG:-abl}
mkdir -p "$OUT"
for a in ${1:-0 8 7}; do
  TWTML_ITER_TIMING=1 timeout -k 10 200 python -u bench.py --ablate "$a" --steps 8 --warmup 3 \
    --json-out "$OUT/abl$a.json" > "$OUT/abl$a.log" 2>&1 || { tail -5 "$OUT/abl$a.log"; exit 1; }
  echo "== ablate $a"
  grep -E "kernel (iteration|far)" "$OUT/abl$a.log" | tail -2
  grep "iter timing" "$OUT/abl$a.log" | tail -2
done
