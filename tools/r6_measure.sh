#!/bin/bash
# Round-6 measurement session (one gpurun call): headline bench x2 (engine
# default raw slots), BASELINE config 1 on the box's CPU, the 8-rank DP
# rehearsal (gloo, one GPU), and the RCCL-footprint stand-in under forced DP.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/${TAG:-r6m}
mkdir -p "$OUT"
step() { echo "=== $1 ($(date +%T))"; }
for rep in 1 2; do
  step "bench default rep $rep"
  timeout -k 10 200 python -u bench.py --json-out "$OUT/bench_default_$rep.json" > "$OUT/bench_default_$rep.log" 2>&1 || exit $?
  tail -1 "$OUT/bench_default_$rep.log" | cut -c1-400
done
step "config 1: local[2] CPU"
timeout -k 10 400 python -u bench.py --master 'local[2]' --steps 20 --warmup 5 --json-out "$OUT/config1_local2.json" \
  > "$OUT/config1_local2.log" 2>&1 || exit $?
tail -1 "$OUT/config1_local2.log" | cut -c1-400
step "stand-in: forced DP, 32 workgroups"
TWTML_ITER_TIMING=1 TWTML_RCCL_STANDIN=32 timeout -k 10 200 python -u bench.py --force-dp --steps 8 --warmup 3 \
  --json-out "$OUT/standin32.json" > "$OUT/standin32.log" 2>&1 || exit $?
grep -c 'kernel rccl stand-in' "$OUT/standin32.log"
step "stand-in baseline: forced DP, no stand-in"
TWTML_ITER_TIMING=1 timeout -k 10 200 python -u bench.py --force-dp --steps 8 --warmup 3 \
  --json-out "$OUT/standin0.json" > "$OUT/standin0.log" 2>&1 || exit $?
step "dp rehearsal 8 ranks (gloo)"
DP_TIMEOUT=500 bash tools/dp_rehearsal.sh 8 || exit $?
cp gpurun_out/dp8.json gpurun_out/dp8.log "$OUT/" 2>/dev/null
echo "=== done"
