#!/bin/bash
# Raw-slot depth sweep of the headline bench (tweets/s vs p50 latency):
#   tools/slot_sweep.sh [depths] [reps] [extra bench args]
# Each run: TWTML_RAW_SLOTS=<d> python bench.py ... -> gpurun_out/$TAG/slots<d>_<rep>.json
# (runs interleaved by rep so box drift spreads over all depths)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
TAG=${TAG:-sweep}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
DEPTHS=${1:-"4 5 6 8"}
REPS=${2:-2}
shift 2 2>/dev/null
for rep in $(seq 1 "$REPS"); do
  for d in $DEPTHS; do
    name=slots${d}_${rep}
    TWTML_RAW_SLOTS=$d timeout -k 10 200 python -u bench.py "$@" --json-out "$OUT/$name.json" > "$OUT/$name.log" 2>&1
    rc=$?
    if [[ $rc != 0 ]]; then tail -20 "$OUT/$name.log"; exit $rc; fi
    python - "$OUT/$name.json" "$d" <<'PY'
import json, sys
r = json.load(open(sys.argv[1]))
print(f"slots {sys.argv[2]}: {r['value']/1e6:.1f} M tweets/s  {r['ms_per_step']:.3f} ms/step  p50 {r['p50_microbatch_latency_ms']:.2f} ms")
PY
  done
done
