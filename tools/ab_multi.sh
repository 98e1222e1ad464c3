#!/bin/bash
# Same-box A/B of environment variants, interleaved over reps:
#   tools/ab_multi.sh <reps> "name1:VAR=a,VAR2=b" "name2:" ... [-- bench args]
# One line per run: name, tweets/s, ms/step, p50, train/prep means.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/${TAG:-ab}
mkdir -p "$OUT"
reps=$1; shift
variants=()
while [[ $# -gt 0 && "$1" != "--" ]]; do variants+=("$1"); shift; done
[[ "$1" == "--" ]] && shift
for r in $(seq "$reps"); do
  for v in "${variants[@]}"; do
    name=${v%%:*}; envs=${v#*:}
    envargs=()
    IFS=',' read -ra kv <<< "$envs"
    for e in "${kv[@]}"; do [[ -n "$e" ]] && envargs+=("$e"); done
    log="$OUT/${name}_$r.log"
    env "${envargs[@]}" timeout -k 10 200 python -u bench.py "$@" --json-out "$OUT/${name}_$r.json" > "$log" 2>&1
    rc=$?
    if [[ $rc != 0 ]]; then echo "FAIL $name rc=$rc"; tail -5 "$log"; exit $rc; fi
    python - "$OUT/${name}_$r.json" "$name" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print(f"{sys.argv[2]:>14}: {d['value']/1e6:7.1f} M/s  {d['ms_per_step']:.3f} ms  p50 {d['p50_microbatch_latency_ms']:.2f}  "
      f"train {d.get('train_ms_mean', 0):.3f}  prep {d.get('prep_ms_mean', 0):.3f}", flush=True)
PY
  done
done
