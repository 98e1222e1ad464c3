#!/bin/bash
# Same-box A/B of the main tree against a variant tree (a copy of csrc/, the
# package and bench.py with its own in-tree build, e.g. abvar/): interleaved
#   tools/ab_tree.sh <variant dir> <reps> [bench args]
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/${TAG:-abtree}
mkdir -p "$OUT"
var=$1; reps=$2; shift 2
for r in $(seq "$reps"); do
  for which in main var; do
    if [[ $which == main ]]; then dir=.; else dir=$var; fi
    (cd "$dir" && timeout -k 10 200 python -u bench.py "$@" --json-out "$GRAFT_REPO_ROOT/$OUT/${which}_$r.json") \
      > "$OUT/${which}_$r.log" 2>&1 || { echo "FAIL $which"; tail -5 "$OUT/${which}_$r.log"; exit 1; }
    python - "$OUT/${which}_$r.json" "$which" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print(f"{sys.argv[2]:>5}: {d['value']/1e6:7.1f} M/s  {d['ms_per_step']:.3f} ms  p50 {d['p50_microbatch_latency_ms']:.2f}  "
      f"train {d.get('train_ms_mean', 0):.3f}  prep {d.get('prep_ms_mean', 0):.3f}", flush=True)
PY
  done
done
