#!/bin/bash
# One parameterised GPU session runner (run through gpurun):
#   tools/gpu_run.sh <step> [<step> ...]
# Each step runs under its own timeout; the first failing step ends the run.
# Output goes to gpurun_out/<tag>/ (TAG env, default "run").
#
# steps:
#   tests[:<pytest -k expr>]   GPU suite (or a selection) in one pytest process
#   tfile:<path>               one GPU test module
#   bench:<name>[@<args>]      python bench.py <args> -> <name>.json
#   prof:<name>[@<args>]       rocprofv3 --kernel-trace --stats of bench.py <args>, kernel
#                              table (tools/kstats.py) and RCCL placement (tools/diag/rccl_order.py)
#   pmc:<c1,c2,..>[@<args>]    one counter pass over bench.py <args> (kernel trace + pmc only)
#   smoke                      __graft_entry__.smoke()
#   cmd:<shell>                an arbitrary command (own timeout: STEP_TIMEOUT, default 300 s)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
TAG=${TAG:-run}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
T=${STEP_TIMEOUT:-300}
for step in "$@"; do
  kind=${step%%:*}
  arg=""
  [[ "$step" == *:* ]] && arg=${step#*:}
  bargs=""
  if [[ "$kind" == bench || "$kind" == prof || "$kind" == pmc ]] && [[ "$arg" == *@* ]]; then
    bargs=${arg#*@}; arg=${arg%%@*}
  fi
  echo "=== $step ($(date +%T))"
  case "$kind" in
    tests)
      sel=()
      [[ -n "$arg" ]] && sel=(-k "$arg")
      timeout -k 10 ${TESTS_TIMEOUT:-1500} python -u -m pytest tests -m gpu -x -q --timeout 300 \
        --timeout-method thread "${sel[@]}" > "$OUT/pytest.log" 2>&1
      rc=$?; tail -5 "$OUT/pytest.log" ;;
    tfile)
      timeout -k 10 ${TESTS_TIMEOUT:-900} python -u -m pytest "$arg" -x -v --timeout 300 \
        --timeout-method thread > "$OUT/$(basename "$arg" .py).log" 2>&1
      rc=$?; tail -25 "$OUT/$(basename "$arg" .py).log" ;;
    bench)
      name=${arg:-bench}
      timeout -k 10 $T python -u bench.py $bargs --json-out "$OUT/$name.json" > "$OUT/$name.log" 2>&1
      rc=$?; tail -2 "$OUT/$name.log" ;;
    prof)
      name=${arg:-prof}
      rm -rf "$OUT/$name"
      timeout -k 10 $T rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$name" -o run -- \
        python -u bench.py $bargs > "$OUT/$name.log" 2>&1
      rc=$?
      if [[ $rc == 0 ]]; then
        python tools/kstats.py "$OUT/$name/run_kernel_stats.csv" 40 > "$OUT/${name}_kernels.txt" 2>&1
        python tools/diag/rccl_order.py "$OUT/$name/run_kernel_trace.csv" > "$OUT/${name}_rccl.txt" 2>&1
        head -40 "$OUT/${name}_kernels.txt"; cat "$OUT/${name}_rccl.txt" | head -40
        rm -f "$OUT/$name/run_kernel_trace.csv.gz"
      else tail -20 "$OUT/$name.log"; fi ;;
    pmc)
      name=pmc_$(echo "$arg" | tr ' ,' '__' | cut -c1-40)
      rm -rf "$OUT/$name"
      timeout -s KILL 120 rocprofv3 --kernel-trace --pmc ${arg//,/ } --output-format csv -d "$OUT/$name" -o run -- \
        python -u bench.py $bargs > "$OUT/$name.log" 2>&1
      rc=$?; tail -2 "$OUT/$name.log" ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
      rc=$?; tail -3 "$OUT/smoke.log" ;;
    cmd)
      log="$OUT/cmd_$(date +%s).log"
      timeout -k 10 $T bash -c "$arg" > "$log" 2>&1
      rc=$?; tail -15 "$log" ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
  echo "=== $step rc=$rc"
  [[ $rc == 0 ]] || exit $rc
done
