#!/bin/bash
# Kernel table of bench.py under an environment variant:
#   tools/prof_env.sh <name> "VAR=a,VAR2=b" [bench args]  -> gpurun_out/$TAG/<name>_kernels.txt
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/${TAG:-prof}
mkdir -p "$OUT"
name=$1; envs=$2; shift 2
IFS=',' read -ra kv <<< "$envs"
for e in "${kv[@]}"; do [[ -n "$e" ]] && export "$e"; done
rm -rf "$OUT/$name"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$name" -o run -- \
  python3 -u bench.py "$@" > "$OUT/$name.log" 2>&1 || { tail -20 "$OUT/$name.log"; exit 1; }
python3 tools/kstats.py "$OUT/$name/run_kernel_stats.csv" 40 > "$OUT/${name}_kernels.txt" 2>&1
rm -f "$OUT/$name/run_kernel_trace.csv"
head -24 "$OUT/${name}_kernels.txt"
