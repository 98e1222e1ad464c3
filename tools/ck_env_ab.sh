#!/bin/bash
# Checkpoint p99 gate under environment variants, interleaved:
#   tools/ck_env_ab.sh <reps> "name1:VAR=a,VAR2=b" "name2:" ...
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/cke
reps=$1; shift
for r in $(seq "$reps"); do
  for v in "$@"; do
    name=${v%%:*}; envs=${v#*:}
    envargs=()
    IFS=',' read -ra kv <<< "$envs"
    for e in "${kv[@]}"; do [[ -n "$e" ]] && envargs+=("$e"); done
    env "${envargs[@]}" timeout -k 10 250 python -u -m pytest tests/test_gpu_checkpoint.py -k p99 -x -q -s \
      --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/cke/${name}_$r.log 2>&1
    echo "$name rep $r rc=$? $(grep -h "p99_ms_no_ckpt" gpurun_out/cke/${name}_$r.log | python3 -c "
import sys,ast
for l in sys.stdin:
    for x in l.split('{')[1:]:
        d=ast.literal_eval('{'+x.split('}')[0]+'}'); print('%.2f/%.2f=%.3f w%d' % (d['p99_ms_no_ckpt'], d['p99_ms_ckpt1'], d['p99_ms_ckpt1']/d['p99_ms_no_ckpt'], d['written']), end='  ')
")"
  done
done
