#!/bin/bash
# Multi-rank engine DP on one GPU through the host-staged gloo communicator
# (RCCL refuses two ranks on one device): the driver's launcher, N processes.
#   $1 ranks, then extra bench args.  Output: gpurun_out/dp<N>.log (+ .json)
# The JSON line carries per-rank peak RSS, pinned bytes and pool generation
# time (per_rank_host) and the whole wall time (wall_s) -- the host budget of
# the driver's 8-rank bench (600 s limit).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
n=$1; shift
port=$((29500 + RANDOM % 2000))
t0=$(date +%s)
timeout -k 10 ${DP_TIMEOUT:-600} python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
  --master-addr 127.0.0.1 --master-port $port bench.py --gpus $n --comm gloo "$@" \
  --json-out gpurun_out/dp$n.json > gpurun_out/dp$n.log 2>&1
rc=$?
echo "launcher wall: $(( $(date +%s) - t0 )) s, rc=$rc"
grep metric gpurun_out/dp$n.log || tail -20 gpurun_out/dp$n.log
exit $rc
