#!/bin/bash
# Multi-rank engine DP on one GPU through the host-staged gloo communicator
# (RCCL refuses two ranks on one device): the real launcher, N processes.
#   $1 ranks, then extra bench args.  Output: gpurun_out/dp<N>.log
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
n=$1; shift
port=$((29500 + RANDOM % 2000))
OMP_NUM_THREADS=2 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
  --master-addr 127.0.0.1 --master-port $port bench.py --gpus $n --comm gloo "$@" > gpurun_out/dp$n.log 2>&1
rc=$?
grep metric gpurun_out/dp$n.log || tail -20 gpurun_out/dp$n.log
exit $rc
