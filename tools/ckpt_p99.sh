#!/bin/bash
# Checkpoint p99 test under snapshot-copy duty cycles (TWTML_SNAP_DUTY): JSON per duty under gpurun_out/ckpt_<duty>/.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for d in ${DUTIES:-0.25 0.05}; do
  TWTML_SNAP_DUTY=$d TWTML_TEST_OUT=gpurun_out/ckpt_$d timeout -k 10 300 python -u -m pytest -x -q \
    tests/test_gpu_checkpoint.py::test_async_checkpoint_p99_wide_1e8 --timeout 240 --timeout-method thread \
    > gpurun_out/ckpt_$d.log 2>&1
  rc=$?
  echo "duty $d rc $rc: $(cat gpurun_out/ckpt_$d/ckpt_p99.json 2>/dev/null)"
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done
