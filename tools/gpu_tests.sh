#!/bin/bash
# GPU test suite (one pytest process), log under gpurun_out/.  Args: extra pytest args.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread "$@" \
  > gpurun_out/pytest_gpu.log 2>&1; rc=$?
grep -E "passed|failed|error" gpurun_out/pytest_gpu.log | tail -5
exit $rc
