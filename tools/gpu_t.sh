#!/bin/bash
# Selected GPU tests in one pytest process: tools/gpu_t.sh <pytest args...>
# (log: gpurun_out/t.log; TEST_TIMEOUT bounds the whole run)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest -x -v --timeout 240 --timeout-method thread -p no:cacheprovider "$@" \
  > gpurun_out/t.log 2>&1; rc=$?
grep -E "PASS|FAIL|ERROR|passed|failed|error" gpurun_out/t.log | tail -60
exit $rc
