#!/bin/bash
# Round-end validation on one box: the GPU suite, smoke(), every README bench
# line (tools/gpu_final.sh), and the wide bench's kernel table.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
TAG=final STEP_TIMEOUT=200 TESTS_TIMEOUT=900 bash tools/gpu_run.sh tests smoke || exit $?
bash tools/gpu_final.sh || exit $?
TAG=final STEP_TIMEOUT=200 bash tools/gpu_run.sh prof:wide
