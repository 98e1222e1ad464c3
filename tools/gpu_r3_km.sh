#!/bin/bash
# k-means: exact-features + config-4 oracle tests, assign-variant A/B, then the config-4 kernel table.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TEST_TIMEOUT=600 bash tools/gpu_t.sh tests/test_gpu_kmeans.py || exit 1
for v in lds lds2; do
  TWTML_KM_ASSIGN=$v TOP=6 bash tools/kprof.sh km_$v --model kmeans --steps 10 --warmup 3 || exit 1
done
