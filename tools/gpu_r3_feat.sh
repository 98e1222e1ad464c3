#!/bin/bash
# Featurizer change check: LR engine + k-means GPU tests, then wide LR and k-means kernel tables.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TEST_TIMEOUT=600 bash tools/gpu_t.sh tests/test_gpu_lr_engine.py tests/test_gpu_kmeans.py tests/test_gpu_tiered.py || exit 1
TOP=14 bash tools/kprof.sh km --model kmeans --steps 10 --warmup 3 || exit 1
TOP=24 bash tools/kprof.sh wide --steps 10 --warmup 3
