#!/bin/bash
# A/B (ab/A.so = HEAD, ab/B.so = working tree): k-means tests, wide bench x3, kernel deltas, k-means kernels.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q tests/test_gpu_kmeans.py --timeout 200 --timeout-method thread > gpurun_out/km_tests.log 2>&1 || { tail -30 gpurun_out/km_tests.log; exit 1; }
tail -1 gpurun_out/km_tests.log
bash tools/ab.sh 3 --steps 12 --warmup 3 || exit 1
bash tools/kprof_ab.sh "decode|normalize|bounds|far_csc|remap|featurize|iter_hyb<true" --steps 10 --warmup 3 || exit 1
TOP=12 bash tools/kprof.sh km --model kmeans --steps 10 --warmup 3
