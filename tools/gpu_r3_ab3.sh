#!/bin/bash
# k-means tests on the tree; A/B kernel tables: LR wide serial (update kernel) and k-means config 4 (featurizer).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q tests/test_gpu_kmeans.py tests/test_gpu_apps.py --timeout 200 --timeout-method thread > gpurun_out/km_tests.log 2>&1 || { tail -30 gpurun_out/km_tests.log; exit 1; }
tail -1 gpurun_out/km_tests.log
TWTML_OVERLAP=0 VARIANTS="A B" bash tools/kprof_vs.sh "update|far_grad|iter_hyb" 0 || exit 1
VARIANTS="A B" bash tools/kprof_vs.sh "km_features|decode|normalize" 2 --model kmeans
