#!/bin/bash
# Final kernel tables (k-means config 4, wide LR overlapped and serial) + k-means PMC passes.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TOP=24 bash tools/kprof.sh km --model kmeans --steps 20 --warmup 5 || exit 1
TOP=24 bash tools/kprof.sh wide --steps 20 --warmup 5 || exit 1
TWTML_OVERLAP=0 TOP=24 bash tools/kprof.sh wide_serial --steps 20 --warmup 5 || exit 1
CASES=km bash tools/pmc_r3.sh
