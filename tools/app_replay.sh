#!/bin/bash
# The real LinearRegression driver on the measured path: replay of 30 distinct
# pre-generated wide batches (page-locked UTF-8), 1M tweets each, vs bench.py.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
set -o pipefail
rm -f gpurun_out/app_metrics.jsonl
TWTML_METRICS=gpurun_out/app_metrics.jsonl timeout -k 10 400 python -m twitter_stream_ml_amd --master 'rocm[1]' \
  --source replay:synthetic:wide:30 --batchSize 1000000 --seconds 0 --numBatches 30 --sourceRate 0 \
  -f 1000000 --lightning http://127.0.0.1:9 --twtweb http://127.0.0.1:9 > gpurun_out/app.log 2>&1 || { tail -30 gpurun_out/app.log; exit 1; }
grep summary gpurun_out/app_metrics.jsonl
