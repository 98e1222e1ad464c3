#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
SO=twitter_stream_ml_amd/_twtml_hip.cpython-310-x86_64-linux-gnu.so
cp $SO ab/orig.so
for v in A B A B; do
  cp ab/$v.so $SO
  timeout -k 10 200 python -m pytest tests/test_gpu_apps.py -q -k plot_does_not_stall -s 2>&1 | grep -E "step p99|passed|failed" | sed "s/^/$v /"
done
cp ab/orig.so $SO
