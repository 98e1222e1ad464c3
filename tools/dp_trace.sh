#!/bin/bash
# Per-stream kernel trace of 2 loopback DP engines (tools/diag/dp_stream_trace.py).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
rm -rf gpurun_out/dptrace
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/dptrace -o run -- \
  python tools/diag/dp_stream_trace.py > gpurun_out/dptrace.log 2>&1 || { tail -20 gpurun_out/dptrace.log; exit 1; }
grep rank gpurun_out/dptrace.log
python tools/diag/stream_kernels.py gpurun_out/dptrace/run_kernel_trace.csv > gpurun_out/dptrace_streams.txt
cat gpurun_out/dptrace_streams.txt
