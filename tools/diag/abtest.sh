cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
SO=twitter_stream_ml_amd/_twtml_hip.cpython-310-x86_64-linux-gnu.so
for v in B B A; do
  cp ab/$v.so $SO
  timeout -k 10 300 python -u -m pytest tests/test_gpu_dp_procs.py tests/test_gpu_tiered.py -x -q -m gpu --timeout 200 -k "world2 or tiered" > gpurun_out/abt_$v.log 2>&1; echo "$v rc=$? $(tail -1 gpurun_out/abt_$v.log)"
done
