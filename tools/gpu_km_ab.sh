cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for v in reg lds1 lds; do
  TWTML_KM_ASSIGN=$v timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -p no:cacheprovider tests/test_gpu_kmeans.py -k "bench_scale" -s > gpurun_out/km_$v.log 2>&1; echo "$v rc=$?"; grep -E "batch [0-9]:|passed|failed|Max abs" gpurun_out/km_$v.log
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -p no:cacheprovider tests/test_gpu_kmeans.py -k "features_exact" > gpurun_out/km_feat.log 2>&1; echo "feat rc=$?"; tail -3 gpurun_out/km_feat.log
