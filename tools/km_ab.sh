set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/km
TAG=km STEP_TIMEOUT=300 TESTS_TIMEOUT=600 bash tools/gpu_run.sh "tests:kmeans"
TWTML_DEBUG_KM=1 timeout -k 10 200 python -u bench.py --model kmeans --steps 6 --warmup 2 > gpurun_out/km/debug_new.log 2>&1
(cd abvar && TWTML_DEBUG_KM=1 timeout -k 10 200 python -u bench.py --model kmeans --steps 6 --warmup 2) > gpurun_out/km/debug_base.log 2>&1
grep "\[km\]" gpurun_out/km/debug_new.log | tail -3; grep "\[km\]" gpurun_out/km/debug_base.log | tail -3
for w in new base; do
  d=.; [ $w = base ] && d=abvar
  (cd $d && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/km/prof_$w -o run -- python -u bench.py --model kmeans --prepacked) > gpurun_out/km/prof_$w.log 2>&1
  python tools/kstats.py gpurun_out/km/prof_$w/run_kernel_stats.csv 12 > gpurun_out/km/kernels_$w.txt
  grep -E "k_km_assign|k_km_refine|k_km_features" gpurun_out/km/kernels_$w.txt | sed "s/^/$w /"
done
TAG=kmab bash tools/ab_tree.sh abvar 2 --model kmeans --prepacked
