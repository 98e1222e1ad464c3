cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
for r in 1 2; do for g in 0 240 224 192 160; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --sgd-grid $g > gpurun_out/grid_$g.log 2>&1 || { echo FAIL $g; tail -3 gpurun_out/grid_$g.log; exit 1; }
  grep metric gpurun_out/grid_$g.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('grid=$g', round(d['value']/1e6,1), 'M/s', d['ms_per_step'], 'ms train', round(d.get('train_ms_mean',0),3), 'prep', round(d.get('prep_ms_mean',0),3), 'it', d['gd_iterations_mean'])"
done; done
