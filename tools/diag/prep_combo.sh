cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for r in 1 2 3; do
  for combo in "1 1" "2 1" "2 4" "1 4"; do
    set -- $combo
    TWTML_PREP_SLICES=$1 TWTML_PREP_WG_MULT=$2 timeout -k 10 200 python bench.py --profile wide --steps 10 --pool 3 > gpurun_out/combo.log 2>&1 || exit 1
    grep metric gpurun_out/combo.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('S=$1 M=$2', round(d['value']/1e6,1), d['ms_per_step'], round(d['train_ms_mean'],3), round(d['prep_ms_mean'],3))"
  done
done
