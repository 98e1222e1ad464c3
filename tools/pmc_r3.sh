#!/bin/bash
# PMC evidence for the final kernels (kernel-trace + counter passes, no
# sys/runtime trace); rounds 3-4.  Passes respect the per-block limits (SQ <= 8,
# TCC <= 4, GRBM <= 2).  Output: gpurun_out/pmc_r3/<case>_p<k>/ + summary.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/pmc_r3; export TMPDIR=/tmp
LR_RE='k_sgd_iter_hyb|k_remap_hybrid|k_featurize|k_far_grad|k_sgd_update|k_sgd_reduce|k_cesu_decode|k_row_normalize|k_tier|k_prep_init|k_scan_excl|k_tile_sum|k_rows_scan|k_batch_stats|k_batch_bounds|k_far_csc'
KM_RE='k_km_'
PASSES=("SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU"
        "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_INSTS_MFMA GRBM_GUI_ACTIVE GRBM_COUNT"
        "FETCH_SIZE"
        "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum")
one() {   # case regex args...
  local name=$1 re=$2; shift 2
  rm -rf gpurun_out/pmc_r3/${name}_kt
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pmc_r3/${name}_kt -o run -- \
    python bench.py "$@" > gpurun_out/pmc_r3/${name}_kt.log 2>&1 || { echo "kt $name rc=$?"; return 1; }
  local k=0
  for SET in "${PASSES[@]}"; do
    k=$((k+1)); rm -rf gpurun_out/pmc_r3/${name}_p$k
    timeout -s KILL 240 rocprofv3 --pmc $SET --kernel-include-regex "$re" --output-format csv \
      -d gpurun_out/pmc_r3/${name}_p$k -o run -- python bench.py "$@" > gpurun_out/pmc_r3/${name}_p$k.log 2>&1
    rc=$?; echo "$name pass $k rc=$rc"
    [ $rc -ne 0 ] && { tail -3 gpurun_out/pmc_r3/${name}_p$k.log; return 1; }
  done
  return 0
}
[ -z "$CASES" ] && CASES="lr_wide km"   # also: lr_forced, lr_bench, lr_1e8 (config 5)
for c in $CASES; do case $c in lr_wide) one lr_wide "$LR_RE" --prepacked --profile wide --pool 3 --steps 2 --warmup 1 || exit 1;; lr_forced) one lr_forced "$LR_RE" --force-dp --prepacked --profile wide --pool 3 --steps 2 --warmup 1 || exit 1;; lr_bench) one lr_bench "$LR_RE" --prepacked --profile bench --pool 4 --steps 3 --warmup 1 || exit 1;; km) one km "$KM_RE" --model kmeans --prepacked --pool 4 --steps 3 --warmup 1 || exit 1;; lr_1e8) one lr_1e8 "$LR_RE" --prepacked --profile wide --features 100000000 --hash murmur3 --pool 3 --steps 2 --warmup 1 || exit 1;; esac; done
python tools/pmc_report.py gpurun_out/pmc_r3 > gpurun_out/pmc_r3/summary.md
head -60 gpurun_out/pmc_r3/summary.md
