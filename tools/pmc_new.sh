#!/bin/bash
# PMC rows for the kernels new or rewritten in round 6 (kernel trace + counter
# passes, no sys/runtime trace; per-block limits as in tools/pmc_r3.sh):
#   row_special  k_row_special beside k_cesu_decode, headline bench (UTF-8 ingest)
#   snapshot     k_nz_pack / k_nz_scan / k_nz_move, the checkpoint gate's run (F = 1e8)
# Output: gpurun_out/pmc_new/<case>_{kt,p1..p4}/ + summary.md
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/pmc_new; export TMPDIR=/tmp
PASSES=("SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU"
        "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_INSTS_MFMA GRBM_GUI_ACTIVE GRBM_COUNT"
        "FETCH_SIZE"
        "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum")
one() {   # case regex program args...
  local name=$1 re=$2; shift 2
  rm -rf gpurun_out/pmc_new/${name}_kt
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pmc_new/${name}_kt -o run -- \
    "$@" > gpurun_out/pmc_new/${name}_kt.log 2>&1 || { echo "kt $name rc=$?"; return 1; }
  local k=0
  for SET in "${PASSES[@]}"; do
    k=$((k+1)); rm -rf gpurun_out/pmc_new/${name}_p$k
    timeout -s KILL 240 rocprofv3 --pmc $SET --kernel-include-regex "$re" --output-format csv \
      -d gpurun_out/pmc_new/${name}_p$k -o run -- "$@" > gpurun_out/pmc_new/${name}_p$k.log 2>&1
    rc=$?; echo "$name pass $k rc=$rc"
    [ $rc -ne 0 ] && { tail -3 gpurun_out/pmc_new/${name}_p$k.log; return 1; }
  done
  return 0
}
MEASURE='import sys, tempfile; sys.path[:0] = [".", "tests"]; import test_gpu_checkpoint as t; print(t._measure(tempfile.mkdtemp()))'
one row_special 'k_row_special|k_cesu_decode' python bench.py --steps 3 --warmup 1 || exit 1
one snapshot 'k_nz_' python -c "$MEASURE" || exit 1
python tools/pmc_report.py gpurun_out/pmc_new > gpurun_out/pmc_new/summary.md
cat gpurun_out/pmc_new/summary.md
