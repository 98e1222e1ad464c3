#!/bin/bash
# PMC counter passes (kernel-trace only, no sys/runtime trace) over a short
# bench run, filtered to one kernel regex.  Usage: tools/pmc.sh <regex> [bench args]
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
RE=${1:-k_featurize}; shift
ARGS=${*:---steps 3 --warmup 1}
i=0
for SET in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU" \
           "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM SQ_WAIT_ANY" \
           "TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum"; do
  i=$((i+1))
  rm -rf gpurun_out/pmc$i
  timeout -k 10 240 rocprofv3 --pmc $SET --kernel-include-regex "$RE" --output-format csv \
      -d gpurun_out/pmc$i -o run -- python bench.py $ARGS > gpurun_out/pmc$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/pmc$i.log; [ $rc -ge 124 ] && exit $rc; fi
done
python tools/pmc_summary.py gpurun_out/pmc*/run_counter_collection.csv
