#!/bin/bash
# Extended PMC passes (kernel-trace only) for one kernel regex: instruction
# mix, waits, LDS, cache hit/miss and HBM traffic.  Usage: tools/pmc2.sh <regex> [bench args]
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
RE=${1:-k_featurize}; shift
ARGS=${*:---steps 3 --warmup 1}
i=0
for SET in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM" \
           "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM SQ_WAIT_ANY SQ_ACTIVE_INST_MISC" \
           "TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum" \
           "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"; do
  i=$((i+1))
  rm -rf gpurun_out/pmcx$i
  timeout -k 10 240 rocprofv3 --pmc $SET --kernel-include-regex "$RE" --output-format csv \
      -d gpurun_out/pmcx$i -o run -- python bench.py $ARGS > gpurun_out/pmcx$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/pmcx$i.log; [ $rc -ge 124 ] && exit $rc; fi
done
python tools/pmc_summary.py gpurun_out/pmcx*/run_counter_collection.csv
