#!/bin/bash
# PMC A/B of an environment switch on the NN kernel: bash tools/pmc_ab_env.sh VAR "v1 v2" [kernel regex]
set -o pipefail
export PMC_SETS="${PMC_SETS:-SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_VMEM SQ_BUSY_CYCLES SQ_WAVES;TCP_TOTAL_CACHE_ACCESSES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum;TA_BUSY_avr TA_DATA_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE;TCC_HIT_sum TCC_MISS_sum}"
VAR=$1
for v in $2; do
  export $VAR=$v
  bash tools/pmc.sh pmc_$v "${3:-k_icp_nn}" > gpurun_out/pmc_$v.txt 2>&1 || { cat gpurun_out/pmc_$v.txt; exit 1; }
  echo "$VAR=$v"; cat gpurun_out/pmc_$v.txt
done
