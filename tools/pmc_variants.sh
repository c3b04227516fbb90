#!/bin/bash
# PMC counters of the NN kernel for prebuilt variants (tools/variants.sh): bash tools/pmc_variants.sh NAME...
set -o pipefail
export PMC_SETS="${PMC_SETS:-SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES;TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum TCC_HIT_sum TCC_MISS_sum TA_BUSY_avr GRBM_GUI_ACTIVE}"
for v in "$@"; do
  AICP_HIP_LIB=$PWD/build_ab/lib_$v.so bash tools/pmc.sh pmcv_$v "${PMC_KERNEL:-k_icp_nn}" > gpurun_out/pmcv_$v.txt 2>&1 || { cat gpurun_out/pmcv_$v.txt; exit 1; }
  echo "== $v"; cat gpurun_out/pmcv_$v.txt
done
