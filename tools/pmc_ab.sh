set -o pipefail
export PMC_SETS="SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_VMEM SQ_BUSY_CYCLES;TCP_TOTAL_CACHE_ACCESSES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum;TA_BUSY_avr TA_DATA_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE"
for e in 3 2; do AICP_NN_ENGINE=$e bash tools/pmc.sh pmc_e$e k_icp_nn > gpurun_out/pmc_e$e.txt 2>&1 || exit 1; echo "engine $e"; cat gpurun_out/pmc_e$e.txt; done
