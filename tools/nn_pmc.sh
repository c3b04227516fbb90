#!/bin/bash
# PMC passes over the C2 NN launches (one pass per counter group): is k_icp_nn bound by its
# address / tag pipeline (TA, TCP) or by waiting on L2?
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
i=0
for set in "TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE GRBM_TA_BUSY" \
           "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_INSTS_SALU SQ_WAVES"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --kernel-include-regex "k_icp_nn" --output-format csv -d gpurun_out/nnpmc/p$i -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-batched > gpurun_out/nnpmc/p$i.log 2>&1 || { tail -20 gpurun_out/nnpmc/p$i.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
for f in sorted(glob.glob('gpurun_out/nnpmc/p*/run_counter_collection.csv')):
    acc=collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        acc[r['Counter_Name']].append(float(r['Counter_Value']))
    print(f, {k: round(sum(v)/len(v)) for k,v in acc.items()}, 'dispatch-rows', {k: len(v) for k,v in acc.items()})
PY
