#!/bin/bash
# PMC passes for one kernel of the bench: bash tools/pmc.sh NAME REGEX
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
N=${1:-pmc}; R=${2:-k_icp_nn}
rm -rf gpurun_out/$N && mkdir -p gpurun_out/$N
i=0
# PMC_SETS="A B C;D E" overrides the counter passes (one pass per ';'-separated set)
SETS=()
if [ -n "$PMC_SETS" ]; then IFS=';' read -ra SETS <<< "$PMC_SETS"; fi
DEFAULT=("SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_WAVES"
         "TCC_HIT_sum TCC_MISS_sum TCC_READ_sum TCC_EA0_RDREQ_sum" \
         "SQ_INSTS_SALU SQ_INST_LEVEL_VMEM SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM_RD SQ_LEVEL_WAVES" \
         "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum")
[ ${#SETS[@]} -eq 0 ] && SETS=("${DEFAULT[@]}")
for C in "${SETS[@]}"; do
  i=$((i+1))
  timeout -k 10 150 rocprofv3 --pmc $C --kernel-include-regex "$R" --output-format csv -d gpurun_out/$N/p$i -o run -- python3 bench.py --config ${CFG:-c2} --steps 1 --warmup 0 --no-cpu-baseline --no-batched > gpurun_out/$N/p$i.log 2>&1 || { tail -5 gpurun_out/$N/p$i.log; exit 1; }
done
python3 - "$N" <<'PY'
import csv, glob, sys, collections
n = sys.argv[1]
agg = collections.defaultdict(float); cnt = collections.defaultdict(int)
for f in glob.glob(f"gpurun_out/{n}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        agg[r["Counter_Name"]] += float(r["Counter_Value"]); cnt[r["Counter_Name"]] += 1
for k in sorted(agg): print(f"{k:40s} {agg[k]:16.0f}  ({cnt[k]} dispatches)")
PY
