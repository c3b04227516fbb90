#!/bin/bash
# A/B of the overlap marking (AICP_OVL_TEST=0: plain byte stores; 1: grouped test-before-store;
# 2: workgroup LDS cache of stored voxels):
# k_ovl_mark's rocprofv3 average and PMC WRITE_SIZE on C5, and the C2 / C5 bench values.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
N=${1:-ovl_ab}
rm -rf gpurun_out/$N && mkdir -p gpurun_out/$N
for v in ${MODES:-0 2}; do
  AICP_OVL_TEST=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$N/t$v -o run -- python3 bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline --no-batched > gpurun_out/$N/t$v.log 2>&1 || { tail -5 gpurun_out/$N/t$v.log; exit 1; }
  python3 tools/kstats_short.py $(find gpurun_out/$N/t$v -name "*kernel_stats.csv" | head -1) 40 | grep -E "ovl|total" 
  AICP_OVL_TEST=$v timeout -k 10 150 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_ovl_mark --output-format csv -d gpurun_out/$N/w$v -o run -- python3 bench.py --config c5 --steps 1 --warmup 0 --no-cpu-baseline --no-batched > gpurun_out/$N/w$v.log 2>&1 || { tail -5 gpurun_out/$N/w$v.log; exit 1; }
  python3 - gpurun_out/$N/w$v <<'PY'
import csv, glob, sys
rows = [r for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True) for r in csv.DictReader(open(f))]
v = [float(r["Counter_Value"]) for r in rows if r["Counter_Name"] == "WRITE_SIZE"]
print("k_ovl_mark WRITE_SIZE per dispatch (KiB x1024 -> GB):", [round(x * 1024 / 1e9, 3) for x in v])
PY
  AICP_OVL_TEST=$v timeout -k 10 200 python3 bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline --no-batched > gpurun_out/$N/c5_$v.json 2> gpurun_out/$N/c5_$v.err || exit 1
  AICP_OVL_TEST=$v timeout -k 10 200 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-batched > gpurun_out/$N/c2_$v.json 2> gpurun_out/$N/c2_$v.err || exit 1
  python3 -c "import json; a=json.load(open('gpurun_out/$N/c5_$v.json')); b=json.load(open('gpurun_out/$N/c2_$v.json')); print('OVL_TEST=$v c5', a['value'], 'c2', b['value'])"
done
