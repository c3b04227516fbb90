#!/bin/bash
# Alternating A/B of context option sets (aicp_hip_options) on one bench config, R rounds:
# CFG=c5 bash tools/opt_ab.sh R "raw_tree_first=0" "raw_tree_first=1 raw_first_at=1"
set -o pipefail
mkdir -p gpurun_out
R=$1; shift
CFG=${CFG:-c5}
for r in $(seq 1 $R); do
  i=0
  for a in "$@"; do
    i=$((i+1))
    o=""; for kv in $a; do o="$o --opt $kv"; done
    timeout -k 10 240 python bench.py --config $CFG $o --steps ${STEPS:-2} --warmup 1 --no-cpu-baseline > gpurun_out/eab_$i.json 2> gpurun_out/eab_$i.err || { tail -20 gpurun_out/eab_$i.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/eab_$i.json'));print('[$a]',d['value'],d['ms_per_step'])"
  done
done
