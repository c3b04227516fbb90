#!/bin/bash
# r04 A/B set: C2 bench per (AICP_SEQ_POLL_EV, AICP_TREE_LVL), then the tree builders on C5.
set -o pipefail
mkdir -p gpurun_out
for pe in 1 0; do
  for lv in 0 1; do
    AICP_SEQ_POLL_EV=$pe AICP_TREE_LVL=$lv timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-batched > gpurun_out/c2_pe${pe}_lv${lv}.json 2> gpurun_out/c2_pe${pe}_lv${lv}.err || { tail -5 gpurun_out/c2_pe${pe}_lv${lv}.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/c2_pe${pe}_lv${lv}.json')); print('POLL_EV=$pe LVL=$lv c2', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['launches'])"
  done
done
bash tools/env_kstats_ab.sh tree_ab AICP_TREE_LVL "0 1" c5 "k_tr_sub|k_tr_mid|k_tr_move|k_tr_scat"
