#!/bin/bash
# A/B of the NN engines on the bench: bash tools/ab.sh
set -o pipefail
mkdir -p gpurun_out
for e in 1 0; do
  AICP_NN_ENGINE=$e timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/ab_e$e.log 2>&1 || { tail -20 gpurun_out/ab_e$e.log; exit 1; }
  python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/ab_e$e.log') if l.startswith('{')][-1]); print('engine $e', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['phase_ms_per_step'])"
done
