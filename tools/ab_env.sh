#!/bin/bash
# A/B of an environment switch on the bench: bash tools/ab_env.sh VAR "v1 v2 ..."
set -o pipefail
mkdir -p gpurun_out
VAR=$1
for v in $2; do
  export $VAR=$v
  timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/ab_$v.log 2>&1 || { tail -20 gpurun_out/ab_$v.log; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/ab_$v.log').read().strip().splitlines()[-1]);print('$VAR=$v',d['value'],d['roofline']['avg_launch_us'],d['phase_ms_per_step'],d['mean_iterations'])"
done
