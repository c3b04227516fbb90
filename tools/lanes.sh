#!/bin/bash
# bench.py with 1..3 concurrent lanes (copies of the step, each its own context and host thread)
set -o pipefail
mkdir -p gpurun_out
for l in ${@:-1 2 3}; do
  timeout -k 10 300 python bench.py --steps 12 --warmup 2 --no-cpu-baseline --lanes $l > gpurun_out/lanes_$l.log 2>&1 || { tail -20 gpurun_out/lanes_$l.log; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/lanes_$l.log').read().strip().splitlines()[-1]);print('lanes $l',d['value'],d['ms_per_step'],d['roofline']['avg_launch_us'],d['roofline']['frac'])"
done
