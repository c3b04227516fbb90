#!/bin/bash
# GPU round-trip for a kernel change: parity tests, then an A/B of an environment switch on the
# bench. bash tools/gpu_ab.sh VAR "v1 v2 ..." [bench args]
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/parity.log 2>&1 || { tail -40 gpurun_out/parity.log; exit 1; }
tail -2 gpurun_out/parity.log
VAR=$1
shift
VALS=$1
shift
for v in $VALS; do
  export $VAR=$v
  timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline "$@" > gpurun_out/ab_$v.log 2>&1 || { tail -20 gpurun_out/ab_$v.log; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/ab_$v.log').read().strip().splitlines()[-1]);print('$VAR=$v',d['value'],d['roofline']['avg_launch_us'],d['roofline']['frac'],d['phase_ms_per_step'],d['mean_iterations'])"
done
