#!/bin/bash
# The BASELINE.json configurations other than the default C2 bench line, one bench run each.
set -o pipefail
mkdir -p gpurun_out
for c in ${@:-c3 c4 c5}; do
  timeout -k 10 500 python bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/cfg_$c.log 2>&1 || { tail -20 gpurun_out/cfg_$c.log; exit 1; }
  tail -1 gpurun_out/cfg_$c.log | cut -c1-1500
done
