#!/bin/bash
# GPU side: one bench config under different environment settings:
#   bash tools/run_env_ab_cfg.sh CONFIG "NAME:ENV=..." ...
set -o pipefail
mkdir -p gpurun_out
CFG=$1
shift
for spec in "$@"; do
  name=${spec%%:*}; envs=${spec#*:}
  env $envs timeout -k 10 400 python bench.py --config $CFG --steps 4 --warmup 2 --no-cpu-baseline > gpurun_out/env_${CFG}_$name.log 2>&1 || { tail -20 gpurun_out/env_${CFG}_$name.log; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/env_${CFG}_$name.log').read().strip().splitlines()[-1]);print('$CFG $name',d['value'],d['roofline']['avg_launch_us'],d['phase_ms_per_step'])"
done
