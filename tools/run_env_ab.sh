#!/bin/bash
# GPU side: C2 bench under different environment settings: bash tools/run_env_ab.sh "NAME=ENV..." ...
# e.g. bash tools/run_env_ab.sh "p11:" "p8:AICP_TREE_PLAN=8"
set -o pipefail
mkdir -p gpurun_out
for spec in "$@"; do
  name=${spec%%:*}; envs=${spec#*:}
  env $envs timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/env_$name.log 2>&1 || { tail -20 gpurun_out/env_$name.log; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/env_$name.log').read().strip().splitlines()[-1]);print('$name',d['value'],d['roofline']['avg_launch_us'],d['phase_ms_per_step'])"
done
