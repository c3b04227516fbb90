#!/bin/bash
# GPU side: bench each prebuilt variant on one bench config: bash tools/run_variants_cfg.sh CONFIG NAME...
set -o pipefail
mkdir -p gpurun_out
CFG=$1
shift
for v in "$@"; do
  AICP_HIP_LIB=$PWD/build_ab/lib_$v.so timeout -k 10 400 python bench.py --config $CFG --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/var_${CFG}_$v.log 2>&1 || { tail -20 gpurun_out/var_${CFG}_$v.log; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/var_${CFG}_$v.log').read().strip().splitlines()[-1]);print('$CFG $v',d['value'],d['roofline']['avg_launch_us'],d['roofline']['frac'],d['phase_ms_per_step'])"
done
