#!/bin/bash
# GPU side: bench each prebuilt variant (tools/variants.sh); one line per variant.
set -o pipefail
mkdir -p gpurun_out
for v in "$@"; do
  AICP_HIP_LIB=$PWD/build_ab/lib_$v.so timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/var_$v.log 2>&1 || { tail -20 gpurun_out/var_$v.log; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/var_$v.log').read().strip().splitlines()[-1]);print('$v',d['value'],d['roofline']['avg_launch_us'],d['roofline']['frac'],d['phase_ms_per_step']['icp_loop_gpu'],d['phase_ms_per_step']['normal_tree_and_normals_gpu (stream 2)'])"
done
