#!/bin/bash
# A/B of library builds on the bench: bash tools/ab_lib.sh path/to/a.so path/to/b.so ...
set -o pipefail
mkdir -p gpurun_out
for lib in "$@"; do
  tag=$(basename $lib .so)
  AICP_HIP_LIB=$PWD/$lib timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/abl_$tag.log 2>&1 || { tail -20 gpurun_out/abl_$tag.log; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/abl_$tag.log').read().strip().splitlines()[-1]);print('$tag',d['value'],d['roofline']['avg_launch_us'],d['phase_ms_per_step'],d['mean_iterations'])"
done
