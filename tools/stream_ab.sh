#!/bin/bash
# GPU side: C2 stream A/B, alternating A B A B ... for REPS rounds so box drift hits every variant
# alike. A variant is a prebuilt library name (build_ab/lib_NAME.so, tools/variants.sh) or an
# environment setting VAR=VALUE run on the in-tree library. bash tools/stream_ab.sh REPS V...
set -o pipefail
mkdir -p gpurun_out
REPS=$1
shift
for r in $(seq 1 $REPS); do
  for v in "$@"; do
    tag=${v//[^A-Za-z0-9_]/_}
    if [[ "$v" == *=* ]]; then envs=("$v"); else envs=("AICP_HIP_LIB=$PWD/build_ab/lib_$v.so"); fi
    env "${envs[@]}" timeout -k 10 120 python bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-batched > gpurun_out/sab_$tag.log 2>&1 || { tail -20 gpurun_out/sab_$tag.log; exit 1; }
    python3 -c "import json;d=json.loads(open('gpurun_out/sab_$tag.log').read().strip().splitlines()[-1]);print('$v',d['value'],d['ms_per_step'],d['roofline']['avg_launch_us'],d['mean_iterations'])"
  done
done
