#!/bin/bash
# C5 (1024 pairs) with the in-tree library and each library given, alternating: clouds/s, NN per
# launch (HIP events). bash tools/lib_ab_c5.sh N lib...
set -o pipefail
mkdir -p gpurun_out
N=${1:-2}; shift
for i in $(seq $N); do
  for v in "" "$@"; do
    AICP_HIP_LIB=$v timeout -k 10 400 python bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/c5ab.json 2> gpurun_out/c5ab.err || { tail -5 gpurun_out/c5ab.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/c5ab.json'));print('${v:-tree}',d['value'],d['ms_per_step'],d['roofline']['avg_launch_us'],d['roofline']['frac'])"
  done
done
