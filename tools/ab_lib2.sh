#!/bin/bash
# Alternating A/B of library builds on the C2 bench (default lib = "default"), R rounds each:
# bash tools/ab_lib2.sh R path/to/a.so ...
set -o pipefail
mkdir -p gpurun_out
R=$1; shift
for r in $(seq 1 $R); do
  for lib in default "$@"; do
    tag=$(basename $lib .so)
    if [ "$lib" = default ]; then unset AICP_HIP_LIB; else export AICP_HIP_LIB=$PWD/$lib; fi
    timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-batched > gpurun_out/ab2_$tag.json 2> gpurun_out/ab2_$tag.err || { tail -20 gpurun_out/ab2_$tag.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/ab2_$tag.json'));print('$tag',d['value'],d['ms_per_step'],d['roofline']['avg_launch_us'])"
  done
done
unset AICP_HIP_LIB
