#!/bin/bash
# One bench config with the in-tree library and each library given, alternating, N rounds:
# CFG=c5 bash tools/lib_ab.sh N lib...   (CFG empty: the default C2 stream)
set -o pipefail
mkdir -p gpurun_out
N=${1:-2}; shift
ARGS="--steps ${STEPS:-2} --warmup 1 --no-cpu-baseline"
[ -n "$CFG" ] && ARGS="--config $CFG $ARGS"
[ -z "$CFG" ] && ARGS="$ARGS --no-batched"
for i in $(seq $N); do
  for v in "" "$@"; do
    AICP_HIP_LIB=$v timeout -k 10 400 python bench.py $ARGS > gpurun_out/libab.json 2> gpurun_out/libab.err || { tail -5 gpurun_out/libab.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/libab.json'));print('${CFG:-c2}','${v:-tree}',d['value'],d['ms_per_step'])"
  done
done
