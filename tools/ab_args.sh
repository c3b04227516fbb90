#!/bin/bash
# Alternating A/B of bench.py argument sets on C2 (--opt profile=1 phase lines kept), R rounds:
# bash tools/ab_args.sh R "" "--ref-normals"
set -o pipefail
mkdir -p gpurun_out
R=$1; shift
for r in $(seq 1 $R); do
  i=0
  for a in "$@"; do
    i=$((i+1))
    timeout -k 10 200 python bench.py --steps 8 --warmup 3 --no-cpu-baseline --no-batched --opt profile=1 $a > gpurun_out/aba_$i.json 2> gpurun_out/aba_$i.err || { tail -20 gpurun_out/aba_$i.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/aba_$i.json'));print('[$a]',d['value'],d['ms_per_step'],d['roofline']['avg_launch_us'])"
    grep 'device ms/window' gpurun_out/aba_$i.err | tail -1
  done
done
