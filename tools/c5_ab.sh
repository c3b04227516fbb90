#!/bin/bash
# C5 (or AB_CONFIG) bench line under env variants: bash tools/c5_ab.sh "VAR=x ..." ...
set -o pipefail
mkdir -p gpurun_out
for v in "$@"; do
  env $v timeout -k 10 200 python -u bench.py --config ${AB_CONFIG:-c5} --steps ${AB_STEPS:-2} --warmup 1 --no-cpu-baseline > gpurun_out/c5ab.json 2> gpurun_out/c5ab.err || { tail -20 gpurun_out/c5ab.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/c5ab.json')); print('$v', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'])"
done
