#!/bin/bash
# Device phase times of the C2 stream (--opt profile=1 prints host ms per part and device ms per
# window phase on stderr), then the same with the early window ticket / graphs toggled by env.
set -o pipefail
mkdir -p gpurun_out
for v in "$@"; do
  echo "== $v"
  timeout -k 10 120 python bench.py --steps ${SEQPROF_STEPS:-5} --warmup 2 --no-cpu-baseline --no-batched --opt profile=1 $v > gpurun_out/seqprof.json 2> gpurun_out/seqprof.err || { tail -20 gpurun_out/seqprof.err; exit 1; }
  grep 'aicp seq' gpurun_out/seqprof.err | tail -2
  python -c "import json; d=json.load(open('gpurun_out/seqprof.json')); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['mean_iterations'])"
done
