#!/bin/bash
# r06z: the NN timing events (bench roofline) without the system-scope fence
# (hipEventDisableSystemFence) against the commit before: value and the events' NN time, alternating.
set -o pipefail
mkdir -p gpurun_out
for r in 1 2 3; do
  for v in "" ablib/lib_prev.so; do
    AICP_HIP_LIB=$v timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-batched > gpurun_out/r06z.json 2> gpurun_out/r06z.err || { tail -20 gpurun_out/r06z.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/r06z.json'));print('${v:-tree}', d['value'], d['roofline']['avg_launch_us'], d['roofline']['frac'])"
  done
done
for v in "" ablib/lib_prev.so; do
  AICP_HIP_LIB=$v timeout -k 10 300 python bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r06z5.json 2> gpurun_out/r06z5.err || { tail -20 gpurun_out/r06z5.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/r06z5.json'));print('c5 ${v:-tree}', d['value'], d['roofline']['avg_launch_us'], d['roofline']['frac'])"
done
# the batch path's stream-ordering events at device scope: single-pair latency and App's per-reading calls
for r in 1 2; do
  for v in "" ablib/lib_prev.so; do
    AICP_HIP_LIB=$v timeout -k 10 200 python bench.py --config single --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r06zs.json 2> gpurun_out/r06zs.err || { tail -20 gpurun_out/r06zs.err; exit 1; }
    AICP_HIP_LIB=$v timeout -k 10 200 python bench.py --config app --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r06za.json 2> gpurun_out/r06za.err || { tail -20 gpurun_out/r06za.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/r06zs.json'));a=json.load(open('gpurun_out/r06za.json'));print('single/app ${v:-tree}', d['value'], a['value'])"
  done
done
