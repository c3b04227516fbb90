#!/bin/bash
# r06q: C4 and C3 kernel traces (rocprofv3) for their per-call timelines (tools/timeline_batch.py)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for c in c4 c3; do
  d=gpurun_out/r06q_$c
  timeout -k 10 170 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- python3 bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline > $d.json 2> gpurun_out/r06q.err || { tail -20 gpurun_out/r06q.err; exit 1; }
  echo "$c $(python3 -c "import json;d=json.load(open('$d.json'));print(d['value'], d['ms_per_step'])")"
  python3 tools/kstats_short.py $d/run_kernel_stats.csv 14
done
