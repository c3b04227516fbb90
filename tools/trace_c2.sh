#!/bin/bash
# rocprofv3 kernel trace of the default C2 stream (no batched leg, no CPU leg) for timelines
# (tools/timeline.py) and per-kernel stats; output under gpurun_out/trace_$1.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
R=${1:-x}
shift
OUT=gpurun_out/trace_$R
rm -rf $OUT && mkdir -p $OUT
timeout -k 10 170 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-batched "$@" > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log | cut -c1-400
python3 tools/kstats_short.py $(find $OUT -name "*kernel_stats.csv" | head -1) 25
