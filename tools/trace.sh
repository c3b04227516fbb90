#!/bin/bash
# quick kernel trace of the bench: bash tools/trace.sh NAME STEPS
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
N=${1:-t}; S=${2:-2}
rm -rf gpurun_out/$N && mkdir -p gpurun_out/$N
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$N -o run -- python3 bench.py --steps $S --warmup 1 --no-cpu-baseline > gpurun_out/$N/bench.log 2>&1 || { tail -20 gpurun_out/$N/bench.log; exit 1; }
grep '^{' gpurun_out/$N/bench.log | cut -c1-400
python3 tools/kstats.py $(find gpurun_out/$N -name "*kernel_stats.csv" | head -1) $((S + 1))
