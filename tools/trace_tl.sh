#!/bin/bash
# Kernel trace of a short bench run + the last run's timeline: bash tools/trace_tl.sh NAME [bench args]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
N=${1:-tl}; shift
rm -rf gpurun_out/$N && mkdir -p gpurun_out/$N
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/$N/trace -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline "$@" > gpurun_out/$N/bench.log 2>&1 || { tail -20 gpurun_out/$N/bench.log; exit 1; }
python3 tools/timeline.py $(find gpurun_out/$N/trace -name "*kernel_trace.csv" | head -1) > gpurun_out/$N/timeline.txt
head -1 gpurun_out/$N/timeline.txt
