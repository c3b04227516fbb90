#!/bin/bash
# rocprofv3 kernel trace + stats of the C2 stream (tools/seqtime.py); results under gpurun_out/prof_$1
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
R=${1:-r03}
OUT=gpurun_out/prof_$R
rm -rf $OUT && mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 tools/seqtime.py > $OUT/seq_trace.log 2>&1 || { tail -20 $OUT/seq_trace.log; exit 1; }
tail -2 $OUT/seq_trace.log
