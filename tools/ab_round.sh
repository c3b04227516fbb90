#!/bin/bash
# GPU side, one call: the -m gpu suite on the in-tree library, then C2 (and optionally C5)
# alternating A/B against prebuilt libraries, then a C2 kernel-stats pass of the in-tree build.
#   bash tools/ab_round.sh TAG "lib..." [c5]
set -o pipefail
TAG=${1:-ab}; LIBS=$2; C5=$3
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1 || { tail -40 gpurun_out/tests_$TAG.log; exit 1; }
tail -2 gpurun_out/tests_$TAG.log
STEPS=3 bash tools/lib_ab.sh 3 $LIBS || exit 1
if [ -n "$C5" ]; then CFG=c5 STEPS=2 bash tools/lib_ab.sh 2 $LIBS || exit 1; fi
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/kstat_$TAG
rm -rf $OUT && mkdir -p $OUT
timeout -k 10 170 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-batched > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
python3 tools/kstats_short.py $(find $OUT/trace -name "*kernel_stats.csv" | head -1) 25
