#!/bin/bash
# rocprofv3 evidence for the bench: kernel trace + stats, then FETCH_SIZE and WRITE_SIZE in
# separate counter passes (MI355X_MICROARCH.md: they do not fit one pass). Results are copied
# into profiles/ by the caller.
# Counter passes serialise kernel dispatch, and the stream's device-side window dependency
# (hipStreamWaitValue64 on a ticket a later kernel writes) cannot complete under serialisation:
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
R=${1:-r01}
CFG=${2:-c2}
OUT=gpurun_out/prof_$R
rm -rf $OUT && mkdir -p $OUT
timeout -k 10 170 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py --config $CFG --steps 5 --warmup 1 --no-cpu-baseline --no-batched > $OUT/bench_trace.log 2>&1 || { tail -20 $OUT/bench_trace.log; exit 1; }
tail -1 $OUT/bench_trace.log
timeout -k 10 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 bench.py --config $CFG --steps 2 --warmup 0 --no-cpu-baseline --no-batched > $OUT/fetch.log 2>&1 || { tail -20 $OUT/fetch.log; exit 1; }
timeout -k 10 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 bench.py --config $CFG --steps 2 --warmup 0 --no-cpu-baseline --no-batched > $OUT/write.log 2>&1 || { tail -20 $OUT/write.log; exit 1; }
python3 tools/pmc_summary.py $OUT/nn_traffic.json $OUT/fetch $OUT/write k_icp_nn
python3 tools/kstats_short.py $(find $OUT/trace -name "*kernel_stats.csv" | head -1) 30
