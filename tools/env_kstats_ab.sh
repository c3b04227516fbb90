#!/bin/bash
# A/B of an environment switch: per value, a rocprofv3 kernel-stats pass of `bench.py --config
# CFG` (kernels matching REGEX) and the bench value of CFG and of C2.
# Usage: bash tools/env_kstats_ab.sh NAME VAR "v1 v2" CFG REGEX
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
N=$1; VAR=$2; VALS=$3; CFG=${4:-c5}; RX=${5:-k_tr}
rm -rf gpurun_out/$N && mkdir -p gpurun_out/$N
for v in $VALS; do
  export $VAR=$v
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$N/t$v -o run -- python3 bench.py --config $CFG --steps 2 --warmup 1 --no-cpu-baseline --no-batched > gpurun_out/$N/t$v.log 2>&1 || { tail -5 gpurun_out/$N/t$v.log; exit 1; }
  python3 tools/kstats_short.py $(find gpurun_out/$N/t$v -name "*kernel_stats.csv" | head -1) 60 | grep -E "$RX|total"
  timeout -k 10 200 python3 bench.py --config $CFG --steps 3 --warmup 1 --no-cpu-baseline --no-batched > gpurun_out/$N/b_$v.json 2> gpurun_out/$N/b_$v.err || exit 1
  timeout -k 10 200 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-batched > gpurun_out/$N/c2_$v.json 2> gpurun_out/$N/c2_$v.err || exit 1
  python3 -c "import json; a=json.load(open('gpurun_out/$N/b_$v.json')); b=json.load(open('gpurun_out/$N/c2_$v.json')); print('$VAR=$v $CFG', a['value'], 'c2', b['value'])"
done
