#!/bin/bash
# C5 SurfaceNormal kNN: the per-lane engine (default above 300k queries) against the octet engine
# (--opt normals_knn_engine=1): kernel time by rocprofv3 --stats, then VALU instructions, waves and busy
# cycles per kNN dispatch in one counter pass each. Output under gpurun_out/knn_c5/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/knn_c5
rm -rf $OUT && mkdir -p $OUT
for v in 0 1; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/t$v -o run -- python3 bench.py --config c5 --steps 1 --warmup 0 --no-cpu-baseline --opt normals_knn_engine=$v > $OUT/t$v.log 2>&1 || { tail -20 $OUT/t$v.log; exit 1; }
  echo "oct=$v $(grep -o '"value": [0-9.]*' $OUT/t$v.log | head -1)"
  python3 tools/kstats_short.py $(find $OUT/t$v -name "*kernel_stats.csv" | head -1) 12
  timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VMEM --kernel-include-regex "k_knn" --output-format csv -d $OUT/p$v -o run -- python3 bench.py --config c5 --steps 1 --warmup 0 --no-cpu-baseline --opt normals_knn_engine=$v > $OUT/p$v.log 2>&1 || { tail -20 $OUT/p$v.log; exit 1; }
done
