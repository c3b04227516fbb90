#!/bin/bash
# rocprofv3 kernel averages of one bench config (CFG, default C2) per library build (default lib = "default"):
# bash tools/lib_kstats.sh REGEX path/to/a.so ...
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
RX=$1; shift
for lib in default "$@"; do
  tag=$(basename $lib .so)
  if [ "$lib" = default ]; then unset AICP_HIP_LIB; else export AICP_HIP_LIB=$PWD/$lib; fi
  rm -rf gpurun_out/lk_$tag
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/lk_$tag -o run -- python3 bench.py ${CFG:+--config $CFG} --steps ${STEPS:-5} --warmup 1 --no-cpu-baseline --no-batched > gpurun_out/lk_$tag.log 2>&1 || { tail -5 gpurun_out/lk_$tag.log; exit 1; }
  echo "== $tag"; python3 tools/kstats_short.py $(find gpurun_out/lk_$tag -name "*kernel_stats.csv" | head -1) 60 | grep -E "$RX|total"
done
unset AICP_HIP_LIB
