#!/bin/bash
# k_ovl_mark A/B: overlap + sequence GPU tests, then rocprofv3 kernel averages of k_ovl_mark on C2
# and C5 for the in-tree library and build_var/lib_head.so
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python3 -u -m pytest tests -x -q -m gpu -k "ovl or overlap or sequence or stream or config" --timeout 120 --timeout-method thread > gpurun_out/mark_t.log 2>&1 || { tail -20 gpurun_out/mark_t.log; exit 1; }
tail -1 gpurun_out/mark_t.log
bash tools/lib_kstats.sh "ovl_mark" build_var/lib_mark1024.so build_var/lib_head.so || exit 1
for lib in default build_var/lib_mark1024.so build_var/lib_head.so; do
  if [ "$lib" = default ]; then unset AICP_HIP_LIB; else export AICP_HIP_LIB=$PWD/$lib; fi
  rm -rf gpurun_out/mk5_$(basename $lib .so)
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/mk5_$(basename $lib .so) -o run -- python3 bench.py --config c5 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/mk5.log 2>&1 || { tail -5 gpurun_out/mk5.log; exit 1; }
  echo "== c5 $lib $(grep -o '"value": [0-9.]*' gpurun_out/mk5.log | head -1)"; python3 tools/kstats_short.py $(find gpurun_out/mk5_$(basename $lib .so) -name "*kernel_stats.csv" | head -1) 60 | grep -E "ovl_mark|total"
done
