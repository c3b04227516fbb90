#!/bin/bash
# GPU side: per-kernel average durations (rocprofv3 --kernel-trace --stats) of the C2 stream for
# prebuilt variants (tools/variants.sh): bash tools/kstat_ab.sh NAME... Prints the ICP loop's
# kernels; the full tables stay under gpurun_out/kab_NAME/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in "$@"; do
  OUT=gpurun_out/kab_$v
  rm -rf $OUT && mkdir -p $OUT
  AICP_HIP_LIB=$PWD/build_ab/lib_$v.so timeout -k 10 170 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-batched > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
  echo "== $v"
  python3 - "$(find $OUT/trace -name '*kernel_stats.csv' | head -1)" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"]
    if any(k in n for k in ("k_icp_nn", "k_sel_", "k_icp_reduce", "k_icp_update", "k_knn_oct", "k_tr_mid", "k_ovl_mark")):
        print("%-28s %6s %9.2f us" % (n.split("(")[0][-28:], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
done
