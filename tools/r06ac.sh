#!/bin/bash
# r06ac: same-box rocprofv3 NN kernel time of the last build against the one before the
# matcher-order normals (r06fin3's profile read 76 us per NN launch, r06fin2's 70 us)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for r in 1 2; do
  for v in "" ablib/lib_prev.so; do
    d=gpurun_out/r06ac_$(basename ${v:-tree} .so)_$r
    AICP_HIP_LIB=$v timeout -k 10 170 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-batched > $d.json 2> gpurun_out/r06ac.err || { tail -20 gpurun_out/r06ac.err; exit 1; }
    echo "${v:-tree} $r $(python3 -c "import json;print(json.load(open('$d.json'))['value'])") $(python3 tools/kstats_short.py $d/run_kernel_stats.csv 40 | grep -E 'k_icp_nn|k_knn_oct')"
  done
done
