#!/bin/bash
# r06g: the octet kNN on treelet records. GPU tests of the kNN / pre-filter / stream callers,
# then rocprofv3 kernel stats of C2 with the default (treelets) and option normals_knn_engine=3
# (node records), then alternating C2 bench lines of both.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_prefilter.py tests/test_sequence.py > gpurun_out/r06g_tests.log 2>&1 || { tail -40 gpurun_out/r06g_tests.log; exit 1; }
tail -2 gpurun_out/r06g_tests.log
for e in 0 3; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06g_k$e -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-batched --opt normals_knn_engine=$e > gpurun_out/r06g_k$e.log 2>&1 || { tail -20 gpurun_out/r06g_k$e.log; exit 1; }
  python3 tools/kstats_short.py gpurun_out/r06g_k$e/run_kernel_stats.csv | grep -E "k_knn|k_icp_nn|k_tl_|k_tr_mid" || true
done
CFG=c2 bash tools/opt_ab.sh 3 "normals_knn_engine=0" "normals_knn_engine=3"
