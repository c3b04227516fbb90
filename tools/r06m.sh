#!/bin/bash
# r06m: the NN's LDS far frames through an LDS-space pointer (ds_ ops for them, scratch_ ops for the
# deeper frames, no flat ops). NN / stream parity, rocprofv3 kernel stats of C2 for the in-tree and
# the HEAD library, then C2 and C5 alternating.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_sequence.py > gpurun_out/r06m_tests.log 2>&1 || { tail -30 gpurun_out/r06m_tests.log; exit 1; }
tail -1 gpurun_out/r06m_tests.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in "" ablib/libaicp_head.so; do
  AICP_HIP_LIB=$v timeout -k 10 170 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06m_k${v:+p} -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-batched > gpurun_out/r06m_k.log 2>&1 || { tail -20 gpurun_out/r06m_k.log; exit 1; }
  python3 tools/kstats_short.py gpurun_out/r06m_k${v:+p}/run_kernel_stats.csv 12 | grep -E "k_knn|k_icp_nn|normals"
done
STEPS=4 bash tools/lib_ab.sh 3 ablib/libaicp_head.so || exit 1
CFG=c5 STEPS=3 bash tools/lib_ab.sh 2 ablib/libaicp_head.so
