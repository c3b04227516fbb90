#!/bin/bash
# r06i: packed FP32 bucket distances in the NN. NN / ICP / sequence parity tests, C2 kernel stats,
# then C2 alternating against the previous library (ablib/libaicp_prev.so).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_sequence.py tests/test_configs.py > gpurun_out/r06i_tests.log 2>&1 || { tail -30 gpurun_out/r06i_tests.log; exit 1; }
tail -1 gpurun_out/r06i_tests.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 170 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06i_k -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-batched > gpurun_out/r06i_k.log 2>&1 || { tail -20 gpurun_out/r06i_k.log; exit 1; }
python3 tools/kstats_short.py gpurun_out/r06i_k/run_kernel_stats.csv 3
STEPS=4 bash tools/lib_ab.sh 4 ablib/libaicp_prev.so
