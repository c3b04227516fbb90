#!/bin/bash
# A/B of prebuilt variants (tools/variants.sh) on the C2 bench, then the GPU parity suite on the
# last variant named. Each step bounded; stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
bash tools/run_variants.sh "$@" || exit 1
last="${@: -1}"
AICP_HIP_LIB=$PWD/build_ab/lib_$last.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/parity_$last.log 2>&1 || { tail -40 gpurun_out/parity_$last.log; exit 1; }
tail -3 gpurun_out/parity_$last.log
