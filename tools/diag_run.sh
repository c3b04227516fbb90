#!/bin/bash
# Diagnostic builds (tools/variants.sh xcd "-DAICP_DIAG=1 -DAICP_XCD_PROF=1" prof "-DAICP_DIAG=1 -DAICP_NN_PROF=1"): a short
# bench per build, stderr kept (per-XCD-group NN launch spans / per-phase NN wave cycles).
set -o pipefail
mkdir -p gpurun_out
for v in "$@"; do
  AICP_HIP_LIB=$PWD/build_ab/lib_$v.so timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --opt profile=1 > gpurun_out/diag_$v.out 2> gpurun_out/diag_$v.err || { tail -20 gpurun_out/diag_$v.err; exit 1; }
  tail -25 gpurun_out/diag_$v.err
done
