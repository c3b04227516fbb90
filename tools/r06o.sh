#!/bin/bash
# r06o: the ITER_PROF diagnostic library on the C2 stream: k_tr_mid's per-segment phases and the
# ICP iteration kernels' bodies / tails ([tree prof] / [iter prof] lines on stderr)
set -o pipefail
mkdir -p gpurun_out
AICP_HIP_LIB=ablib/lib_iterprof.so timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-batched --opt profile=1 > gpurun_out/r06o.json 2> gpurun_out/r06o.err || { tail -20 gpurun_out/r06o.err; exit 1; }
grep -E "tree prof|iter prof|device ms" gpurun_out/r06o.err | tail -12
