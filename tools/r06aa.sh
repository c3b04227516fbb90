#!/bin/bash
# r06aa: the stream's raw build's point-independent kernels (state, zero, frames) before the
# reference wait. Stream parity, per-window device times,
# a C2 kernel trace for the cross-queue gaps, C2 alternating against the commit before.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_sequence.py tests/test_gpu_parity.py > gpurun_out/r06aa_tests.log 2>&1 || { tail -30 gpurun_out/r06aa_tests.log; exit 1; }
echo "in-tree $(tail -1 gpurun_out/r06aa_tests.log)"
for v in "" ablib/lib_prev.so; do
  AICP_HIP_LIB=$v timeout -k 10 120 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-batched --opt profile=1 > gpurun_out/r06aa_prof.json 2> gpurun_out/r06aa_prof.err || exit 1
  echo "${v:-tree} $(grep 'device ms/window' gpurun_out/r06aa_prof.err | tail -1)"
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 170 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06aa_k -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-batched > gpurun_out/r06aa_k.json 2> gpurun_out/r06aa.err || { tail -20 gpurun_out/r06aa.err; exit 1; }
STEPS=4 bash tools/lib_ab.sh 4 ablib/lib_prev.so
