#!/bin/bash
# r06s: the reference build's enqueue order. In-tree: the raw tree's first kernels before the
# matcher tree's graph (and no counter fill ahead of the octet kNN); rawall: the whole raw chain
# before the graph; prev: the commit before. Stream parity, per-window device times, C2 alternating.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_sequence.py tests/test_gpu_parity.py > gpurun_out/r06s_tests.log 2>&1 || { tail -30 gpurun_out/r06s_tests.log; exit 1; }
echo "in-tree $(tail -1 gpurun_out/r06s_tests.log)"
AICP_HIP_LIB=ablib/lib_rawall.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_sequence.py > gpurun_out/r06s_tests2.log 2>&1 || { tail -30 gpurun_out/r06s_tests2.log; exit 1; }
echo "rawall $(tail -1 gpurun_out/r06s_tests2.log)"
for v in "" ablib/lib_rawall.so ablib/lib_prev.so; do
  AICP_HIP_LIB=$v timeout -k 10 120 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-batched --opt profile=1 > gpurun_out/r06s_prof.json 2> gpurun_out/r06s_prof.err || exit 1
  echo "${v:-tree} $(grep 'device ms/window' gpurun_out/r06s_prof.err | tail -1)"
done
STEPS=4 bash tools/lib_ab.sh 4 ablib/lib_rawall.so ablib/lib_prev.so
