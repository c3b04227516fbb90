#!/bin/bash
# r06ab (r06u again, with the device-scope slot events): the stream's normals written in the matcher tree's order by k_normals_from_ids (inverse
# permutation on r3 behind the matcher tree) instead of k_inv_perm + k_scatter_normals on the raw
# chain. Stream / parity tests, per-window device times, C2 alternating against the commit before.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_sequence.py tests/test_gpu_parity.py > gpurun_out/r06ab_tests.log 2>&1 || { tail -30 gpurun_out/r06ab_tests.log; exit 1; }
echo "in-tree $(tail -1 gpurun_out/r06ab_tests.log)"
for v in "" ablib/lib_prev.so; do
  AICP_HIP_LIB=$v timeout -k 10 120 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-batched --opt profile=1 > gpurun_out/r06ab_prof.json 2> gpurun_out/r06ab_prof.err || exit 1
  echo "${v:-tree} $(grep 'device ms/window' gpurun_out/r06ab_prof.err | tail -1)"
done
STEPS=4 bash tools/lib_ab.sh 5 ablib/lib_prev.so
