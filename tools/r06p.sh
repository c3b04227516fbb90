#!/bin/bash
# r06p: k_tr_mid with 512 / 256 threads per workgroup against 1024 (head): tree / stream parity of
# each, rocprofv3 kernel stats of C2, then C2 alternating
set -o pipefail
mkdir -p gpurun_out
for v in mid512 mid256; do
  AICP_HIP_LIB=ablib/lib_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_sequence.py > gpurun_out/r06p_tests.log 2>&1 || { tail -30 gpurun_out/r06p_tests.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/r06p_tests.log)"
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in libaicp_head lib_mid512 lib_mid256; do
  d=gpurun_out/r06p_$v
  AICP_HIP_LIB=ablib/$v.so timeout -k 10 170 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-batched > $d.json 2> gpurun_out/r06p.err || { tail -20 gpurun_out/r06p.err; exit 1; }
  echo "$v $(python3 -c "import json;print(json.load(open('$d.json'))['value'])")"; python3 tools/kstats_short.py $d/run_kernel_stats.csv 40 | grep -E 'k_tr_mid|subtree_blk|k_icp_nn'
done
STEPS=4 bash tools/lib_ab.sh 3 ablib/lib_mid512.so ablib/lib_mid256.so
