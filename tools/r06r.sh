#!/bin/bash
# r06r: the small-build tree finishers: k_tr_mid on 512 threads (mid512), k_tr_subtree_blk on 16
# waves (sw16), both (m512sw16), against head. Tree / stream parity, C2 kernel stats, C2
# alternating, then C3 / C4 / C5 once each.
set -o pipefail
mkdir -p gpurun_out
for v in sw16 m512sw16; do
  AICP_HIP_LIB=ablib/lib_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_sequence.py > gpurun_out/r06r_tests.log 2>&1 || { tail -30 gpurun_out/r06r_tests.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/r06r_tests.log)"
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in libaicp_head lib_m512sw16; do
  d=gpurun_out/r06r_$v
  AICP_HIP_LIB=ablib/$v.so timeout -k 10 170 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-batched > $d.json 2> gpurun_out/r06r.err || { tail -20 gpurun_out/r06r.err; exit 1; }
  echo "$v $(python3 -c "import json;print(json.load(open('$d.json'))['value'])")"; python3 tools/kstats_short.py $d/run_kernel_stats.csv 40 | grep -E 'k_tr_mid|subtree_blk|k_icp_nn'
done
STEPS=4 bash tools/lib_ab.sh 3 ablib/lib_mid512.so ablib/lib_sw16.so ablib/lib_m512sw16.so || exit 1
for c in c5 c3 c4; do CFG=$c STEPS=2 bash tools/lib_ab.sh 1 ablib/lib_m512sw16.so || exit 1; done
