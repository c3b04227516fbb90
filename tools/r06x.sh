#!/bin/bash
# r06x: the subtree builders' segment size kSubMax 2048 / 512 against 1024 (in-tree). Tree /
# stream / config parity of each, C2 kernel stats, C2 alternating, C5 / C3 / C4 once each.
set -o pipefail
mkdir -p gpurun_out
for v in sub2048 sub512; do
  AICP_HIP_LIB=ablib/lib_$v.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_sequence.py tests/test_configs.py > gpurun_out/r06x_tests.log 2>&1 || { tail -30 gpurun_out/r06x_tests.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/r06x_tests.log)"
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in "" ablib/lib_sub2048.so ablib/lib_sub512.so; do
  d=gpurun_out/r06x_$(basename ${v:-tree} .so)
  AICP_HIP_LIB=$v timeout -k 10 170 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-batched > $d.json 2> gpurun_out/r06x.err || { tail -20 gpurun_out/r06x.err; exit 1; }
  echo "${v:-tree} $(python3 -c "import json;print(json.load(open('$d.json'))['value'])")"; python3 tools/kstats_short.py $d/run_kernel_stats.csv 60 | grep -E 'k_tr_mid|subtree|k_tr_scan1|k_tr_move1'
done
STEPS=4 bash tools/lib_ab.sh 3 ablib/lib_sub2048.so ablib/lib_sub512.so || exit 1
for c in c5 c3 c4; do CFG=$c STEPS=2 bash tools/lib_ab.sh 1 ablib/lib_sub2048.so ablib/lib_sub512.so || exit 1; done
