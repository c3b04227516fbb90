#!/bin/bash
# r06n: NN far-frame access variants, rocprofv3 kernel stats on C2 and C5, alternating:
# head (generic pointer: merged flat push and pop), as3 (ds_ / scratch_ push and pop),
# pushsplit (ds_ / scratch_ push, merged flat pop). NN parity of the two variants first.
set -o pipefail
mkdir -p gpurun_out
for v in ablib/libaicp_as3.so ablib/libaicp_pushsplit.so; do
  AICP_HIP_LIB=$v timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py > gpurun_out/r06n_tests.log 2>&1 || { tail -30 gpurun_out/r06n_tests.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/r06n_tests.log)"
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for r in 1 2; do
  for c in c2 c5; do
    for v in head as3 pushsplit; do
      d=gpurun_out/r06n_${c}_${v}_$r
      AICP_HIP_LIB=ablib/libaicp_$v.so timeout -k 10 170 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- python3 bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline $([ $c = c2 ] && echo --no-batched) > $d.json 2> gpurun_out/r06n.err || { tail -20 gpurun_out/r06n.err; exit 1; }
      echo "$c $v $r $(python3 -c "import json;print(json.load(open('$d.json'))['value'])") $(python3 tools/kstats_short.py $d/run_kernel_stats.csv 12 | grep -E 'k_icp_nn')"
    done
  done
done
