#!/bin/bash
# r06v: persistent NN / kNN waves steal chunks from other XCD groups once their own group is
# exhausted (AICP_NN_STEAL). Parity tests, C2 and C5 kernel stats for both, C2 / C5 alternating
# against the commit before (ablib/lib_prev.so).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_sequence.py tests/test_configs.py > gpurun_out/r06v_tests.log 2>&1 || { tail -30 gpurun_out/r06v_tests.log; exit 1; }
echo "in-tree $(tail -1 gpurun_out/r06v_tests.log)"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for c in c2 c5; do
  for v in "" ablib/lib_prev.so; do
    d=gpurun_out/r06v_${c}${v:+_prev}
    AICP_HIP_LIB=$v timeout -k 10 170 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- python3 bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline $([ $c = c2 ] && echo --no-batched) > $d.json 2> gpurun_out/r06v.err || { tail -20 gpurun_out/r06v.err; exit 1; }
    echo "$c ${v:-tree} $(python3 -c "import json;print(json.load(open('$d.json'))['value'])") $(python3 tools/kstats_short.py $d/run_kernel_stats.csv 40 | grep -E 'k_icp_nn|k_knn_ids')"
  done
done
STEPS=4 bash tools/lib_ab.sh 4 ablib/lib_prev.so || exit 1
CFG=c5 STEPS=3 bash tools/lib_ab.sh 2 ablib/lib_prev.so
