#!/bin/bash
# r06w: idle-only cross-group stealing. In-tree: the persistent normals kNN steals; nnsteal: the
# ICP NN too; prev: neither (the commit before). Parity, kernel stats (C2, C5), alternating runs.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_sequence.py tests/test_configs.py > gpurun_out/r06w_tests.log 2>&1 || { tail -30 gpurun_out/r06w_tests.log; exit 1; }
echo "in-tree $(tail -1 gpurun_out/r06w_tests.log)"
AICP_HIP_LIB=ablib/lib_nnsteal.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_configs.py > gpurun_out/r06w_tests2.log 2>&1 || { tail -30 gpurun_out/r06w_tests2.log; exit 1; }
echo "nnsteal $(tail -1 gpurun_out/r06w_tests2.log)"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for c in c2 c5; do
  for v in "" ablib/lib_nnsteal.so ablib/lib_prev.so; do
    d=gpurun_out/r06w_${c}_$(basename ${v:-tree} .so)
    AICP_HIP_LIB=$v timeout -k 10 170 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- python3 bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline $([ $c = c2 ] && echo --no-batched) > $d.json 2> gpurun_out/r06w.err || { tail -20 gpurun_out/r06w.err; exit 1; }
    echo "$c ${v:-tree} $(python3 -c "import json;print(json.load(open('$d.json'))['value'])") $(python3 tools/kstats_short.py $d/run_kernel_stats.csv 40 | grep -E 'k_icp_nn|k_knn_ids')"
  done
done
STEPS=4 bash tools/lib_ab.sh 3 ablib/lib_nnsteal.so ablib/lib_prev.so || exit 1
for c in c5 c4 c3; do CFG=$c STEPS=3 bash tools/lib_ab.sh 2 ablib/lib_nnsteal.so ablib/lib_prev.so || exit 1; done
