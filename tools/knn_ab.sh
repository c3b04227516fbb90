#!/bin/bash
# GPU side: parity suite, then the treelet kNN engine A/B on C2 and on the pre-filter bench
set -o pipefail
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 180 --timeout-method thread > gpurun_out/knn_tests.log 2>&1 || { tail -30 gpurun_out/knn_tests.log; exit 1; }
tail -2 gpurun_out/knn_tests.log
bash tools/run_env_ab.sh "tl:" "nodes:AICP_KNN_TREELETS=0" "tl2:" "nodes2:AICP_KNN_TREELETS=0" || exit 1
for spec in "tl:" "nodes:AICP_KNN_TREELETS=0"; do
  name=${spec%%:*}; envs=${spec#*:}
  env $envs timeout -k 10 300 python bench.py --config prefilter --steps 8 --warmup 2 --no-cpu-baseline > gpurun_out/pfab_$name.log 2>&1 || exit 1
  python3 -c "import json;d=json.loads([l for l in open('gpurun_out/pfab_$name.log') if l.startswith('{')][-1]);print('prefilter $name',d['value'],d['phase_ms_per_cloud'],d['roofline']['avg_launch_us'])"
done
