#!/bin/bash
# r06j: the next reference started once its source reading stopped (early_reference). The GPU
# suite, a C2 kernel trace, then C2 alternating against the previous library and option 0.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/r06j_tests.log 2>&1 || { tail -40 gpurun_out/r06j_tests.log; exit 1; }
tail -1 gpurun_out/r06j_tests.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 170 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06j_k -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-batched > gpurun_out/r06j_k.log 2>&1 || { tail -20 gpurun_out/r06j_k.log; exit 1; }
python3 tools/kstats_short.py gpurun_out/r06j_k/run_kernel_stats.csv 4
timeout -k 10 120 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-batched --opt profile=1 > gpurun_out/r06j_prof.json 2> gpurun_out/r06j_prof.err || exit 1
grep "device ms/window\|hand-off" gpurun_out/r06j_prof.err | tail -2
STEPS=4 bash tools/lib_ab.sh 3 ablib/libaicp_prev.so
CFG=c2 STEPS=4 bash tools/opt_ab.sh 2 "early_reference=1" "early_reference=0"
