#!/bin/bash
# End-to-end GPU evidence for one build: parity tests, smoke, the default bench line (with the
# CPU baseline), then the rocprofv3 kernel-trace + PMC passes of tools/profile.sh. Each step is
# bounded and the script stops at the first failure.
set -o pipefail
R=${1:-r02d}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/parity_$R.log 2>&1 || { tail -40 gpurun_out/parity_$R.log; exit 1; }
tail -3 gpurun_out/parity_$R.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$R.log 2>&1 || { tail -30 gpurun_out/smoke_$R.log; exit 1; }
tail -1 gpurun_out/smoke_$R.log
timeout -k 10 300 python bench.py > gpurun_out/bench_$R.json 2> gpurun_out/bench_$R.err || { tail -30 gpurun_out/bench_$R.err; exit 1; }
cat gpurun_out/bench_$R.json
bash tools/profile.sh $R
