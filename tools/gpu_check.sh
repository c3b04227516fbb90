#!/bin/bash
# GPU round-trip: parity tests, smoke, short bench. Each step bounded; stop at first failure.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/parity.log 2>&1 || { tail -40 gpurun_out/parity.log; exit 1; }
tail -3 gpurun_out/parity.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -30 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench.log 2>&1 || { tail -30 gpurun_out/bench.log; exit 1; }
cat gpurun_out/bench.log
