#!/bin/bash
# GPU round-trip: parity tests, NN microbench, short bench. Each step bounded; stop at first failure.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -m pytest tests/test_gpu_parity.py -m gpu -x -q > gpurun_out/parity.log 2>&1 || { tail -30 gpurun_out/parity.log; exit 1; }
tail -3 gpurun_out/parity.log
python tools/mkpair.py /tmp/p 120000 1000 && timeout -k 10 120 ./tools/microbench /tmp/p_ref.bin /tmp/p_read.bin > gpurun_out/mb.log 2>&1 && AICP_NN_ENGINE=1 timeout -k 10 120 ./tools/microbench /tmp/p_ref.bin /tmp/p_read.bin >> gpurun_out/mb.log 2>&1 || { cat gpurun_out/mb.log; exit 1; }
cat gpurun_out/mb.log
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench.log 2>&1 || { tail -30 gpurun_out/bench.log; exit 1; }
cat gpurun_out/bench.log
AICP_NN_ENGINE=1 timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_e1.log 2>&1 || { tail -30 gpurun_out/bench_e1.log; exit 1; }
cat gpurun_out/bench_e1.log
AICP_NN_ENGINE=1 timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -m gpu -x -q > gpurun_out/parity_e1.log 2>&1 || { tail -30 gpurun_out/parity_e1.log; exit 1; }
tail -2 gpurun_out/parity_e1.log
