set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tests_r06d.log 2>&1 || { tail -40 gpurun_out/tests_r06d.log; exit 1; }
tail -2 gpurun_out/tests_r06d.log
STEPS=4 bash tools/lib_ab.sh 3 $PWD/build_ab/lib_h8.so || exit 1
timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-batched --opt profile=1 > gpurun_out/seqprof_r06d.json 2> gpurun_out/seqprof_r06d.err || { tail -20 gpurun_out/seqprof_r06d.err; exit 1; }
grep "aicp seq" gpurun_out/seqprof_r06d.err | tail -8
