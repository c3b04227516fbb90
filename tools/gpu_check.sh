# GPU suite (TESTS=0 skips it), then N alternating C2 bench runs (--opt profile=1 phase times) of the
# in-tree library and each library given: bash tools/gpu_check.sh N [path/to/lib.so ...]
# Steps are chained so that a failure stops the call.
cd $GRAFT_REPO_ROOT
N=${1:-3}
shift
if [ "${TESTS:-1}" != 0 ]; then
  timeout -k 10 600 python3 -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/gpu_t.log 2>&1; rc=$?
  tail -2 gpurun_out/gpu_t.log; [ $rc -eq 0 ] || exit $rc
fi
for i in $(seq $N); do
  for v in "" "$@"; do
    AICP_HIP_LIB=$v timeout -k 10 200 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-batched --opt profile=1 > gpurun_out/b.log 2>&1 || exit 1
    echo "${v:-tree} $(grep -o '"value": [0-9.]*' gpurun_out/b.log | head -1) $(grep "device ms" gpurun_out/b.log | tail -1)"
  done
done
