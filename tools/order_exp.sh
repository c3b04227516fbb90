set -o pipefail
mkdir -p gpurun_out
for o in raster morton shuffle; do
  if [ $o = raster ]; then unset AICP_BENCH_READ_ORDER; else export AICP_BENCH_READ_ORDER=$o; fi
  timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/order_$o.log 2>&1 || { tail -20 gpurun_out/order_$o.log; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/order_$o.log').read().strip().splitlines()[-1]);print('$o',d['value'],d['roofline']['avg_launch_us'],d['phase_ms_per_step'],d['mean_iterations'])"
done
