set -o pipefail
for v in "AICP_READ_ORDER_MIN=0" "AICP_READ_ORDER_MIN=200000" "AICP_READ_ORDER_MIN=0" "AICP_READ_ORDER_MIN=200000"; do
  env $v timeout -k 10 300 python bench.py --config app --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/app.json 2> gpurun_out/app.err || { tail -5 gpurun_out/app.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/app.json'));print('$v',d['value'],d['reading_ms_reference_reused'],d['reading_ms_reference_built'],d['reused_split_ms'])"
done
