set -o pipefail
for i in 1 2 3; do
for v in "" ablib/libaicp_poll0.so; do
  AICP_HIP_LIB=$v timeout -k 10 200 python bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-batched > gpurun_out/nnev.json 2> gpurun_out/nnev.err || { tail -5 gpurun_out/nnev.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/nnev.json'));print('${v:-tree}', d['value'], d['roofline']['avg_launch_us'], d['roofline']['launches'])"
done; done
