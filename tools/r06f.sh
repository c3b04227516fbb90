# C2: the reference-side marks' workgroup cap (option ref_mark_blocks), alternating, with phase lines
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  for v in 0 64 128 256; do
    timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-batched --opt profile=1 --opt ref_mark_blocks=$v > gpurun_out/rmb_$v.json 2> gpurun_out/rmb_$v.err || { tail -20 gpurun_out/rmb_$v.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/rmb_$v.json'));print('ref_mark_blocks $v', d['value'], d['ms_per_step'])"
    grep "device ms/window" gpurun_out/rmb_$v.err | tail -1
  done
done
