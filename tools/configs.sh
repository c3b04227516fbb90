#!/bin/bash
# C3 / C4 / C5 / single / app bench lines on the current build, each with its bounded cpu_baseline and
# parity_vs_oracle (+ a C5 rocprofv3 trace and PMC traffic pass); each step bounded; output under
# gpurun_out/. Usage: tools/configs.sh <round tag, e.g. r04>
set -o pipefail
mkdir -p gpurun_out
R=${1:-r04}
for c in c3 c4; do
  timeout -k 10 400 python -u bench.py --config $c --steps 3 --warmup 1 --cpu-reps 3 --no-batched > gpurun_out/${R}_$c.json 2> gpurun_out/${R}_$c.err || { tail -20 gpurun_out/${R}_$c.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/${R}_$c.json')); print('$c', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['frac'], d.get('cpu_baseline',{}).get('value'), d.get('parity_vs_oracle'))"
done
timeout -k 10 300 python -u bench.py --config single --steps 20 --warmup 3 > gpurun_out/${R}_single.json 2> gpurun_out/${R}_single.err || { tail -20 gpurun_out/${R}_single.err; exit 1; }
python3 -c "import json,sys; d=json.load(open('gpurun_out/${R}_single.json')); print('single', d['value'], d.get('cpu_baseline',{}).get('value'), d.get('parity_vs_oracle'))"
timeout -k 10 300 python -u bench.py --config app --steps 3 --warmup 1 > gpurun_out/${R}_app.json 2> gpurun_out/${R}_app.err || { tail -20 gpurun_out/${R}_app.err; exit 1; }
python3 -c "import json,sys; d=json.load(open('gpurun_out/${R}_app.json')); print('app', d['value'], {k: d[k] for k in d if k.startswith('reading_ms') or k == 'parity_vs_oracle'})"
for m in debug robot; do
  timeout -k 10 400 python -u bench.py --config c2 --raw --working-mode $m --steps 2 --warmup 1 --cpu-reps 2 --no-batched > gpurun_out/${R}_raw_$m.json 2> gpurun_out/${R}_raw_$m.err || { tail -20 gpurun_out/${R}_raw_$m.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/${R}_raw_$m.json')); print('raw $m', d['value'], d['ms_per_step'], d.get('cpu_baseline',{}).get('value'), d.get('parity_vs_oracle'))"
done
timeout -k 10 400 python -u bench.py --config c5 --steps 3 --warmup 1 --cpu-budget 4 --cpu-reps 3 > gpurun_out/${R}_c5.json 2> gpurun_out/${R}_c5.err || { tail -20 gpurun_out/${R}_c5.err; exit 1; }
python3 -c "import json,sys; d=json.load(open('gpurun_out/${R}_c5.json')); print('c5', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['frac'], d.get('cpu_baseline',{}).get('value'), d.get('cpu_baseline_all_cores',{}).get('value'))"
bash tools/profile.sh ${R}_c5 c5
