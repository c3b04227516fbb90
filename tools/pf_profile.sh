#!/bin/bash
# GPU side: pre-filter parity tests, then rocprofv3 kernel stats of bench.py --config prefilter.
# Usage (via gpurun): bash tools/pf_profile.sh [tag]
set -o pipefail
T=${1:-pf}
timeout -k 10 400 python -u -m pytest tests/test_prefilter.py -q -m gpu --timeout 180 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1
tail -2 gpurun_out/${T}_tests.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
rm -rf gpurun_out/${T}_prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof -o run -- python3 bench.py --config prefilter --steps 8 --warmup 2 --no-cpu-baseline > gpurun_out/${T}_prof.log 2>&1 || { tail -5 gpurun_out/${T}_prof.log; exit 1; }
python3 - "$T" <<'PY'
import csv, glob, json, sys
t = sys.argv[1]
line = [l for l in open(f"gpurun_out/{t}_prof.log") if l.startswith("{")][-1]
d = json.loads(line)
print("value", d["value"], "ms", d["ms_per_step"], "phases", d["phase_ms_per_cloud"], "passes", d["propagation_passes"],
      "knn frac", d["roofline"]["frac"])
f = glob.glob(f"gpurun_out/{t}_prof/**/run_kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
print("kernel ms/cloud", sum(float(r["TotalDurationNs"]) for r in rows) / 10e6)
for r in rows[:12]:
    print(r["Name"][:60], r["Calls"], round(float(r["TotalDurationNs"]) / 10e3, 1), r["Percentage"])
PY
