#!/bin/bash
# GPU side: library-build A/B with per-kernel averages: KERN=regex bash tools/lib_ab_prof.sh a.so b.so ...
# per build: the GPU test suite (TESTS=0 skips it), the C2 bench under rocprofv3 --kernel-trace
# --stats (kernels matching KERN), then the plain C2 bench.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
KERN=${KERN:-k_icp}
for lib in "$@"; do
  tag=$(basename $lib .so)
  export AICP_HIP_LIB=$PWD/$lib
  if [ "${TESTS:-1}" = 1 ]; then
    timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/lab_t_$tag.log 2>&1 || { tail -30 gpurun_out/lab_t_$tag.log; exit 1; }
    echo "$tag tests: $(tail -1 gpurun_out/lab_t_$tag.log)"
  fi
  rm -rf gpurun_out/lab_p_$tag
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/lab_p_$tag -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/lab_pb_$tag.log 2>&1 || { tail -20 gpurun_out/lab_pb_$tag.log; exit 1; }
  python3 - "$tag" "$KERN" <<'PY'
import csv, glob, re, sys
tag, kern = sys.argv[1], sys.argv[2]
f = glob.glob(f"gpurun_out/lab_p_{tag}/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if re.search(kern, r["Name"]):
        print(tag, r["Name"].split("(")[0][:48], "calls", r["Calls"], "avg_us", round(float(r["AverageNs"]) / 1e3, 1))
PY
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/lab_b_$tag.log 2>&1 || { tail -20 gpurun_out/lab_b_$tag.log; exit 1; }
  python3 -c "import json;d=json.loads([l for l in open('gpurun_out/lab_b_$tag.log') if l.startswith('{')][-1]);print('$tag C2',d['value'],d['ms_per_step'],d['roofline']['avg_launch_us'],d['phase_ms_per_step'])"
done
