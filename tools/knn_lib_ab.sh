#!/bin/bash
# GPU side: k-NN kernel A/B over library builds: bash tools/knn_lib_ab.sh a.so b.so ...
# per build: the kNN / normals / pre-filter parity tests, the C2 bench under rocprofv3 (kNN-20
# launch average) and the pre-filter bench (kNN-30 launch average from its roofline object).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for lib in "$@"; do
  tag=$(basename $lib .so)
  export AICP_HIP_LIB=$PWD/$lib
  timeout -k 10 300 python -u -m pytest tests -x -q -m gpu -k "knn or normal or prefilter or golden" --timeout 120 --timeout-method thread > gpurun_out/kab_t_$tag.log 2>&1 || { tail -30 gpurun_out/kab_t_$tag.log; exit 1; }
  echo "$tag tests: $(tail -1 gpurun_out/kab_t_$tag.log)"
  rm -rf gpurun_out/kab_p_$tag
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kab_p_$tag -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/kab_b_$tag.log 2>&1 || { tail -20 gpurun_out/kab_b_$tag.log; exit 1; }
  python3 - "$tag" <<'PY'
import csv, glob, json, sys
tag = sys.argv[1]
f = glob.glob(f"gpurun_out/kab_p_{tag}/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "k_knn_ids" in r["Name"] or "k_icp_nn" in r["Name"] or "k_normals_from" in r["Name"]:
        print(tag, r["Name"].split("(")[0], "calls", r["Calls"], "avg_us", round(float(r["AverageNs"]) / 1e3, 1))
d = json.loads([l for l in open(f"gpurun_out/kab_b_{tag}.log") if l.startswith("{")][-1])
print(tag, "C2 (under rocprof)", d["value"], d["phase_ms_per_step"])
PY
  timeout -k 10 300 python bench.py --config prefilter --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/kab_pf_$tag.log 2>&1 || { tail -20 gpurun_out/kab_pf_$tag.log; exit 1; }
  python3 -c "import json;d=json.loads([l for l in open('gpurun_out/kab_pf_$tag.log') if l.startswith('{')][-1]);print('$tag prefilter',d['value'],d['phase_ms_per_cloud'],d['roofline']['avg_launch_us'])"
done
