set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tests_r06b.log 2>&1 || { tail -40 gpurun_out/tests_r06b.log; exit 1; }
tail -2 gpurun_out/tests_r06b.log
bash tools/kstat_ab.sh tree cur heads8 heads2 deal tree cur heads8 || exit 1
STEPS=3 bash tools/lib_ab.sh 2 $PWD/build_ab/lib_tree.so $PWD/build_ab/lib_heads8.so
