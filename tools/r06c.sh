set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tests_r06c.log 2>&1 || { tail -40 gpurun_out/tests_r06c.log; exit 1; }
tail -2 gpurun_out/tests_r06c.log
bash tools/kstat_ab.sh h8 heads16 tree h8 heads16 || exit 1
STEPS=3 bash tools/lib_ab.sh 2 $PWD/build_ab/lib_tree.so $PWD/build_ab/lib_heads16.so || exit 1
CFG=c5 STEPS=2 bash tools/lib_ab.sh 2 $PWD/build_ab/lib_tree.so $PWD/build_ab/lib_heads16.so
