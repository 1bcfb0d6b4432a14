set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r02j
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
bash tools/gpu_ab.sh r02j_ab "libm3.so" "libm3_mega.so" "libm3_wps5.so" && \
bash tools/gpu_pmc.sh $OUT/wf libm3.so && bash tools/gpu_pmc.sh $OUT/mega libm3_mega.so
