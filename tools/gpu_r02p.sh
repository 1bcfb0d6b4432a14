set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r02p
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
bash tools/gpu_ab.sh r02p_ab "libm3.so" "libm3_c3.so" "libm3_w5.so" "libm3_w3.so" "libm3.so" "libm3_c3.so" "libm3.so --shape 16x16x8 --boards 262144"
