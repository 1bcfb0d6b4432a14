set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r02s
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
bash tools/gpu_ab.sh r02s_ab "libm3.so" "libm3_prev.so" "libm3.so" "libm3_prev.so" "libm3.so --shape 16x16x8 --boards 262144"
