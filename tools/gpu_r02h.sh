set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r02hc
mkdir -p $OUT
M3_LIB=$PWD/element-crush-gym_amd/build/libm3_h9.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dist.py -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests_h9.log 2>&1 || { tail -40 $OUT/gpu_tests_h9.log; exit 1; }
tail -1 $OUT/gpu_tests_h9.log
bash tools/gpu_ab.sh r02hc_ab "libm3.so" "libm3_h7.so" "libm3_h9.so" "libm3_h12.so" "libm3.so" "libm3_h7.so" "libm3_h9.so" "libm3_h12.so"
