set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r02w
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
M3_LIB=$PWD/element-crush-gym_amd/build/libm3_cl2.so timeout -k 10 600 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests_cl2.log 2>&1 || { tail -40 $OUT/gpu_tests_cl2.log; exit 1; }
tail -1 $OUT/gpu_tests_cl2.log
bash tools/gpu_ab.sh r02w_ab "libm3.so" "libm3_cl1.so" "libm3_cl2.so" "libm3_cl3.so" "libm3.so" "libm3_cl1.so" "libm3_cl2.so" "libm3_cl3.so"
