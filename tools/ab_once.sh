set -o pipefail
O=gpurun_out/ab_defer; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1; echo "tests rc=$?"; tail -3 $O/gpu_tests.log
bash tools/gpu_ab.sh ab_defer "libm3_defer.so" "libm3_cfix.so" "libm3_defer.so" "libm3_cfix.so" "libm3_defer.so" "libm3_cfix.so" && \
M3_LIB=$PWD/element-crush-gym_amd/build/libm3_defer.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt9 -o kt --output-format csv -- python3 bench.py --steps 60 --warmup 10 --no-cpu-baseline > $O/kt9.log 2>&1
