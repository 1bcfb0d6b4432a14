# write-through work-stealing continuation (libm3_fusedwt.so): parity suite parts against it, then the A/B
set -o pipefail
mkdir -p gpurun_out/r04j
M3_LIB=$PWD/element-crush-gym_amd/build/libm3_fusedwt.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bench.py tests/test_gpu_env.py tests/test_gpu_checkpoint.py tests/test_gpu_dist.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r04j/tests_fusedwt.log 2>&1
rc=$?; echo "fusedwt pytest rc=$rc"; tail -3 gpurun_out/r04j/tests_fusedwt.log; [ $rc -eq 0 ] || exit 1
SKIP_TESTS=1 bash tools/gpu_check.sh r04j libm3_fusedwt.so
