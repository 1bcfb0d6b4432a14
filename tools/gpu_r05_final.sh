# round 5 evidence: tools/gpu_final.sh r05 (smoke, -m gpu suite, bench lines, kernel traces, PMC passes),
# then the lane-interference regression test against the pre-fix library (expected to fail there)
set -o pipefail
export TMPDIR=/tmp
bash tools/gpu_final.sh r05 || exit 1
M3_LIB=$PWD/element-crush-gym_amd/build/libm3_pre.so timeout -k 10 400 python3 -u -m pytest tests/test_gpu_shapes.py -m gpu -v \
  -k frame_rollouts --timeout 300 --timeout-method thread > gpurun_out/r05/pre_regression.log 2>&1
echo "pre-fix library: pytest rc=$?"
grep -E "PASSED|FAILED|passed|failed" gpurun_out/r05/pre_regression.log | tail -12
exit 0
