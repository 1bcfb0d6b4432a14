# round 5 final tree, part 1: smoke, the whole -m gpu suite, then the lane-interference regression
# test against the pre-fix library (expected to FAIL there)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05; mkdir -p $O
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && echo smoke ok &&
{ timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 $O/gpu_tests.log; [ $rc -eq 0 ]; } || exit 1
M3_LIB=$PWD/element-crush-gym_amd/build/libm3_pre.so timeout -k 10 400 python3 -u -m pytest tests/test_gpu_shapes.py -m gpu -v \
  -k frame_rollouts --timeout 300 --timeout-method thread > $O/pre_regression.log 2>&1
echo "pre-fix library: pytest rc=$?"
grep -E "PASSED|FAILED|passed|failed" $O/pre_regression.log | tail -12
exit 0
