# Round 2: FullMT twist unroll + bulk tile draws (default), LDS-resident reset state (variant lds): tests + A/B.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r02j}
mkdir -p $OUT
B=$PWD/element-crush-gym_amd/build
[ -n "$SKIP_ALL" ] || timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
M3_LIB=$B/libm3_lds.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_mcts.py -x -v --timeout 120 --timeout-method thread > $OUT/lds.tests.log 2>&1 || { tail -30 $OUT/lds.tests.log; exit 1; }
echo "lds: $(tail -1 $OUT/lds.tests.log)"
S="--shape 16x16x8 --boards 262144"
bash tools/gpu_ab.sh ${1:-r02j}/ab "libm3_xbase.so $S" "libm3.so $S" "libm3_lds.so $S" "libm3_xbase.so $S" "libm3.so $S" "libm3_lds.so $S" "libm3_xbase.so" "libm3.so" "libm3_lds.so"
