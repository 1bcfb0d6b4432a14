# Round 2: GPU suite; 16x16 + 9x9 bench.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r02m}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
S="--shape 16x16x8 --boards 262144"
bash tools/gpu_ab.sh ${1:-r02m}/ab "libm3.so $S" "libm3.so"
