# Round 2: inline wave reset of overflowing resets in k_init (default) vs k_init_fix_wave (noinl): tests + A/B.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r02o}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
bash tools/gpu_ab.sh ${1:-r02o}/ab libm3.so libm3_noinl.so libm3.so libm3_noinl.so libm3.so libm3_noinl.so
