# Round 2: -m gpu suite on libm3.so (wavefront step), then A/B of the step variants (9x9 and 16x16).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r02g}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
bash tools/gpu_ab.sh ${1:-r02g}_ab "libm3.so" "libm3_mega.so" "libm3_wps5.so" "libm3_wps3.so" "libm3.so --shards 1" "libm3.so --shards 3" "libm3.so --shape 16x16x8 --boards 262144" "libm3_mega.so --shape 16x16x8 --boards 262144"
