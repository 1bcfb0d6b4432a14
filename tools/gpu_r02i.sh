# Round 2: 16x16 resets on the wave-cooperative pass (variants w16a grid 64, w16b grid 1024): parity + A/B.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r02i}
mkdir -p $OUT
B=$PWD/element-crush-gym_amd/build
for L in libm3_xw16a.so libm3_xw16b.so; do
  M3_LIB=$B/$L timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k "16x16 or c4" > $OUT/$L.tests.log 2>&1 || { tail -30 $OUT/$L.tests.log; exit 1; }
  echo "$L: $(tail -1 $OUT/$L.tests.log)"
done
bash tools/gpu_ab.sh ${1:-r02i}/ab16 "libm3.so --shape 16x16x8 --boards 262144" "libm3_xw16a.so --shape 16x16x8 --boards 262144" "libm3_xw16b.so --shape 16x16x8 --boards 262144" "libm3.so --shape 16x16x8 --boards 262144" "libm3_xw16b.so --shape 16x16x8 --boards 262144" "libm3.so" "libm3_xw16b.so"
