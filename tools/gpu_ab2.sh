# -m gpu suite on the default build, then bench A/B (9x9 and 16x16) of the given libs.
# usage: bash tools/gpu_ab2.sh <tag> libA.so libB.so ...
set -o pipefail
TAG=$1; shift
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit 1
for L in "$@"; do
  M3_LIB=$PWD/element-crush-gym_amd/build/$L timeout -k 10 300 python3 bench.py --steps 60 --warmup 10 --no-cpu-baseline > $OUT/$L.9.log 2>&1 || exit 1
  M3_LIB=$PWD/element-crush-gym_amd/build/$L timeout -k 10 300 python3 bench.py --shape 16x16x8 --boards 262144 --steps 40 --warmup 10 --no-cpu-baseline > $OUT/$L.16.log 2>&1 || exit 1
done
