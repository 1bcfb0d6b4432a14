# A/B throughput check: bench.py with each library in turn, twice (M3_LIB selects the build).
# usage: bash tools/ab_bench.sh <tag> libA.so libB.so ...  (paths relative to element-crush-gym_amd/build)
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
for r in 1 2; do
  for L in "$@"; do
    M3_LIB=$PWD/element-crush-gym_amd/build/$L timeout -k 10 300 python3 bench.py --steps 60 --warmup 10 --no-cpu-baseline > $OUT/$L.$r.log 2>&1 || exit 1
    python3 -c "import json;d=json.loads(open('$OUT/$L.$r.log').read().strip().splitlines()[-1]);print('$L run $r: %.4g env-steps/s  %.3f ms/step  kernel %.3f ms'%(d['value'],d['ms_per_step'],d['roofline']['avg_kernel_ms']))"
  done
done
