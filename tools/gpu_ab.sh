# A/B bench of library variants x bench options (9x9x6 headline config).
# usage: bash tools/gpu_ab.sh <tag> "<lib> <bench args>" ...   (lib relative to element-crush-gym_amd/build)
set -o pipefail
export TMPDIR=/tmp
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
i=0
for spec in "$@"; do
  set -- $spec
  L=$1; shift
  i=$((i+1))
  M3_LIB=$PWD/element-crush-gym_amd/build/$L timeout -k 10 200 python3 bench.py --steps 40 --warmup 10 --no-cpu-baseline "$@" > $OUT/$i.log 2>&1 || { tail -5 $OUT/$i.log; exit 1; }
  python3 -c "import json;d=json.loads(open('$OUT/$i.log').read().strip().splitlines()[-1]);print('$L $*: %.4g env-steps/s  %.3f ms/step  kernel %.3f ms'%(d['value'],d['ms_per_step'],d['roofline']['avg_kernel_ms']))"
done
