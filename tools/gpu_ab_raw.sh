# Timing-only A/B of library variants (NO parity gate: for measurement experiments that are not
# bit-exact by design, e.g. a cost-free refill stand-in). usage: bash tools/gpu_ab_raw.sh <tag> <lib>...
# (libs relative to element-crush-gym_amd/build); 9x9x6 C3 and 16x16x8 C4, two alternating rounds.
set -o pipefail
export TMPDIR=/tmp
TAG=$1; shift
O=gpurun_out/$TAG; mkdir -p $O
for i in 1 2; do
for L in "$@"; do
  export M3_LIB=$PWD/element-crush-gym_amd/build/$L
  timeout -k 10 200 python3 bench.py --steps 40 --warmup 10 --no-cpu-baseline --check-boards 0 > $O/9_${L}_$i.log 2>&1 || exit 1
  timeout -k 10 200 python3 bench.py --shape 16x16x8 --boards 262144 --steps 40 --warmup 10 --no-cpu-baseline --check-boards 0 > $O/16_${L}_$i.log 2>&1 || exit 1
done; done
for f in $O/*.log; do python3 -c "import json,sys;d=json.loads(open('$f').read().strip().splitlines()[-1]);print('$f', '%.4g'%d['value'], '%.3f'%d['ms_per_step'], '%.3f'%d['roofline']['hbm']['avg_kernel_ms'])"; done
