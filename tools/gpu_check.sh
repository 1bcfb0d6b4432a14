# One GPU pass over the current tree: the -m gpu suite (gate), then the bench at both shapes
# and optional library variants (no parity gate: diagnostics such as libm3_nopf.so are not
# bit-exact by construction, so their lines run with --check-boards 0).
# usage: bash tools/gpu_check.sh <tag> [variant.so ...]
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-dev}; shift
O=gpurun_out/$TAG; mkdir -p $O
S16="--shape 16x16x8 --boards 262144"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/gpu_tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python3 bench.py --steps 40 --warmup 10 --no-cpu-baseline > $O/b9.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py $S16 --steps 40 --warmup 10 --no-cpu-baseline > $O/b16.log 2>&1 || exit 1
for L in "$@"; do
  M3_LIB=$PWD/element-crush-gym_amd/build/$L timeout -k 10 300 python3 bench.py --steps 40 --warmup 10 --no-cpu-baseline --check-boards 0 > $O/b9_$L.log 2>&1 || exit 1
  M3_LIB=$PWD/element-crush-gym_amd/build/$L timeout -k 10 300 python3 bench.py $S16 --steps 40 --warmup 10 --no-cpu-baseline --check-boards 0 > $O/b16_$L.log 2>&1 || exit 1
done
for f in $O/b*.log; do python3 -c "import json;d=json.loads(open('$f').read().strip().splitlines()[-1]);r=d['roofline'];print('$f', '%.4g env-steps/s'%d['value'], '%.3f ms/step'%d['ms_per_step'], 'kernel %.3f ms'%r.get('avg_kernel_ms', r.get('hbm',{}).get('avg_kernel_ms',0)), 'oracle_match', d['parity'].get('oracle_match'), d['path_stats'])"; done
