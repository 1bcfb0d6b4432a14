# One GPU pass over the current tree: the -m gpu suite (gate), then the bench at both shapes for
# libm3.so and each library variant given, in two alternating rounds (same box, so the variants
# compare). Every bench line replays 64 timed boards through the oracle after its clock stops,
# except diagnostics whose name contains "nopf" (no prefetched episodes: not bit-exact by design).
# usage: bash tools/gpu_check.sh <tag> [variant.so ...]      (SKIP_TESTS=1 to skip the suite)
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-dev}; shift
O=gpurun_out/$TAG; mkdir -p $O
S16="--shape 16x16x8 --boards 262144"
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 $O/gpu_tests.log
  [ $rc -eq 0 ] || exit 1
fi
for round in 1 2; do
  for L in libm3.so "$@"; do
    CHK=64; case $L in *nopf*) CHK=0;; esac
    export M3_LIB=$PWD/element-crush-gym_amd/build/$L
    timeout -k 10 300 python3 bench.py --steps 40 --warmup 10 --no-cpu-baseline --check-boards $CHK > $O/b9_${L}_$round.log 2>&1 || exit 1
    timeout -k 10 300 python3 bench.py $S16 --steps 40 --warmup 10 --no-cpu-baseline --check-boards $CHK > $O/b16_${L}_$round.log 2>&1 || exit 1
  done
done
unset M3_LIB
for f in $O/b*.log; do python3 -c "import json;d=json.loads(open('$f').read().strip().splitlines()[-1]);r=d['roofline'];r=r.get('hbm',r);print('$f', '%.4g env-steps/s'%d['value'], '%.3f ms/step'%d['ms_per_step'], 'kernel %.3f ms'%r['avg_kernel_ms'], 'oracle_match', d['parity'].get('oracle_match'), d['path_stats'])"; done
