# Quick iteration: -m gpu parity suite, phase breakdown, bench without CPU baseline.
# usage: bash tools/gpu_quick.sh <tag>
set -o pipefail
TAG=${1:-dev}
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
{ timeout -k 10 900 python -m pytest tests -m gpu -x -q > $OUT/gpu_tests.log 2>&1; rc=$?; echo "pytest rc=$rc"; [ $rc -le 1 ]; } && \
timeout -k 10 300 python3 tools/phase_prof.py --shards 1 > $OUT/phase_s1.log 2>&1 && \
timeout -k 10 300 python3 bench.py --steps 60 --warmup 10 --no-cpu-baseline > $OUT/bench.log 2>&1
rc=$?
tail -2 $OUT/gpu_tests.log
grep -v '^{' $OUT/phase_s1.log
python3 -c "import json;d=json.loads(open('$OUT/bench.log').read().strip().splitlines()[-1]);print('value %.4g ms/step %.3f kernel_ms %.3f'%(d['value'],d['ms_per_step'],d['roofline']['avg_kernel_ms']), d.get('path_stats'))"
exit $rc
