# Round evidence on the shipped library: smoke, the whole -m gpu suite, both bench shapes with their
# rocprofv3 kernel trace and PMC passes (tools/gpu_profile.sh: the driver's own command line), the
# rollout lines and the batch-1 latencies.
# usage: [SKIP_TESTS=1] bash tools/gpu_final.sh <tag>
#   then: python3 tools/collect_profiles.py gpurun_out/<tag>/s9 <round>; ... s16 <round>
set -o pipefail
TAG=${1:-dev}
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
S16="--shape 16x16x8 --boards 262144"
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && echo "smoke ok" && \
{ [ -n "$SKIP_TESTS" ] || { timeout -k 10 1100 python3 -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -1 $O/gpu_tests.log; [ $rc -eq 0 ]; }; } && \
bash tools/gpu_profile.sh $TAG 9 && bash tools/gpu_profile.sh $TAG 16 && \
timeout -k 10 300 python3 bench.py --rollouts --steps 5 --warmup 1 > $O/rollouts9.log 2>&1 && \
timeout -k 10 300 python3 bench.py --rollouts $S16 --steps 3 --warmup 1 > $O/rollouts16.log 2>&1 && \
timeout -k 10 300 python3 tools/latency.py --out $O/latency.json > $O/latency.log 2>&1 && \
for f in s9/bench s16/bench; do python3 -c "import json;d=json.loads([l for l in open('$O/$f.log').read().splitlines() if l.startswith('{')][-1]);r=d['roofline'];print('$f %.4g env-steps/s %.3f ms/step valu frac %.3f simt %.3f oracle %s'%(d['value'],d['ms_per_step'],r['frac'],r.get('simt',0),d['parity']['oracle_match']))"; done
