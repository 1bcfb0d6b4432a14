# round 5, final library (after the last source change): smoke, the whole -m gpu suite, both bench lines
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05f2; mkdir -p $O
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && echo smoke ok &&
{ timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 $O/gpu_tests.log; [ $rc -eq 0 ]; } &&
timeout -k 10 300 python3 bench.py > $O/bench9.log 2>&1 &&
timeout -k 10 300 python3 bench.py --shape 16x16x8 --boards 262144 --steps 40 --warmup 10 > $O/bench16.log 2>&1 &&
timeout -k 10 300 python3 tools/latency.py --out $O/latency.json > $O/latency.log 2>&1 &&
for f in bench9 bench16; do python3 -c "import json;d=json.loads([l for l in open('$O/$f.log').read().splitlines() if l.startswith('{')][-1]);print('$f %.4g env-steps/s %.3f ms frac %.3f oracle %s'%(d['value'],d['ms_per_step'],d['roofline']['frac'],d['parity']['oracle_match']))"; done
