# final-tree confirmation: smoke, the whole -m gpu suite, the default bench line and the 16x16x8 one
set -o pipefail
O=gpurun_out/r04k; mkdir -p $O
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
{ timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 $O/gpu_tests.log; [ $rc -eq 0 ]; } && \
timeout -k 10 300 python3 bench.py > $O/bench.log 2>&1 && \
timeout -k 10 300 python3 bench.py --shape 16x16x8 --boards 262144 --steps 40 --warmup 10 > $O/bench16.log 2>&1 && \
python3 -c "
import json
for f in ['$O/bench.log', '$O/bench16.log']:
    d = json.loads(open(f).read().strip().splitlines()[-1]); r = d['roofline']
    print(f, '%.4g' % d['value'], d['unit'], '%.3f ms/step' % d['ms_per_step'], 'bound', r['bound'], 'frac %.3f' % r['frac'], 'oracle_match', d['parity']['oracle_match'])"
