# One parametrised GPU pass (replaces round 5's one-shot gpu_r05*.sh scripts).
# usage: bash tools/gpu_run.sh <tag> <step> [<step> ...]
#   smoke                 __graft_entry__.smoke()
#   tests[:<pytest args>] the -m gpu suite (or the given files / -k filter), e.g. "tests:tests/test_gpu_parity.py -k prefetched"
#   bench9 | bench16      bench.py at C3 / C4 (driver command for C3: defaults)
#   ab:<lib>[:<args>]     parity gate (tools/gpu_ab.sh) + timing of a library variant in build/
# Every GPU step runs under its own time limit; the first failing step ends the call.
set -o pipefail
export TMPDIR=/tmp
TAG=$1; shift
O=gpurun_out/$TAG; mkdir -p $O
n=0
for step in "$@"; do
  n=$((n+1))
  case $step in
    smoke) timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 ;;
    tests) timeout -k 10 1100 python3 -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1 ;;
    tests:*) timeout -k 10 900 python3 -u -m pytest ${step#tests:} -m gpu -x -v --timeout 400 --timeout-method thread > $O/tests_$n.log 2>&1 ;;
    bench9) timeout -k 10 300 python3 bench.py > $O/bench9_$n.log 2>&1 ;;
    bench16) timeout -k 10 300 python3 bench.py --shape 16x16x8 --boards 262144 --steps 40 --warmup 10 > $O/bench16_$n.log 2>&1 ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
  rc=$?
  echo "step $n ($step): rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
for f in $O/bench*.log; do
  [ -f "$f" ] && python3 -c "import json;d=json.loads([l for l in open('$f').read().splitlines() if l.startswith('{')][-1]);print('$f %.4g env-steps/s %.3f ms frac %.3f oracle %s'%(d['value'],d['ms_per_step'],d['roofline']['frac'],d['parity']['oracle_match']))"
done
exit 0
