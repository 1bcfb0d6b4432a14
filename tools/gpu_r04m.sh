# flag-only variants of the 9x9 / 16x16 step: waves per SIMD of k_env_step / k_env_cont, -O2
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04m; mkdir -p $O
for round in 1 2; do
  for L in libm3.so libm3_wps5.so libm3_cwps2.so libm3_cwps8.so libm3_o2.so; do
    M3_LIB=$PWD/element-crush-gym_amd/build/$L timeout -k 10 300 python3 bench.py --steps 40 --warmup 10 --no-cpu-baseline --check-boards 64 > $O/b9_${L}_$round.log 2>&1 || exit 1
  done
  for L in libm3.so libm3_o2.so; do
    M3_LIB=$PWD/element-crush-gym_amd/build/$L timeout -k 10 300 python3 bench.py --shape 16x16x8 --boards 262144 --steps 40 --warmup 10 --no-cpu-baseline --check-boards 64 > $O/b16_${L}_$round.log 2>&1 || exit 1
  done
done
for f in $O/b*.log; do python3 -c "import json;d=json.loads(open('$f').read().strip().splitlines()[-1]);print('$f'.split('/')[-1], '%.4g env-steps/s'%d['value'], '%.3f ms/step'%d['ms_per_step'], 'oracle_match', d['parity'].get('oracle_match'))"; done
