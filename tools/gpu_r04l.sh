# staggered shards A/B (libm3_stagger.so: shard s starts its step kernel after shard s-1's)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04l; mkdir -p $O
for round in 1 2; do
  for cfg in "libm3.so 2" "libm3_stagger.so 2" "libm3_stagger.so 3" "libm3_stagger.so 4" "libm3.so 3"; do
    set -- $cfg
    M3_LIB=$PWD/element-crush-gym_amd/build/$1 timeout -k 10 300 python3 bench.py --steps 40 --warmup 10 --no-cpu-baseline --check-boards 64 --shards $2 > $O/b9_$1_s$2_$round.log 2>&1 || exit 1
  done
  for L in libm3.so libm3_stagger.so; do
    M3_LIB=$PWD/element-crush-gym_amd/build/$L timeout -k 10 300 python3 bench.py --shape 16x16x8 --boards 262144 --steps 40 --warmup 10 --no-cpu-baseline --check-boards 64 > $O/b16_${L}_$round.log 2>&1 || exit 1
  done
done
for f in $O/b*.log; do python3 -c "import json;d=json.loads(open('$f').read().strip().splitlines()[-1]);print('$f'.split('/')[-1], '%.4g env-steps/s'%d['value'], '%.3f ms/step'%d['ms_per_step'], 'oracle_match', d['parity'].get('oracle_match'))"; done
