# 16x16x8 resets: chain pass first, only the resets past the first MT block on FullMT (libm3_r16c.so)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04n; mkdir -p $O
M3_LIB=$PWD/element-crush-gym_amd/build/libm3_r16c.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_env.py tests/test_gpu_checkpoint.py tests/test_gpu_bench.py -x -q --timeout 300 --timeout-method thread > $O/tests_r16c.log 2>&1
rc=$?; echo "r16c pytest rc=$rc"; tail -2 $O/tests_r16c.log; [ $rc -eq 0 ] || exit 1
for round in 1 2; do
  for L in libm3.so libm3_r16c.so; do
    M3_LIB=$PWD/element-crush-gym_amd/build/$L timeout -k 10 300 python3 bench.py --shape 16x16x8 --boards 262144 --steps 40 --warmup 10 --no-cpu-baseline --check-boards 64 > $O/b16_${L}_$round.log 2>&1 || exit 1
  done
done
for f in $O/b*.log; do python3 -c "import json;d=json.loads(open('$f').read().strip().splitlines()[-1]);print('$f'.split('/')[-1], '%.4g env-steps/s'%d['value'], '%.3f ms/step'%d['ms_per_step'], 'oracle_match', d['parity'].get('oracle_match'), d['path_stats'])"; done
