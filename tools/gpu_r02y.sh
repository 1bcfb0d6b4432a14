set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r02y
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
for L in libm3.so libm3_prev.so libm3.so libm3_prev.so; do
  M3_LIB=$PWD/element-crush-gym_amd/build/$L timeout -k 10 300 python3 bench.py --rollouts --steps 5 --warmup 1 --no-cpu-baseline > $OUT/ro_$L.log 2>&1 || exit 1
  python3 -c "import json;d=json.loads(open('$OUT/ro_$L.log').read().strip().splitlines()[-1]);print('$L rollouts/s %.4g  env-steps/s %.4g'%(d['rollouts_per_s'],d['env_steps_per_s']))"
done
bash tools/gpu_ab.sh r02y_ab "libm3.so" "libm3_prev.so"
