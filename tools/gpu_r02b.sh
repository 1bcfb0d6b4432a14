# Round 2: gather/upload tests, the negative control for the in-flight gather test, cascade/legal A/B timings.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r02b
mkdir -p $OUT
B=element-crush-gym_amd/build
timeout -k 10 300 python -u -m pytest tests/test_gpu_dist.py -x -v --timeout 120 --timeout-method thread > $OUT/dist.log 2>&1 || exit 1
# negative control: without the gather wait the in-flight test must fail
M3_LIB=$PWD/$B/libm3_nowait.so timeout -k 10 300 python -u -m pytest tests/test_gpu_dist.py -v -k async_double --timeout 120 --timeout-method thread > $OUT/nowait.log 2>&1
echo "nowait rc=$?"
for L in libm3.so libm3_it1.so libm3_it2.so libm3_it3.so libm3_nolegal.so; do
  M3_LIB=$PWD/$B/$L timeout -k 10 200 python3 bench.py --steps 40 --warmup 10 --no-cpu-baseline > $OUT/$L.log 2>&1 || exit 1
  python3 -c "import json;d=json.loads(open('$OUT/$L.log').read().strip().splitlines()[-1]);print('$L: %.4g env-steps/s  %.3f ms/step  kernel %.3f ms'%(d['value'],d['ms_per_step'],d['roofline']['avg_kernel_ms']))"
done
