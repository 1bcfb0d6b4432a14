# Round 2: full -m gpu suite on libm3.so, negative control of the in-flight gather test, cascade-limit A/B (9x9, 16x16).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r02c}
mkdir -p $OUT
B=element-crush-gym_amd/build
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
# negative control: without the gather wait the in-flight test must fail on its assertion
M3_LIB=$PWD/$B/libm3_nowait.so timeout -k 10 300 python -u -m pytest tests/test_gpu_dist.py -v -k async_double --timeout 120 --timeout-method thread > $OUT/nowait.log 2>&1
echo "nowait rc=$? (1 = the test caught the missing wait)"; grep -E "^E .*words differ" $OUT/nowait.log | head -3
for L in libm3.so libm3_limoff.so libm3_lim1.so libm3_lim3.so; do
  M3_LIB=$PWD/$B/$L timeout -k 10 200 python3 bench.py --steps 40 --warmup 10 --no-cpu-baseline > $OUT/$L.9.log 2>&1 || exit 1
  M3_LIB=$PWD/$B/$L timeout -k 10 200 python3 bench.py --shape 16x16x8 --boards 262144 --steps 30 --warmup 10 --no-cpu-baseline > $OUT/$L.16.log 2>&1 || exit 1
  for s in 9 16; do
    python3 -c "import json;d=json.loads(open('$OUT/$L.$s.log').read().strip().splitlines()[-1]);print('$L $s: %.4g env-steps/s  %.3f ms/step  kernel %.3f ms'%(d['value'],d['ms_per_step'],d['roofline']['avg_kernel_ms']), d['path_stats'])"
  done
done
