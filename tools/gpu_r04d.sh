# A/B: continuation kernel (grid vs persistent) and 16x16 resets (FullMT vs ChainMT2), against the
# round-3 library and its no-prefetch diagnostic; then one kernel trace per variant of interest.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04d; mkdir -p $O
SKIP_TESTS=1 bash tools/gpu_check.sh r04d libm3_pc.so libm3_c2.so libm3_r03.so libm3_nopf.so || exit 1
for L in libm3.so libm3_pc.so libm3_r03.so; do
  M3_LIB=$PWD/element-crush-gym_amd/build/$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt9_$L -o kt --output-format csv -- python3 bench.py --steps 40 --warmup 10 --no-cpu-baseline --check-boards 0 > $O/kt9_$L.log 2>&1 || exit 1
done
for L in libm3.so libm3_c2.so libm3_nopf.so; do
  M3_LIB=$PWD/element-crush-gym_amd/build/$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt16_$L -o kt --output-format csv -- python3 bench.py --shape 16x16x8 --boards 262144 --steps 40 --warmup 10 --no-cpu-baseline --check-boards 0 > $O/kt16_$L.log 2>&1 || exit 1
done
for f in $O/kt*/kt_kernel_stats.csv; do echo "== $f"; cut -d, -f1-4 $f | sed 's/(anonymous namespace):://; s/m3::Cfg<\([0-9, ]*\)>/\1/' | head -8; done
