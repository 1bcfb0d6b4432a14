# round 5: two-stage 16x16x8 reset (ts: 16 boards per stream wave, ts8: 8) -- parity gate, A/B vs gd
# (fix_lane reset, same gravity), and a kernel-trace of the 16x16 bench with ts
S16="--shape 16x16x8 --boards 262144"
FAST=1 bash tools/gpu_ab.sh r05t "libm3_ts.so $S16" "libm3_ts8.so $S16" "libm3_gd.so $S16" \
  "libm3_ts.so $S16" "libm3_ts8.so $S16" "libm3_gd.so $S16" "libm3_ts.so" "libm3_gd.so" &&
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT &&
M3_LIB=$PWD/element-crush-gym_amd/build/libm3_ts.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05t/kt16 -o kt -- \
  python3 bench.py $S16 --steps 40 --warmup 10 --no-cpu-baseline --check-boards 0 > gpurun_out/r05t/kt16.log 2>&1
